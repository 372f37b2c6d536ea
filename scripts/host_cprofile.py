"""Host-side hot spots of the round loop: cProfile over a bench run on the GPU, summarised (tottime and
cumtime top lists) -- the round is host-bound, so this is where its time goes.

    python scripts/host_cprofile.py --steps 200 --warmup 10 > gpurun_out/cprof.txt
"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench

    argv = ["bench.py"] + sys.argv[1:]
    sys.argv = argv
    pr = cProfile.Profile()
    pr.enable()
    try:
        bench.main()
    finally:
        pr.disable()
    for key in ("tottime", "cumtime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        print(f"==== by {key}\n" + s.getvalue())


if __name__ == "__main__":
    main()
