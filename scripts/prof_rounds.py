"""cProfile of steady-state headline rounds only (the engine built and warmed outside the profile): which Python
functions and which torch / native calls hold the round's host thread.

    python scripts/prof_rounds.py [--warm 30] [--rounds 200] [--emulate-world N] [-o out.txt]

--emulate-world N profiles rank 0 of an N-rank job (bench.py --emulate-world: the collectives filled locally).
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd.parallel.comm import Comm  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402
from biscotti_amd.protocol.engine import BiscottiEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--emulate-world", type=int, default=0)
    ap.add_argument("-o", "--out", default=None)
    a = ap.parse_args()
    comm = Comm.emulated(a.emulate_world) if a.emulate_world > 1 else Comm.init()
    torch.set_num_threads(1)
    eng = BiscottiEngine(RunConfig(num_nodes=100, seed=0, max_iterations=10**9, host_threads=14, lazy_eval=True), comm)
    for _ in range(a.warm):
        eng.run_round()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.rounds):
        eng.run_round()
    pr.disable()
    torch.cuda.synchronize()
    eng.drain()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(70)
    st.sort_stats("cumulative").print_stats(90)
    txt = s.getvalue()
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt[:6000])
    eng.close()


if __name__ == "__main__":
    main()
