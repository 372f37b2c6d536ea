"""Host-side profile of engine rounds (cProfile): where the Python thread spends a round, incl.
calls that block on the device (`tolist`, `item`, `synchronize`, pinned allocations).

    python scripts/host_profile.py [--rounds 30] [--top 45]
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
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    comm = Comm.init()
    torch.set_num_threads(min(4, torch.get_num_threads()))
    eng = BiscottiEngine(RunConfig(num_nodes=100, seed=0, max_iterations=10**9, host_threads=16, phase_sync=False),
                         comm)
    for _ in range(5):
        eng.run_round()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.rounds):
        eng.run_round()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(40)
    print(s.getvalue())
    eng.close()


if __name__ == "__main__":
    main()
