"""Probe host/GPU interplay inside engine rounds: VRF job timings and isolated host timings."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd.parallel.comm import Comm  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402
from biscotti_amd.protocol import engine as E  # noqa: E402


def main():
    comm = Comm.init()
    torch.set_num_threads(min(4, torch.get_num_threads()))
    threads = int(os.environ.get("BSC_HOST_THREADS", "16"))
    eng = E.BiscottiEngine(RunConfig(num_nodes=100, seed=0, max_iterations=10**9, host_threads=threads), comm)
    R = eng.R
    jobs = []
    orig = R.vrf_prove_batch_async

    class Spy:
        def __getattr__(self, k):
            return getattr(R, k)

        def vrf_prove_batch_async(self, *a):
            j = orig(*a)
            jobs.append((len(a[0]), j))
            return j
    eng.R = Spy()
    for _ in range(3):
        eng.run_round()
    jobs.clear()
    walls = []
    for _ in range(10):
        r = eng.run_round()
        walls.append(r.wall)
    tim = [(n, j.timing_us()) for n, j in jobs]
    seeds = [os.urandom(32) for _ in range(100)]
    iso = []
    for _ in range(5):
        t = time.perf_counter()
        R.vrf_prove_batch(seeds, b"x" * 32, threads)
        iso.append((time.perf_counter() - t) * 1e6)
    iso_async = []
    for _ in range(5):
        t = time.perf_counter()
        R.vrf_prove_batch_async(seeds, b"x" * 32, threads).result()
        iso_async.append((time.perf_counter() - t) * 1e6)
    print(json.dumps({"threads": threads, "round_ms": [w * 1e3 for w in walls], "jobs": tim[:8],
                      "isolated_sync_us": iso, "isolated_async_us": iso_async,
                      "last_phases": r.phases}, indent=0))


if __name__ == "__main__":
    main()
