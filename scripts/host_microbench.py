"""Host-runtime microbenchmarks: VRF / Schnorr batch throughput vs thread count, CPU share."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from biscotti_amd.native import rt


def main():
    R = rt()
    info = {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        info["cpu.max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    seeds = [os.urandom(32) for _ in range(100)]
    h = os.urandom(32)
    res = {}
    for th in (1, 2, 4, 8, 16, 32):
        R.vrf_prove_batch(seeds, h, th)
        t = time.perf_counter()
        for _ in range(5):
            R.vrf_prove_batch(seeds, h, th)
        res[f"vrf100_t{th}_ms"] = (time.perf_counter() - t) / 5 * 1e3
    info["results"] = res
    print(json.dumps(info))


if __name__ == "__main__":
    main()
