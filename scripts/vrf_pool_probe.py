"""Host VRF outputs on the bench box: per-output cost and the wall time of one round's batch (100
outputs) on the native pool, cold (workers asleep) and back to back.

    python scripts/vrf_pool_probe.py
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd.native import rt  # noqa: E402


def main():
    R = rt()
    seeds = [bytes([i]) * 32 for i in range(100)]
    out = {"cpus_affinity": len(os.sched_getaffinity(0))}
    try:
        out["cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    for thr in (1, 8, 15, 16):
        ts = []
        for k in range(6):
            time.sleep(0.005)   # workers go back to sleep: the engine's case (one batch per round)
            t = time.perf_counter()
            j = R.vrf_prove_batch_async(seeds, bytes([k]) * 32, thr, None, True)
            j.betas()
            ts.append(time.perf_counter() - t)
            del j
        out[f"wall_us_100_outputs_{thr}thr"] = round(float(np.median(ts[1:])) * 1e6, 1)
    out["us_per_output_1thr"] = out["wall_us_100_outputs_1thr"] / 100
    print(json.dumps(out))


if __name__ == "__main__":
    main()
