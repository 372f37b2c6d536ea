"""Latency of one device ECVRF prover launch (kernels/vrf.hip) at round size (~200 proofs) and at one
workgroup (16 proofs), timed with HIP events; bit-exactness is tests/test_gpu_vrf.py's job."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd.ops.vrf import DeviceVrfProver  # noqa: E402


def main():
    prover = DeviceVrfProver("cuda")
    rng = np.random.default_rng(0)
    seeds = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(200)]
    out = {}
    for n in (16, 64, 200):
        ts = []
        for rep in range(6):
            alpha = [bytes(rng.integers(0, 256, 32, dtype=np.uint8))] * n
            prover._rows(seeds[:n])
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            prover.prove(seeds[:n], alpha)
            b.record()
            torch.cuda.synchronize()
            if rep:
                ts.append(a.elapsed_time(b))
        out[n] = {"ms_mean": float(np.mean(ts)), "ms_min": float(np.min(ts)), "ms_max": float(np.max(ts))}
    print(json.dumps({"vrf_prove_latency": out}))


if __name__ == "__main__":
    main()
