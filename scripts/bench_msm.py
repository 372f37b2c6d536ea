"""Micro-benchmark of the BN256 share/commitment MSM at the MNIST size (d = 7850).

python scripts/bench_msm.py [--rows 35] [--workers 94] [--scale 30000]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np
import torch

from biscotti_amd.native import rt
from biscotti_amd.ops import bn256 as B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=7850)
    ap.add_argument("--rows", type=int, default=35)
    ap.add_argument("--workers", type=int, default=94)
    ap.add_argument("--scale", type=int, default=30000, help="uniform coefficient range (--dist uniform)")
    ap.add_argument("--dist", default="real", choices=["real", "uniform"],
                    help="real: N(0, 1500^2) integers, the measured spread of quantised MNIST updates")
    ap.add_argument("--density", type=float, default=1.0,
                    help="fraction of nonzero coefficients (quantised updates after the first rounds: 0.1-0.25)")
    ap.add_argument("--b0", type=int, default=None)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lib", default=None, help="another build of libbiscotti_hip.so (same-box A/B of kernels)")
    a = ap.parse_args()
    if a.lib:
        import ctypes

        from biscotti_amd import native
        from biscotti_amd.ops import _abi

        lib = ctypes.CDLL(str(Path(a.lib).resolve()))
        _abi.declare(lib)
        native._hip = lib
    t0 = time.time()
    key = rt().CommitKey.generate(a.d, 2)
    t1 = time.time()
    eng = B.DeviceCommitEngine(key, 10, 21, b0=a.b0)
    torch.cuda.synchronize()
    t2 = time.time()
    rng = np.random.default_rng(0)
    if a.dist == "real":
        c = np.rint(rng.normal(0.0, 1500.0, size=(a.workers, a.d))).astype(np.int64)
    else:
        c = rng.integers(-a.scale, a.scale, size=(a.workers, a.d), dtype=np.int64)
    if a.density < 1.0:
        c = np.where(rng.random(c.shape) < a.density, c, 0)
    coeffs = torch.from_numpy(c).cuda()
    allrows = torch.arange(a.workers, dtype=torch.int32, device="cuda")
    rows = allrows[: a.rows].contiguous()
    res = {"lib": a.lib or "default", "d": a.d, "dist": a.dist, "density": a.density, "b0": eng.b0, "key_gen_s": t1 - t0, "table_build_s": t2 - t1,
           "table_gb": eng.table_bytes() / 1e9}
    for name, fn in [
        ("commit_rows_all_workers", lambda: eng.commit_rows(coeffs, allrows)),
        ("shares_approved", lambda: eng.shares(coeffs, rows)),
        ("shares_witness_only", lambda: eng.shares(coeffs, rows, commit_only=2)),
    ]:
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            s = time.time()
            fn()
            torch.cuda.synchronize()
            ts.append(time.time() - s)
        res[name + "_ms"] = 1e3 * float(np.median(ts))
    n_mults = a.rows * (a.d + (a.d // 10) * 21 * 9)
    res["shares_scalar_mults"] = n_mults
    res["shares_Gmult_per_s"] = n_mults / (res["shares_approved_ms"] / 1e3) / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
