"""Isolated latency of the aggregate audit kernel (k_chunk_check) at the MNIST shapes, by
coefficient magnitude (= number of window additions per lane), and of the commitment sums.

    python scripts/audit_microbench.py [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from biscotti_amd.native import rt  # noqa: E402
from biscotti_amd.ops import bn256 as B  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--d", type=int, default=7850)
    a = ap.parse_args()
    d = a.d
    key = rt().CommitKey.generate(d, 2)
    eng = B.DeviceCommitEngine(key, 10, 21, b0=14)
    nch = eng.nchunks
    rng = np.random.default_rng(0)
    res = {"b0": eng.b0, "nw": eng.nw}
    csum = torch.zeros((3, nch, 24), dtype=torch.int32, device="cuda")
    for mag in (0, 1000, 5 * 10**5, 10**8, 10**12):
        c = torch.from_numpy(rng.integers(-mag, mag + 1, size=(nch, 10), dtype=np.int64)).cuda()
        res[f"chunk_check_mag{mag:.0e}_us"] = round(timed(lambda: eng.check_chunks(c, csum), a.iters), 1)
    q = torch.from_numpy(rng.integers(-3000, 3000, size=(70, d), dtype=np.int64)).cuda()
    pts, _ = eng.shares(q, torch.arange(70, dtype=torch.int32, device="cuda"))
    flat = pts.view(70, nch * 22, 24)
    cols = torch.from_numpy((np.arange(nch) * 22 + 21).astype(np.int32)).cuda().repeat(3)
    mask = torch.ones(70, dtype=torch.int32, device="cuda")
    res["sum_rows_csum_us"] = round(timed(lambda: B.sum_rows(flat, None, cols, check=False, row_mask=mask), a.iters), 1)
    res["shares_msm_70_us"] = round(timed(lambda: eng.shares(q, torch.arange(70, dtype=torch.int32, device="cuda")),
                                          3), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
