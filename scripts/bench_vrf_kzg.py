"""Microbench of the device audit kernels: DeviceVrfProver.prove (N proofs) and the KZG RLC sums of an
MNIST-sized aggregate (785 chunks x 21 share points).  Prints one JSON line."""
import argparse
import json
import os
import time

import numpy as np
import torch

from biscotti_amd.native import rt
from biscotti_amd.ops import bn256 as B
from biscotti_amd.ops.vrf import DeviceVrfProver


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=1560)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    out = {}
    pr = DeviceVrfProver("cuda")
    seeds = [os.urandom(32) for _ in range(a.proofs)]
    alpha = [os.urandom(32)] * a.proofs
    out["vrf_prove_ms"] = timed(lambda: pr.prove(seeds, alpha), a.iters)
    R = rt()
    key = R.CommitKey.generate(7850, 2)
    eng = B.DeviceCommitEngine(key, 10, 21, b0=8)
    coeffs = torch.from_numpy(np.random.default_rng(0).integers(-3000, 3000, size=(3, 7850))).cuda()
    pts, ys = eng.shares(coeffs, torch.arange(3, dtype=torch.int32, device="cuda"))
    nch = eng.nchunks
    flat = pts.reshape(3, nch * 22, 24)
    base = np.arange(nch) * 22
    c = lambda v: torch.from_numpy(np.asarray(v, np.int32)).cuda()
    csum = B.sum_rows(flat, None, c(base + 21))
    wcols = np.concatenate([(base[:, None] + 7 * m + np.arange(7)[None, :]).reshape(-1) for m in range(3)])
    wsum = B.sum_rows(flat, None, c(wcols))
    yagg = ys.sum(0).contiguous()
    xs = c(np.arange(21) - 10)
    out["kzg_rlc_ms"] = timed(lambda: eng.kzg_rlc(csum, wsum, yagg, xs, 7, False, 1234), a.iters)
    res = eng.kzg_rlc(csum, wsum, yagg, xs, 7, False, 99).cpu().numpy().view(np.uint32)
    g2 = R.g2_generator()
    t = time.perf_counter()
    out["kzg_ok"] = R.kzg_check_device_async(res, g2, R.g2_mul(g2, 2)).result()
    out["pairing_ms"] = (time.perf_counter() - t) * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
