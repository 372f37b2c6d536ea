"""Isolated timings of the round's non-MSM kernels at the MNIST-100 shapes (no concurrent MSM):
how much of their in-round duration is contention with the speculative MSM.

    python scripts/kernel_microbench.py [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd.ops import ml as K  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, d = 70, 7850
    g = torch.Generator(device=dev).manual_seed(0)
    delta = torch.randn((n, d), device=dev, generator=g) * 0.01
    X = torch.randn((n, d), device=dev, generator=g)
    tbl = K.noise_table(100, d, 1, dev)
    noisers = torch.randint(0, 100, (n, 2), device=dev, dtype=torch.int32, generator=g)
    scales = torch.full((n, 2), -0.5, device=dev)
    rows = torch.randperm(n, device=dev, generator=g).to(torch.int32)
    ex = torch.rand((3349, 784), device=dev, generator=g)
    ey = torch.randint(0, 10, (3349,), device=dev, dtype=torch.int32, generator=g)
    W = torch.randn(7850, device=dev, dtype=torch.float64, generator=g) * 0.01
    res = {
        "dp_noise_tbl_us": timed(lambda: K.dp_noise(delta, noisers, scales, 1, 3, table=tbl, rows=rows), a.iters),
        "dp_noise_philox_us": timed(lambda: K.dp_noise(delta, noisers, scales, 1, 3), a.iters),
        "krum_us": timed(lambda: K.krum_async(X, 35, 35), a.iters),
        "eval_two_sets_us": timed(lambda: K.eval_errors_async(ex, ey, 2000, W, 784, 10), a.iters),
    }
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
