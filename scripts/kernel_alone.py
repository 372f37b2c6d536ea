"""The round's side kernels timed ALONE on the GPU (nothing else queued), against their times inside the round
(rocprofv3 kernel stats, where they share the chip with the share MSMs): the noise-aware Krum Gram, the test-set
evaluation, the aggregate audit (chunk commitments of the recovered coefficients), the miners' witness sums
and the commitment sums.  Headline shapes (100 peers, d = 7850, T = 21).  One JSON line per op:
{"op", "alone_us_median", "alone_us_min", "reps"}.

    python scripts/kernel_alone.py [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd.ops import bn256 as B  # noqa: E402
from biscotti_amd.ops import ml as K  # noqa: E402
from biscotti_amd.parallel.comm import Comm  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402
from biscotti_amd.protocol.engine import BiscottiEngine  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    out.sort()
    return out[len(out) // 2], out[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    eng = BiscottiEngine(RunConfig(num_nodes=100, seed=0, max_iterations=10**9, lazy_eval=True), Comm.init())
    for _ in range(12):
        eng.run_round()
    eng.drain()
    torch.cuda.synchronize()
    dev, d, nch, T = eng.dev, eng.d, eng.nchunks, eng.T
    g = torch.Generator(device="cpu").manual_seed(1)
    res = []

    # noise-aware Krum Gram: [100 deltas; 100 noise rows] with the noise x noise tiles from the table
    delta = (torch.randn((100, d), generator=g) * 0.05).float().to(dev)
    nn = eng._noise_gram_table()
    rows = eng.noise_rows.rows(7)
    res.append(("k_gram_pairs (Krum Gram, 100+100 rows)",
                timed(lambda: K.gram_stacked_async(delta, rows, nn=nn[7] if nn is not None else None), a.reps)))
    # evaluation of the test and attack sets
    W = eng.W
    res.append(("k_eval_error_t (test + attack sets)", timed(lambda: eng.task.evaluate_async(W), a.reps)))
    # the share MSM's outputs for 35 rows (witness sums, commitment sums, audit)
    q = eng._pre["qdelta"] if eng._pre is not None else None
    if q is None:
        q = torch.randint(-3000, 3000, (100, d), generator=g, dtype=torch.int64).to(dev)
    rows35 = torch.arange(35, dtype=torch.int32, device=dev)
    pts, ys = eng.crypto.eng.shares(q, rows35, check_rows=False)
    torch.cuda.synchronize()
    flat = pts.view(35, nch * (T + 1), 24)
    wcols = torch.tensor([k * (T + 1) + s for k in range(nch) for s in range(T)], dtype=torch.int32, device=dev)
    ccols = torch.tensor([k * (T + 1) + T for k in range(nch)], dtype=torch.int32, device=dev)
    mask = torch.ones(35, dtype=torch.int32, device=dev)
    res.append(("k_sum_rows2 (witness sums: 35 rows x 21 points x chunks)",
                timed(lambda: B.sum_rows(flat, None, wcols, check=False, row_mask=mask), a.reps)))
    res.append(("k_sum_rows2 (commitment sums: 35 rows x chunks)",
                timed(lambda: B.sum_rows(flat, None, ccols, check=False, row_mask=mask), a.reps)))
    csum = B.sum_rows(flat, None, ccols, check=False, row_mask=mask).view(1, nch, 24)
    coeffs = torch.randint(-3000, 3000, (nch, eng.cfg.poly_size), generator=g, dtype=torch.int64).to(dev)
    res.append(("k_chunk_check (audit, 1 miner)", timed(lambda: eng.crypto.eng.check_chunks(coeffs, csum), a.reps)))
    res.append(("k_shares_msm (35 rows, all lanes)",
                timed(lambda: eng.crypto.eng.shares(q, rows35, check_rows=False), max(5, a.reps // 4))))
    for name, (med, mn) in res:
        print(json.dumps({"op": name, "alone_us_median": round(med, 1), "alone_us_min": round(mn, 1), "reps": a.reps}))
    eng.close()


if __name__ == "__main__":
    main()
