"""LSH sieve: the third poisoning defence of the reference's research code, next to Krum and RONI
(ML/code/logistic_aggregator.py:7-29).

    lsh_sieve(deltas):  full_grad = sum_i deltas[i] / #neighbours(i),
    neighbours(i) = { j : ||c_i - c_j||^2 < 1/d },  c = deltas - mean(deltas)   (i itself included)

so a cluster of near-identical (sybil) updates contributes the weight of ONE update.  The reference
asks a FALCONN random-projection LSH index for the neighbours (`find_near_neighbors(c_i, 1/d)`, squared
Euclidean distance, an approximate query).  Here the candidates come from L tables of K random
hyperplane sign bits (kernels ml.hip LS1) -- or from every pair (tables=0: the exact query) -- and
every candidate is confirmed on the f64 Gram of the updates (KC1 + LS2), so a reported neighbour is a
true neighbour; the LSH can only miss some (as FALCONN can).  The weighted sum is LS3.

As a Biscotti verifier (`--defense LSH`, protocol/verify.py) each verifier runs the sieve over its own
inbox and signs the updates of weight 1 (no near-duplicate): an update inside a cluster of c sybils
would carry weight 1/c, and a verifier can only accept or reject (the secure aggregation sums whole
updates).
"""
from __future__ import annotations

import numpy as np
import torch

from ..native import hip
from . import ml as K


def _p(t):
    return None if t is None else t.data_ptr()


def planes(tables: int, bits: int, D: int, seed: int, device) -> torch.Tensor:
    """The L*K random hyperplanes [L*K, D] (fp32, N(0,1)), the same for every rank and the CPU path."""
    g = torch.Generator().manual_seed(int(seed) & (2**63 - 1))
    return torch.randn((tables * bits, D), generator=g, dtype=torch.float32).to(device)


def codes(X: torch.Tensor, mu: torch.Tensor, P: torch.Tensor, tables: int, bits: int) -> torch.Tensor:
    """int32 [n, tables]: bucket of each row in each table (bit b = sign of <x - mu, plane>)."""
    n, D = X.shape
    out = torch.empty((n, tables), dtype=torch.int32, device=X.device)
    if tables == 0 or n == 0:
        return out
    if X.device.type == "cuda":
        err = hip().bsc_lsh_codes(_p(X.contiguous()), _p(mu.contiguous()), n, D, _p(P.contiguous()), tables, bits,
                                  _p(out), torch.cuda.current_stream(X.device).cuda_stream)
        if err != 0:
            raise RuntimeError(f"HIP launch of lsh_codes failed ({err})")
        return out
    proj = ((X - mu).double() @ P.double().T) > 0                       # [n, L*K]
    w = (1 << torch.arange(bits, dtype=torch.int64))
    return (proj.view(n, tables, bits).long() * w).sum(-1).to(torch.int32)


def neighbour_counts(X: torch.Tensor, thr: float, rows_sets, tables: int = 4, bits: int = 12, seed: int = 0):
    """For each list of row indices in rows_sets (e.g. each verifier's inbox): the neighbour count of
    every listed row among the rows of the same list.  One Gram over all rows of X."""
    n, D = X.shape
    mu = X.mean(0)
    P = planes(tables, bits, D, seed, X.device) if tables else None
    cd = codes(X, mu, P, tables, bits) if tables else torch.zeros((n, 0), dtype=torch.int32, device=X.device)
    if X.device.type == "cuda":
        pre = K.gram_stacked_async(X.contiguous(), X[:0])
        outs = []
        for rows in rows_sets:
            r = torch.as_tensor(rows, dtype=torch.int32).to(X.device)
            c = torch.empty((r.numel(),), dtype=torch.int32, device=X.device)
            err = hip().bsc_lsh_count(_p(pre["gram"]), n, _p(cd.contiguous()), tables, _p(r), r.numel(), float(thr),
                                      _p(c), torch.cuda.current_stream(X.device).cuda_stream)
            if err != 0:
                raise RuntimeError(f"HIP launch of lsh_count failed ({err})")
            outs.append(c)
        return [o.cpu() for o in outs]
    G = K._gram_exact_order(X)
    sq = torch.diagonal(G)
    outs = []
    for rows in rows_sets:
        r = torch.as_tensor(rows, dtype=torch.long)
        d2 = sq[r][:, None] + sq[r][None, :] - 2.0 * G[r][:, r]
        cand = torch.ones((len(r), len(r)), dtype=torch.bool) if tables == 0 else \
            (cd[r][:, None, :] == cd[r][None, :, :]).any(-1)
        near = cand & (d2 < thr)
        near.fill_diagonal_(True)
        outs.append(near.sum(1).to(torch.int32))
    return outs


def lsh_sieve(deltas: torch.Tensor, thr: float | None = None, tables: int = 4, bits: int = 12, seed: int = 0):
    """logistic_aggregator.lsh_sieve: (full_grad fp64 [d], neighbour counts int32 [n]).  thr defaults to
    the reference's 1/d; tables = 0 asks the exact neighbour query."""
    n, D = deltas.shape
    thr = 1.0 / D if thr is None else float(thr)
    X = deltas.float().contiguous()
    cnt = neighbour_counts(X, thr, [list(range(n))], tables, bits, seed)[0]
    w = (1.0 / cnt.double()).to(X.device)
    if X.device.type == "cuda":
        out = torch.empty((D,), dtype=torch.float64, device=X.device)
        err = hip().bsc_weighted_rows(_p(X), n, D, _p(w.contiguous()), _p(out),
                                      torch.cuda.current_stream(X.device).cuda_stream)
        if err != 0:
            raise RuntimeError(f"HIP launch of weighted_rows failed ({err})")
        return out, cnt
    return (w[:, None] * X.double()).sum(0), cnt


def sieve_accept(X: torch.Tensor, inboxes: list, d: int, tables: int = 4, bits: int = 12, seed: int = 0):
    """Verifier decisions of the LSH-sieve defence: acc[v][i] = update inbox[v][i] has no near-duplicate
    (weight 1) among verifier v's inbox.  X: the candidates' noised updates, inbox entries are rows."""
    counts = neighbour_counts(X.float().contiguous(), 1.0 / d, inboxes, tables, bits, seed)
    return np.stack([(c.numpy() == 1) for c in counts]) if counts else np.zeros((0, 0), bool)
