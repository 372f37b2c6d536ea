"""Protocol-level robustness model of a Biscotti MNIST run (CPU, seconds per 100 rounds).

It reproduces the *learning* dynamics of the engine without the cryptography (exact secure
aggregation recovers exactly the sum of the quantised deltas, so the model trajectory does not
depend on it):

  * every worker: one clipped minibatch gradient of the softmax model (client.py:38-65), delta = -g
  * noise: each worker's noisers' getNoise vectors averaged (client_obj.py:97-98, main.go:1592-1660)
  * each verifier: its OWN inbox = first KRUM_UPDATETHRESH arrivals in its own arrival order,
    sorted by SourceID, Multi-Krum on the noised deltas (krum.go:284-322, client_obj.py:114-143)
  * approval: >= floor(nv/2) signatures (main.go:1686)
  * the leader miner fires at NUM_SAMPLES/2 shares (main.go:360): the block carries the first
    approved updates to arrive, W += their (un-noised) sum, honest.go:405-411

It is a research tool for calibrating data and checking defence behaviour before spending GPU
time; the numbers that are reported come from the engine itself (bench.py presets).

    python scripts/robustness_sim.py --peers 100 --po 0.3 --ep 1.0 --nv 3 --seeds 3
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def krum_accept(X: torch.Tensor) -> torch.Tensor:
    n = X.shape[0]
    clip = n // 2
    g = n - clip
    sq = (X * X).sum(1)
    dist = sq[:, None] + sq[None] - 2 * X @ X.T
    srt, _ = torch.sort(dist, 1)
    hi = max(1, min(g - 1, n))
    sc = srt[:, 1:hi].sum(1)
    order = torch.argsort(sc, stable=True)
    acc = torch.zeros(n, dtype=torch.bool)
    acc[order[: n - clip]] = True
    return acc


def run(a, seed: int, fed) -> dict:
    from biscotti_amd.data import mnist_federation  # noqa: F401

    N = a.peers
    rng = np.random.default_rng(seed)
    poison_index = math.ceil(N * (1 - a.po)) if a.po > 0 else N + 1
    poisoners = {i for i in range(N) if i > poison_index}
    Xs = [torch.from_numpy(fed.bad_X if i in poisoners else fed.shards_X[i]) for i in range(N)]
    ys = [torch.from_numpy(fed.bad_y if i in poisoners else fed.shards_y[i]) for i in range(N)]
    Xte = torch.from_numpy(fed.test_X).float() * 2 - 1
    yte = torch.from_numpy(fed.test_y)
    Xat = torch.from_numpy(fed.attack_X).float() * 2 - 1
    yat = torch.from_numpy(fed.attack_y)
    W = torch.zeros(10, 784, dtype=torch.float64)
    b = torch.zeros(10, dtype=torch.float64)
    sigma = math.sqrt(2 * math.log(1.25 / 1e-5)) / a.ep if a.ep > 0 else 0.0
    nsamp = min(int(N * a.ns / 100), N - a.nv - a.na)
    thresh = nsamp
    hist = []
    pa_hist = []
    for it in range(a.rounds):
        committee = set(rng.choice(N, a.nv + a.na, replace=False).tolist())
        verifiers = sorted(list(committee))[: a.nv]
        workers = [i for i in range(N) if i not in committee]
        # local step (all workers)
        xb, yb = [], []
        for w in workers:
            idx = rng.choice(Xs[w].shape[0], a.batch, replace=False)
            xb.append(Xs[w][idx])
            yb.append(ys[w][idx])
        xb = torch.stack(xb).float() * 2 - 1            # (x - 0.5) / 0.5
        yb = torch.stack(yb).long()
        Wf, bf = W.float(), b.float()
        logits = xb @ Wf.T + bf
        p = torch.softmax(logits, -1)
        oh = torch.nn.functional.one_hot(yb, 10).float()
        gz = (p - oh) / a.batch                          # [P, B, 10]
        dW = torch.einsum("pbk,pbd->pkd", gz, xb)
        db = gz.sum(1)
        flat = torch.cat([dW.reshape(len(workers), -1), db], 1).double()
        nrm = flat.norm(dim=1, keepdim=True)
        coef = (100.0 / (nrm + 1e-6)).clamp(max=1.0)
        delta = -(flat * coef)
        delta = torch.trunc(delta * 1e4) / 1e4            # quantise (kyber.go:698-710)
        noise = torch.zeros_like(delta)
        if sigma > 0 and a.noise:
            noise = (-sigma / math.sqrt(a.batch)) * torch.randn(delta.shape, generator=torch.Generator().manual_seed(
                seed * 100003 + it)).double() / math.sqrt(a.nn)  # mean of nn independent noisers
        noised = delta + noise
        # per-verifier inboxes + Krum
        sigs = np.zeros(len(workers), np.int64)
        for v in verifiers:
            if a.shared_inbox:
                order = np.random.default_rng(seed * 7 + it).permutation(len(workers))
            else:
                order = rng.permutation(len(workers))
            inbox = np.sort(order[:thresh])
            acc = krum_accept(noised[torch.from_numpy(inbox)]) if a.krum else torch.ones(len(inbox), dtype=torch.bool)
            sigs[inbox[acc.numpy()]] += 1
        need = a.nv // 2 if a.krum else 0
        approved = [k for k in range(len(workers)) if sigs[k] >= need]
        # leader fires at NUM_SAMPLES/2 shares: first arrivals in its own order
        if a.miner_cap:
            order = rng.permutation(len(approved))
            approved = sorted(approved[k] for k in order[: nsamp // 2])
        if len(approved) > 1:
            s = delta[approved].sum(0)
            W += s[:7850 - 10].view(10, 784)
            b += s[7850 - 10:]
        npois = sum(1 for k in approved if workers[k] in poisoners)
        pa_hist.append((len(approved), npois))
        with torch.no_grad():
            pred = (Xte @ W.float().T + b.float()).argmax(1)
            err = float((pred != yte).float().mean())
            pa = (Xat @ W.float().T + b.float()).argmax(1)
            att = float((pa != yat).float().mean())
        hist.append((err, att))
    e = np.array(hist)
    return {"seed": seed, "final_err": e[-1, 0], "final_attack": e[-1, 1], "err_last10": e[-10:, 0].mean(),
            "attack_last10": e[-10:, 1].mean(), "approved_mean": float(np.mean([x[0] for x in pa_hist])),
            "poisoners_in_block_last10": float(np.mean([x[1] for x in pa_hist[-10:]])),
            "curve_err": [round(float(x), 4) for x in e[:, 0]], "curve_attack": [round(float(x), 4) for x in e[:, 1]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=100)
    ap.add_argument("--po", type=float, default=0.0)
    ap.add_argument("--ep", type=float, default=2.0)
    ap.add_argument("--nv", type=int, default=3)
    ap.add_argument("--na", type=int, default=3)
    ap.add_argument("--nn", type=int, default=2)
    ap.add_argument("--ns", type=int, default=70)
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--seeds", type=int, default=1)
    ap.add_argument("--no-noise", dest="noise", action="store_false")
    ap.add_argument("--no-krum", dest="krum", action="store_false", help="accept every update (FedSys-like)")
    ap.add_argument("--shared-inbox", action="store_true", help="round-1 semantics: one inbox for all verifiers")
    ap.add_argument("--no-miner-cap", dest="miner_cap", action="store_false")
    ap.add_argument("--data-seed", type=int, default=1234)
    ap.add_argument("--curves", action="store_true")
    a = ap.parse_args()
    from biscotti_amd.data import mnist_federation

    fed = mnist_federation(a.peers, seed=a.data_seed)
    res = [run(a, s, fed) for s in range(a.seeds)]
    keys = ["final_err", "final_attack", "err_last10", "attack_last10", "approved_mean", "poisoners_in_block_last10"]
    summ = {k: (float(np.mean([r[k] for r in res])), float(np.std([r[k] for r in res]))) for k in keys}
    out = {"args": vars(a), "summary": summ}
    if a.curves:
        out["runs"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
