"""CentralBlockML prototype (CentralBlockML/code/*.py): model *branches* instead of one chain.

Each client computes one softmax-regression step against every branch head
(``privateFun``: delta = -alpha * (grad/batch + lambda W), alpha 1e-2, lambda 0.01, batch 100,
softmax_model_obj.py:56-100), picks a branch by comparing that delta with the branch's previous
update, and submits it there; every branch then appends W + mean(pending deltas)
(modelBranch.py:11-25).  Clients hold per-class shards (``mnist_unif{i}``), poisoners the 4->9
flipped set, and the run reports each client's best-branch test error and the 4->9 attack rate
(client.py:33-61).  ``invert`` reproduces inversion.py's gradient-to-image view.

Quirk kept (and flagged): the reference compares with ``scipy.spatial.distance.cosine`` -- a
*distance* -- under a variable named ``sim`` and keeps the *largest*, i.e. it selects the LEAST
similar branch.  ``select="reference"`` keeps that; ``select="similar"`` picks the most similar.

MI355X mapping: all clients x branches gradients are one batched GEMM pass on the device.
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np
import torch


class CentralBlock:
    def __init__(self, n_branches: int = 1, poisoners: int = 6, batch: int = 100, alpha: float = 1e-2,
                 lammy: float = 0.01, select: str = "reference", seed: int = 0, device=None):
        from . import data as D

        self.dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        Xtr, ytr, Xte, yte = D.synthetic_mnist(20000, 4000, seed)
        Xtr, _, _ = D.standardize_cols(Xtr.astype(np.float64))
        Xte, _, _ = D.standardize_cols(Xte.astype(np.float64))
        self.C, self.F = 10, Xtr.shape[1]
        g = torch.Generator().manual_seed(seed)
        self.clients = []                           # (X, y) per client: 10 per-class shards + poisoners
        for k in range(10):
            idx = np.nonzero(ytr == k)[0]
            self.clients.append((idx, None))
        bad = np.nonzero(ytr == 4)[0]
        for _ in range(poisoners):
            self.clients.append((bad, 9))              # mnist_unif_bad_4_9: 4s labelled 9
        self.X = torch.from_numpy(Xtr).float().to(self.dev)
        self.y = torch.from_numpy(ytr).long().to(self.dev)
        self.Xte = torch.from_numpy(Xte).float().to(self.dev)
        self.yte = torch.from_numpy(yte).long().to(self.dev)
        self.batch, self.alpha, self.lammy, self.select = batch, alpha, lammy, select
        w0 = torch.rand(self.C * self.F, generator=g, dtype=torch.float64) / 100.0
        # chain per branch: [(W, previous update)], initial grad = initial W (main.py:33-35)
        self.branches = [[(w0.to(self.dev), w0.to(self.dev))] for _ in range(n_branches)]
        self.history: list = []
        self.gen = torch.Generator(device=self.dev).manual_seed(seed)

    def _deltas(self, W: torch.Tensor) -> torch.Tensor:
        """privateFun for every client at branch weights W: [clients, C*F]."""
        Xs, Ys = [], []
        for idx, flip in self.clients:
            ii = torch.from_numpy(idx).to(self.dev)
            pick = ii[torch.randint(0, len(ii), (self.batch,), generator=self.gen, device=self.dev)]
            Xs.append(self.X[pick])
            Ys.append(self.y[pick] if flip is None else torch.full((self.batch,), flip, device=self.dev))
        X = torch.stack(Xs).double()                          # [n, b, F]
        Y = torch.stack(Ys)
        Wm = W.view(self.C, self.F)
        XW = X @ Wm.T                                         # [n, b, C]
        P = torch.softmax(XW, dim=2)
        P.scatter_add_(2, Y[..., None], -torch.ones_like(Y[..., None], dtype=P.dtype))
        g = torch.einsum("nbc,nbf->ncf", P, X) / self.batch + self.lammy * Wm
        return -self.alpha * g.reshape(len(self.clients), -1)

    def step(self) -> None:
        heads = [b[-1] for b in self.branches]
        deltas = [self._deltas(W) for W, _ in heads]          # per branch [n, C*F]
        pending = [[] for _ in self.branches]
        for c in range(len(self.clients)):
            best, best_v = 0, None
            for bi, (W, prev) in enumerate(heads):
                d = deltas[bi][c]
                cos = torch.dot(d, prev) / (d.norm() * prev.norm() + 1e-300)
                v = float(1.0 - cos) if self.select == "reference" else float(cos)   # scipy cosine distance
                if best_v is None or v > best_v:
                    best, best_v = bi, v
            pending[best].append(deltas[best][c])
        for bi, br in enumerate(self.branches):
            if pending[bi]:
                new_grad = torch.stack(pending[bi]).mean(0)
                br.append((br[-1][0] + new_grad, new_grad))
        self.history.append([len(p) for p in pending])

    def evaluate(self) -> dict:
        best_err, best_att = 1.0, 0.0
        for br in self.branches:
            W = br[-1][0].float().view(self.C, self.F)
            pred = (self.Xte @ W.T).argmax(1)
            err = float((pred != self.yte).float().mean())
            m4 = self.yte == 4
            att = float((pred[m4] == 9).float().mean()) if bool(m4.any()) else 0.0
            if err < best_err:
                best_err, best_att = err, att
        return {"best_test_error": best_err, "attack_rate_4_to_9": best_att}


def invert(grad: np.ndarray, num_classes: int = 10, num_features: int = 784, cls: int = 1) -> np.ndarray:
    """inversion.py: one class row of a gradient, scaled so the maximum reads 2.55."""
    g = np.asarray(grad, dtype=np.float64)
    return np.reshape(g, (num_classes, num_features))[cls] * 2.55 / np.amax(g)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="biscotti_amd.centralblock", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--branches", type=int, default=1)
    ap.add_argument("--poisoners", type=int, default=6)
    ap.add_argument("--select", default="reference", choices=["reference", "similar"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    cb = CentralBlock(a.branches, a.poisoners, select=a.select, seed=a.seed, device=a.device)
    for _ in range(a.iters):
        cb.step()
    print(json.dumps(cb.evaluate()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
