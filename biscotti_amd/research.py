"""The reference's research scripts outside the peer runtime (ML/code/*), MI355X-side where it pays:

  lsh         LSH-sieve aggregation of a set of updates (logistic_aggregator.py:7-29; kernels in
              ops/lsh.py), the reference's demo data or a poisoned federation's deltas
  linear      linear least-squares model with AdaGrad steps and top-k (theta) update sparsification
              (linear_model.py:1-129, linear_model_test.py)
  inversion   the model-inversion comparison: a victim model trained with (or without) DP noise at
              source on the label-flipped credit set, against the optimal hinge classifier of that
              set (logistic_main.py, inversion_compare.py:1-41)
  bystander   inversion error when the attacker only sees the victim's update summed with k
              bystanders' updates, for no DP / epsilon 1 / epsilon 5 (inversion_bystander_plot.py);
              writes the bar chart and the numbers

    python -m biscotti_amd.research lsh [--device cuda]
    python -m biscotti_amd.research linear --theta 0.1 --iters 2000
    python -m biscotti_amd.research inversion --epsilon 5 --iters 4000 --runs 5
    python -m biscotti_amd.research bystander --iters 2000 -o bystander.pdf

Data: the reference's logisticData.pkl / linTest / creditbad files are not shipped; `linear` draws a
synthetic regression set, `inversion`/`bystander` use creditcard.csv (shipped) and its label-flipped
copy (data.credit_poisoned), so their numbers are parity-unpinned.
"""
from __future__ import annotations

import argparse
import json
import math
import sys

import numpy as np
import torch


# ---------------------------------------------------------------------------- linear model
class LinearModel:
    """linear_model.py: f = 1/2 ||Xw - y||^2, AdaGrad step -alpha g / (1e-6 + sqrt(sum g^2)), and only the
    top theta*d coordinates of the step kept (privateFun's argpartition filter)."""

    alpha = 1e-2
    lammy = 0.1

    def __init__(self, X: np.ndarray, y: np.ndarray, seed: int = 0, l2: bool = False):
        self.X, self.y = np.asarray(X, np.float64), np.asarray(y, np.float64)
        self.d = self.X.shape[1]
        self.hist_grad = np.zeros(self.d)
        self.rng = np.random.default_rng(seed)
        self.l2 = l2

    def fun_obj(self, ww, X, y):
        r = X @ ww - y
        f = 0.5 * r @ r
        g = X.T @ r
        if self.l2:
            f += 0.5 * self.lammy * ww @ ww
            g = g + self.lammy * ww
        return f, g

    def private_fun(self, theta: float, ww, batch_size: int = 0) -> np.ndarray:
        nn = self.X.shape[0]
        idx = self.rng.choice(nn, batch_size, replace=False) if 0 < batch_size < nn else np.arange(nn)
        _, g = self.fun_obj(np.asarray(ww, np.float64), self.X[idx], self.y[idx])
        self.hist_grad += g ** 2
        delta = -self.alpha * g / (1e-6 + np.sqrt(self.hist_grad))
        if theta < 1:
            k = int(self.d * theta)
            keep = np.argpartition(np.abs(delta), -k)[-k:] if k > 0 else np.zeros(0, np.int64)
            mask = np.zeros(self.d, bool)
            mask[keep] = True
            delta[~mask] = 0.0
        return delta

    @staticmethod
    def test(ww, Xtest, ytest) -> float:
        """linear_model_test.test: 1/2 mean squared error."""
        yhat = Xtest @ np.asarray(ww)
        return float(0.5 * np.sum((ytest - yhat) ** 2 / yhat.size))


def synthetic_regression(n: int = 4000, d: int = 20, noise: float = 0.1, seed: int = 0):
    rng = np.random.default_rng(seed)
    w = rng.normal(size=d)
    X = rng.normal(size=(n, d))
    y = X @ w + noise * rng.normal(size=n)
    cut = int(0.8 * n)
    return X[:cut], y[:cut], X[cut:], y[cut:], w


def run_linear(theta: float, iters: int, batch: int, seed: int) -> dict:
    Xtr, ytr, Xte, yte, w_true = synthetic_regression(seed=seed)
    m = LinearModel(Xtr, ytr, seed)
    w = np.zeros(Xtr.shape[1])
    curve = []
    for it in range(iters):
        w = w + m.private_fun(theta, w, batch)
        if it % max(1, iters // 20) == 0 or it == iters - 1:
            curve.append((it, LinearModel.test(w, Xte, yte)))
    return {"theta": theta, "test_error": curve[-1][1], "curve": curve,
            "weight_error": float(np.linalg.norm(w - w_true) / np.linalg.norm(w_true))}


# ---------------------------------------------------------------------------- model inversion
def _credit(poisoned: bool):
    from . import data as D

    cd = D.creditcard()
    return D.credit_poisoned(cd) if poisoned else cd


def _logistic_deltas(X, y, ww, rng, batch: int, sigma: float, alpha: float = 1e-2, lammy: float = 0.01):
    """logistic_model.privateFun: -alpha * (minibatch gradient + lammy w) plus DP noise at source."""
    idx = rng.choice(X.shape[0], batch, replace=False)
    xb, yb = X[idx], y[idx]
    t = yb * (xb @ ww)
    res = -yb / np.exp(np.logaddexp(0, t))
    g = xb.T @ res / batch + lammy * ww
    d = -alpha * g
    if sigma > 0:
        d = d + (-alpha / batch) * sigma * math.sqrt(batch) * rng.normal(size=ww.shape)
    return d


def train_victim(epsilon: float | None, iters: int, batch: int = 10, bystanders: int = 0, seed: int = 0):
    """Weights the attacker reconstructs: the victim (label-flipped credit data) trained alone, or summed
    with k honest bystanders' updates (the attacker only sees the sum), DP at source when epsilon."""
    rng = np.random.default_rng(seed)
    bad, good = _credit(True), _credit(False)
    sigma = math.sqrt(2 * math.log(1.25)) / epsilon if epsilon else 0.0
    w = rng.random(bad.X.shape[1])
    for _ in range(iters):
        d = _logistic_deltas(bad.X, bad.y, w, rng, batch, sigma)
        for _ in range(bystanders):
            d = d + _logistic_deltas(good.X, good.y, w, rng, batch, sigma)
        w = w + d
    return w


def inversion_compare(victim_w) -> float:
    """inversion_compare.compare: disagreement between the victim model's and the optimal hinge
    classifier's predictions (trained on the attacked set) on the validation rows."""
    from sklearn.linear_model import SGDClassifier

    bad, val = _credit(True), _credit(False)
    clf = SGDClassifier(loss="hinge", penalty="l2", random_state=0)
    clf.fit(bad.X, bad.y)
    real = clf.predict(val.Xvalid)
    victim = np.sign(val.Xvalid @ np.asarray(victim_w))
    return float(np.sum(victim != real) / real.shape[0])


def bystander_table(iters: int, runs: int = 3, seed: int = 0) -> dict:
    out = {}
    for name, eps in (("no_dp", None), ("eps1", 1.0), ("eps5", 5.0)):
        means, stds = [], []
        for by in range(4):
            errs = [inversion_compare(train_victim(eps, iters, bystanders=by, seed=seed + 97 * r)) for r in range(runs)]
            means.append(float(np.mean(errs)))
            stds.append(float(np.std(errs)))
        out[name] = {"mean": means, "std": stds}
    return out


def plot_bystanders(table: dict, path: str) -> None:
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    ind, width = np.arange(4), 0.25
    fig, ax = plt.subplots()
    for k, (name, label, color) in enumerate((("eps1", r"$\varepsilon$ = 1", "red"),
                                              ("eps5", r"$\varepsilon$ = 5", "orange"),
                                              ("no_dp", "No Privacy", "green"))):
        ax.bar(ind + k * width, table[name]["mean"], width, yerr=table[name]["std"], color=color, label=label)
    ax.set_ylabel("Reconstruction Error")
    ax.set_xlabel("# of bystanders (k-2)")
    ax.set_xticks(ind + width)
    ax.set_xticklabels(["0", "1", "2", "3"])
    ax.set_ylim([0, 1])
    ax.legend(loc="best", ncol=3)
    fig.tight_layout()
    fig.savefig(path)


# ---------------------------------------------------------------------------- CLI
def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m biscotti_amd.research")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("lsh")
    p.add_argument("--device", default="cpu")
    p.add_argument("--tables", type=int, default=4)
    p = sub.add_parser("linear")
    p.add_argument("--theta", type=float, default=1.0)
    p.add_argument("--iters", type=int, default=2000)
    p.add_argument("--batch", type=int, default=10)
    p = sub.add_parser("inversion")
    p.add_argument("--epsilon", type=float, default=0.0)
    p.add_argument("--iters", type=int, default=4000)
    p.add_argument("--runs", type=int, default=5)
    p = sub.add_parser("bystander")
    p.add_argument("--iters", type=int, default=2000)
    p.add_argument("--runs", type=int, default=3)
    p.add_argument("-o", "--out", default=None)
    for q in sub.choices.values():
        q.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    if a.cmd == "lsh":
        from .ops.lsh import lsh_sieve

        rng = np.random.default_rng(a.seed)
        good = (rng.random((50, 5)) - 0.5) * 2
        attackers = np.repeat(rng.random((1, 5)) + 0.5, 10, axis=0)
        X = torch.from_numpy(np.vstack((good, attackers))).float().to(a.device)
        grad, cnt = lsh_sieve(X, tables=a.tables)
        res = {"full_grad": grad.cpu().tolist(), "neighbours": cnt.tolist()}
    elif a.cmd == "linear":
        res = run_linear(a.theta, a.iters, a.batch, a.seed)
    elif a.cmd == "inversion":
        errs = [inversion_compare(train_victim(a.epsilon or None, a.iters, seed=a.seed + r)) for r in range(a.runs)]
        res = {"epsilon": a.epsilon, "errors": errs, "mean": float(np.mean(errs)), "std": float(np.std(errs))}
    else:
        res = bystander_table(a.iters, a.runs, a.seed)
        if a.out:
            plot_bystanders(res, a.out)
    json.dump(res, sys.stdout)
    print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
