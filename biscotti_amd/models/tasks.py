"""Batched learning tasks: all virtual peers hosted by one rank as device tensors.

SoftmaxTask  -- MNIST softmax regression (the Biscotti path; ML/Pytorch/client_obj.py + client.py)
LogisticTask -- creditcard logistic regression (ML/code/logistic_model.py), DP noise at source

``step(W, iteration)`` runs the local update of every *listed* local peer in one fused kernel and
returns (delta fp32 [n, d], qdelta int64 [n, d]); ``evaluate(W)`` returns the logged metrics.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import data as D
from ..ops import ml as K
from ..utils import h2d


class SoftmaxTask:
    d_in, d_out = 784, 10
    stateless_step = True   # step() of a peer depends only on (W, peer, iteration): it can run ahead

    def __init__(self, peers: range, num_peers: int, device, seed: int, poisoned: set[int] | None = None,
                 batch_size: int = 10, data_dir: str | None = None, federation: D.MnistFederation | None = None,
                 dims: tuple | None = None):
        if dims is not None:
            self.d_in, self.d_out = dims
        fed = federation or D.mnist_federation(num_peers, seed=seed, data_dir=data_dir)
        self.source = fed.source
        self.peers = list(peers)
        self.device = torch.device(device)
        self.batch = batch_size
        self.seed = seed
        self.nparam = self.d_out * self.d_in + self.d_out
        poisoned = poisoned or set()
        Xs, ys, offs, ns = [], [], [], []
        o = 0
        for p in self.peers:
            X, y = (fed.bad_X, fed.bad_y) if p in poisoned else (fed.shards_X[p], fed.shards_y[p])
            Xs.append(X)
            ys.append(y)
            offs.append(o)
            ns.append(X.shape[0])
            o += X.shape[0]
        self.X = torch.from_numpy(np.concatenate(Xs).astype(np.float32)).to(self.device)
        self.y = torch.from_numpy(np.concatenate(ys).astype(np.int32)).to(self.device)
        self.off = torch.tensor(offs, dtype=torch.int64, device=self.device)
        self.ntrain = torch.tensor(ns, dtype=torch.int32, device=self.device)
        self.test_X = torch.from_numpy(fed.test_X).to(self.device)
        self.test_y = torch.from_numpy(fed.test_y.astype(np.int32)).to(self.device)
        self.att_X = torch.from_numpy(fed.attack_X).to(self.device)
        self.att_y = torch.from_numpy(fed.attack_y.astype(np.int32)).to(self.device)
        # test | attack rows back to back: both metrics come from one kernel launch + one read-back
        self.eval_X = torch.cat([self.test_X, self.att_X]).contiguous()
        self.eval_y = torch.cat([self.test_y, self.att_y]).contiguous()
        self.eval_split = int(self.test_X.shape[0])
        assert self.peers == list(range(self.peers[0], self.peers[0] + len(self.peers))), "local peers are contiguous"
        self._local_index = {p: i for i, p in enumerate(self.peers)}
        self._sel_cache: dict = {}

    def noise_sigma(self, epsilon: float, delta: float = 1e-5) -> float:
        """client_obj.py:61: sigma = sqrt(2 ln(1.25/delta)) / epsilon (0 when epsilon == 0)."""
        return math.sqrt(2 * math.log(1.25 / delta)) / epsilon if epsilon > 0 else 0.0

    def noise_scale(self, sigma: float) -> float:
        """getNoise = -(1/B) * sum over B of sigma*N(0,1) == -(sigma/sqrt(B)) * N(0,1)."""
        return -sigma / math.sqrt(self.batch)

    def step(self, W: torch.Tensor, iteration: int, peers: list[int]):
        """Local step of the listed local peers -> (delta fp32 [n, d], qdelta int64 [n, d])."""
        if not peers:
            z = torch.empty((0, self.nparam), device=self.device)
            return z.float(), z.long()
        key = tuple(peers)
        pid = self._sel_cache.get(key)
        if pid is None:   # only the peer ids travel; off / ntrain stay resident over all local peers
            pid = h2d(peers, torch.int32, self.device)
            if len(self._sel_cache) < 64:
                self._sel_cache[key] = pid
        delta, qdelta, loss = K.softmax_step(self.X, self.y, self.off, self.ntrain, pid, W, self.d_in, self.d_out,
                                             self.batch, self.seed, iteration, 100.0, 1e4, lo=self.peers[0])
        self.last_loss = loss
        return delta, qdelta

    def evaluate(self, W: torch.Tensor) -> dict:
        return self.evaluate_async(W)()

    def evaluate_async(self, W: torch.Tensor):
        """Queue the test / attack evaluations now; the returned callable reads them back."""
        if self.device.type == "cuda" and getattr(self, "_eval_Xt", None) is None:
            self._eval_Xt = K.eval_tiles(self.eval_X, transform=True)   # the test rows never change
        both = K.eval_errors_async(self.eval_X, self.eval_y, self.eval_split, W, self.d_in, self.d_out,
                                   transform=True, Xt=getattr(self, "_eval_Xt", None))

        def result():
            err, att = both()
            return {"test_error": err, "attack_rate": att}
        result.ready = getattr(both, "ready", lambda: True)
        return result

    def train_error(self, W: torch.Tensor, peer: int, iteration: int) -> float:
        """RONI's getTrainErr: error on a (random) minibatch of the verifier's own shard."""
        i = self._local_index[peer]
        o, n = int(self.off[i]), int(self.ntrain[i])
        rows = K.minibatch_indices(peer, iteration, n, self.batch, self.seed ^ 0xB0B)
        sel = h2d([o + r for r in rows], torch.long, self.device)
        return K.eval_error(self.X[sel].contiguous(), self.y[sel].contiguous(), W, self.d_in, self.d_out, True)


class LogisticTask:
    """creditcard logistic regression: every peer loads the full dataset (logistic_model.py:26)."""

    alpha = 1e-2
    lammy = 0.01

    def __init__(self, peers: range, num_peers: int, device, seed: int, poisoned: set[int] | None = None,
                 batch_size: int = 10, epsilon: float = 0.0, colluders: set[int] | None = None, **_):
        cd = D.creditcard()
        bad = D.credit_poisoned(cd)
        self.peers = list(peers)
        self.device = torch.device(device)
        self.batch = batch_size
        self.seed = seed
        self.nparam = cd.X.shape[1]
        poisoned = poisoned or set()
        Xs, ys, offs, ns = [], [], [], []
        o = 0
        # share one copy of the dataset between honest peers; poisoners point at the flipped copy
        Xs.append(cd.X)
        ys.append(cd.y)
        Xs.append(bad.X)
        ys.append(bad.y)
        n = cd.X.shape[0]
        for p in self.peers:
            offs.append(n if p in poisoned else 0)
            ns.append(n)
        self.X = torch.from_numpy(np.concatenate(Xs)).to(self.device)
        self.y = torch.from_numpy(np.concatenate(ys)).to(self.device)
        self.off = torch.tensor(offs, dtype=torch.int64, device=self.device)
        self.nrows = torch.tensor(ns, dtype=torch.int32, device=self.device)
        # diffPriv16 noise at source: sigma = sqrt(2 ln 1.25)/epsilon (logistic_model.py:81)
        s = math.sqrt(2 * math.log(1.25)) / epsilon if epsilon > 0 else 0.0
        colluders = colluders or set()
        self.sigma = torch.tensor([0.0 if p in colluders else s for p in self.peers], dtype=torch.float64,
                                  device=self.device)
        self.calls = torch.ones((len(self.peers),), dtype=torch.int32, device=self.device)  # `iteration = 1`
        self.Xv = torch.from_numpy(cd.Xvalid).to(self.device)
        self.yv = torch.from_numpy(cd.yvalid).to(self.device)
        self.Xt = torch.from_numpy(cd.X).to(self.device)
        self.yt = torch.from_numpy(cd.y).to(self.device)
        assert self.peers == list(range(self.peers[0], self.peers[0] + len(self.peers))), "local peers are contiguous"
        self._local_index = {p: i for i, p in enumerate(self.peers)}

    def noise_sigma(self, epsilon: float, delta: float = 1e-5) -> float:
        return math.sqrt(2 * math.log(1.25)) / epsilon if epsilon > 0 else 0.0

    def noise_scale(self, sigma: float) -> float:
        return -self.alpha * sigma / math.sqrt(self.batch)

    def step(self, W: torch.Tensor, iteration: int, peers: list[int]):
        idx = [self._local_index[p] for p in peers]
        sel = h2d(idx, torch.long, self.device)
        off, nr = self.off[sel].contiguous(), self.nrows[sel].contiguous()
        sig, calls = self.sigma[sel].contiguous(), self.calls[sel].contiguous()
        pid = h2d(peers, torch.int32, self.device)
        delta, qdelta = K.logreg_step(self.X, self.y, off, nr, pid, W, self.batch, self.seed, calls, self.alpha,
                                      self.lammy, sig, 1e4)
        self.calls[sel] += 1
        return delta, qdelta

    def _err(self, X, y, W) -> float:
        yhat = torch.sign(X @ W)
        return float((yhat != y).sum()) / y.numel()

    def evaluate_async(self, W: torch.Tensor):
        v = self.evaluate(W)
        return lambda: v

    def evaluate(self, W: torch.Tensor) -> dict:
        # logistic_model_test.py: train_error on credittrain, test_error on credittest
        return {"test_error": self._err(self.Xt, self.yt, W), "valid_error": self._err(self.Xv, self.yv, W),
                "attack_rate": 0.0}

    def train_error(self, W: torch.Tensor, peer: int, iteration: int) -> float:
        return self._err(self.Xv, self.yv, W)


def make_task(dataset: str, peers: range, num_peers: int, device, seed: int, **kw):
    if dataset == "mnist":
        kw.pop("epsilon", None)
        kw.pop("colluders", None)
        return SoftmaxTask(peers, num_peers, device, seed, **kw)
    if dataset == "lfw":
        kw.pop("epsilon", None)
        kw.pop("colluders", None)
        kw.pop("data_dir", None)
        _, d_in, d_out = D.dataset_dims("lfw")
        return SoftmaxTask(peers, num_peers, device, seed, federation=D.lfw_federation(num_peers, seed=seed),
                           dims=(d_in, d_out), **kw)
    if dataset == "creditcard":
        kw.pop("data_dir", None)
        kw.pop("federation", None)
        return LogisticTask(peers, num_peers, device, seed, **kw)
    raise ValueError(f"unsupported dataset {dataset!r}")
