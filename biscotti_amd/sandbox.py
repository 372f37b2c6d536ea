"""Standalone training sandboxes (ML/Pytorch/ml_main_{mnist,cifar,lfw,credit,diffpriv}.py).

    python -m biscotti_amd.sandbox --model softmax --dataset mnist --clients 10 --poisoned 4
    python -m biscotti_amd.sandbox --model mnist_cnn --iters 500
    python -m biscotti_amd.sandbox --model cifar_cnn --dataset cifar
    python -m biscotti_amd.sandbox --model lfw_cnn --dataset lfw
    python -m biscotti_amd.sandbox --model softmax --dp-epsilon 1.0      # ml_main_diffpriv

Reference loop (ml_main_mnist.py): ``clients`` peers (the last ``poisoned`` train on the 1->7
label-flipped set) each compute the gradient of one minibatch on the shared model, the gradients
are SUMMED, one SGD step (lr 1e-3, momentum 0.75, weight decay 1e-3, client.py:30) is taken, and
every ``eval_every`` iterations the loss, test error and 1-attack rate are printed.

MI355X mapping: the per-client gradient sum equals the gradient of the summed per-client mean
losses, so all clients' minibatches go through ONE forward/backward over a [clients*batch, ...]
batch on the GPU instead of ``clients`` tiny ones (PyTorch-ROCm; MIOpen convolutions for the CNNs).
DP (ml_main_diffpriv): Gaussian noise sigma = sqrt(2 ln(1.25/delta))/eps per client, averaged over
the batch like client_obj.getNoise.
"""
from __future__ import annotations

import argparse
import json
import math
import sys

import numpy as np
import torch
import torch.nn.functional as F


def _data(dataset: str, seed: int):
    from . import data as D

    if dataset == "mnist":
        Xtr, ytr, Xte, yte = D.synthetic_mnist(60000, 10000, seed)
        Xtr, mu, sd = D.standardize_cols(Xtr.astype(np.float64))
        Xte, _, _ = D.standardize_cols(Xte.astype(np.float64))
        return Xtr.astype(np.float32), ytr, Xte.astype(np.float32), yte, 10
    if dataset == "cifar":
        X, y = D.synthetic_images(12000, (3, 32, 32), 10, seed)
        return X[:10000], y[:10000], X[10000:], y[10000:], 10
    if dataset == "lfw":
        X, y = D.synthetic_images(3000, (3, 62, 47), 12, seed)
        return X[:2400], y[:2400], X[2400:], y[2400:], 12
    if dataset == "creditcard":
        cd = D.creditcard()
        y = (cd.y > 0).astype(np.int64)
        yv = (cd.yvalid > 0).astype(np.int64)
        return cd.X.astype(np.float32), y, cd.Xvalid.astype(np.float32), yv, 2
    raise ValueError(dataset)


def _model(name: str, d_in: int, n_classes: int):
    from .models import zoo as Z

    return {"softmax": lambda: Z.SoftmaxModel(d_in, n_classes), "svm": lambda: Z.SVMModel(d_in, n_classes),
            "mnist_cnn": Z.MNISTCNNModel, "lfw_cnn": lambda: Z.LFWCNNModel(n_classes),   # the reference's head has 2 outputs; the
            # synthetic LFW stand-in has 12 identities, so the head is sized to the data
            "cifar_cnn": Z.CIFARCNNModel}[name]()


def run(model="softmax", dataset="mnist", clients=10, poisoned=0, iters=2000, batch=10, lr=1e-3, momentum=0.75,
        weight_decay=1e-3, eval_every=100, dp_epsilon=0.0, seed=0, device=None, verbose=True) -> dict:
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    torch.manual_seed(seed)
    Xtr, ytr, Xte, yte, C = _data(dataset, seed)
    shards = np.array_split(np.random.default_rng(seed).permutation(len(Xtr)), max(1, clients - poisoned))
    Xtr_t, ytr_t = torch.from_numpy(Xtr).to(dev), torch.from_numpy(ytr).to(dev)
    Xte_t, yte_t = torch.from_numpy(Xte).to(dev), torch.from_numpy(yte).to(dev)
    ones = torch.nonzero(ytr_t == 1).flatten()
    bad_y = torch.full_like(ytr_t[ones], 7 if C > 7 else 0)   # generate_poisoned: 1 -> 7
    net = _model(model, Xtr.shape[1], C).to(dev)
    opt = torch.optim.SGD(net.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)
    sigma = math.sqrt(2 * math.log(1.25 / 1e-5)) / dp_epsilon if dp_epsilon > 0 else 0.0
    g = torch.Generator(device=dev).manual_seed(seed)
    shard_t = [torch.from_numpy(s).to(dev) for s in shards]
    hist = []
    for it in range(iters):
        xs, ys, owners = [], [], []
        for c in range(clients):
            if c < clients - poisoned:
                idx = shard_t[c][torch.randint(0, len(shard_t[c]), (batch,), generator=g, device=dev)]
                xs.append(Xtr_t[idx]); ys.append(ytr_t[idx])
            else:
                k = torch.randint(0, len(ones), (batch,), generator=g, device=dev)
                xs.append(Xtr_t[ones[k]]); ys.append(bad_y[k])
        X, Y = torch.cat(xs), torch.cat(ys)
        opt.zero_grad(set_to_none=True)
        per = F.cross_entropy(net(X), Y, reduction="none").view(clients, batch)
        loss = per.mean(1).sum()          # sum over clients of each client's mean minibatch loss
        loss.backward()
        if sigma > 0:
            for p in net.parameters():    # client_obj.getNoise: per client, averaged over the batch
                p.grad.add_(torch.randn(p.shape, generator=g, device=dev) * (sigma * math.sqrt(clients) / batch))
        opt.step()
        if it % eval_every == 0 or it == iters - 1:
            with torch.no_grad():
                pred = net(Xte_t).argmax(1)
                err = float((pred != yte_t).float().mean())
                m1 = yte_t == 1
                att = float((pred[m1] != 1).float().mean()) if bool(m1.any()) else float("nan")
            hist.append({"iter": it, "loss": float(loss.detach()) / clients, "test_error": err, "attack_rate": att})
            if verbose:
                print(f"Average loss is {hist[-1]['loss']:.5f}\nTest error: {err:.5f}\nAttack rate on 1s: {att:.5f}\n")
    return {"model": model, "dataset": dataset, "final_test_error": hist[-1]["test_error"],
            "final_attack_rate": hist[-1]["attack_rate"], "history": hist}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="biscotti_amd.sandbox", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="softmax", choices=["softmax", "svm", "mnist_cnn", "lfw_cnn", "cifar_cnn"])
    ap.add_argument("--dataset", default="mnist", choices=["mnist", "cifar", "lfw", "creditcard"])
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--poisoned", type=int, default=0)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--momentum", type=float, default=0.75)
    ap.add_argument("--eval-every", type=int, default=100)
    ap.add_argument("--dp-epsilon", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    res = run(a.model, a.dataset, a.clients, a.poisoned, a.iters, a.batch, a.lr, a.momentum, 1e-3, a.eval_every,
              a.dp_epsilon, a.seed, a.device)
    print(json.dumps({k: v for k, v in res.items() if k != "history"}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
