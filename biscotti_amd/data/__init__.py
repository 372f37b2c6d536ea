"""Datasets and partitioners.

MNIST: the raw MNIST image files are not in the reference (``.MISSING_LARGE_BLOBS``) and there is
no network, so the default MNIST source is *synthetic MNIST-shaped digits*: scikit-learn's bundled
real 8x8 handwritten digits (1797 images), upsampled into a 20x20 box centred on a 28x28 canvas and
augmented (random sub-pixel shift, rotation, stroke scaling and pixel noise) into 60000 train /
10000 test images with values in [0, 255] -- the MNIST shapes and label set.  Real MNIST ``.npy``
shards in the reference layout (``mnist{i}.npy``, ``mnist_test.npy``, ``mnist_digit1.npy``,
``mnist_bad.npy``; last column = label) are used instead when a directory is given.

Partitioning follows ``ML/Pytorch/data/mnist/parse_mnist.py``:
  * standardize_cols on train and (separately) on test                          (:295-306)
  * slice_uniform: shuffle train, N equal shards mnist{i}                        (:111-163)
  * slice_for_tm: per-digit files (mnist_digit{k}) from standardized train        (:65-109)
  * generate_poisoned: mnist_bad = digit-1 rows relabelled 7                     (:309-315)
and ``MNISTDataset`` (mnist_dataset.py:16-44): first 80% of a file is train, last 20% is test.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

FILES = Path(__file__).resolve().parent / "files"
TRAIN_CUT = 0.8
# Augmentation strength, calibrated against the reference's own *federated* learning curve rather
# than a full-batch fit: Biscotti's update is the SUM of ~35 clipped minibatch gradients with lr = 1
# (honest.go:405-411), so how far the model oscillates round to round depends on how coherent the
# peers' gradients are -- which the augmentation controls.  The calibration target is the undefended,
# un-noised FedSys run over real MNIST (eval/eval_poison/mnist_poison_30_100.pdf "Federated Learning -
# No Poison", last-10 test error 0.0775; nsdi-eval/scaleup/fed_baseline_100: 0.064).  Measured with
# scripts/robustness_sim.py (3 seeds, 100 peers): rot 6 / shift 1.25 (round 1) gave 0.132 and a clean
# digit-1 error of 0.20; rot 3 / shift 0.6 gives 0.072 and 0.070 (docs/ROBUSTNESS.md).
ROT_DEG = 3.0
SHIFT_PX = 0.6


def standardize_cols(X, mu=None, sigma=None):
    if mu is None:
        mu = X.mean(0)
    if sigma is None:
        sigma = X.std(0)
        sigma = np.where(sigma < 1e-8, 1.0, sigma)
    return (X - mu) / sigma, mu, sigma


# ------------------------------------------------------------------------------------ MNIST
def _digits_8x8():
    """sklearn's bundled 8x8 digits (1797 images, the same arrays as load_digits()), read straight from
    the package's CSV: importing sklearn itself costs ~1.4 s of every run's setup."""
    import gzip
    import importlib.util
    import os

    spec = importlib.util.find_spec("sklearn")   # locates the package without importing it
    path = os.path.join(os.path.dirname(spec.origin), "datasets", "data", "digits.csv.gz") if spec else ""
    if not os.path.exists(path):
        from sklearn.datasets import load_digits

        d = load_digits()
        return d.images, d.target
    with gzip.open(path) as f:
        a = np.loadtxt(f, delimiter=",")
    return a[:, :-1].reshape(-1, 8, 8), a[:, -1].astype(np.int64)


def synthetic_mnist(n_train: int = 60000, n_test: int = 10000, seed: int = 1234):
    """MNIST-shaped digits from sklearn's real 8x8 digits; returns uint8-range float32 arrays."""
    import torch
    import torch.nn.functional as F
    images, target = _digits_8x8()
    base = torch.from_numpy(images.astype(np.float32) / 16.0)  # [1797, 8, 8] in [0, 1]
    labels = torch.from_numpy(target.astype(np.int64))
    g = torch.Generator().manual_seed(seed)
    n = n_train + n_test
    # split source images so train/test digits come from disjoint writers' samples
    perm = torch.randperm(base.shape[0], generator=g)
    n_src_test = base.shape[0] // 6
    src_test, src_train = perm[:n_src_test], perm[n_src_test:]
    pick_train = src_train[torch.randint(0, src_train.numel(), (n_train,), generator=g)]
    pick_test = src_test[torch.randint(0, src_test.numel(), (n_test,), generator=g)]
    pick = torch.cat([pick_train, pick_test])
    out = torch.empty((n, 28 * 28), dtype=torch.float32)
    bs = 8192
    for s in range(0, n, bs):
        idx = pick[s:s + bs]
        m = idx.numel()
        img = base[idx].unsqueeze(1)  # [m,1,8,8]
        img = F.interpolate(img, size=(20, 20), mode="bilinear", align_corners=False)
        canvas = torch.zeros((m, 1, 28, 28))
        canvas[:, :, 4:24, 4:24] = img
        ang = (torch.rand(m, generator=g) - 0.5) * (2 * math.pi * ROT_DEG / 360)
        scl = 1.0 + (torch.rand(m, generator=g) - 0.5) * 0.2
        shift = (torch.rand(m, 2, generator=g) - 0.5) * (2 * SHIFT_PX / 14.0)
        cos, sin = torch.cos(ang) / scl, torch.sin(ang) / scl
        theta = torch.stack([torch.stack([cos, -sin, shift[:, 0]], 1), torch.stack([sin, cos, shift[:, 1]], 1)], 1)
        grid = F.affine_grid(theta, (m, 1, 28, 28), align_corners=False)
        warped = F.grid_sample(canvas, grid, mode="bilinear", padding_mode="zeros", align_corners=False)
        thick = 0.9 + 0.3 * torch.rand(m, 1, 1, 1, generator=g)
        warped = torch.clamp(warped * thick, 0, 1)
        noise = torch.rand(warped.shape, generator=g) * 0.04
        warped = torch.clamp(warped + noise * (warped > 0.05), 0, 1)
        out[s:s + m] = (warped * 255.0).reshape(m, -1)
    y = labels[pick].numpy()
    X = out.numpy()
    return X[:n_train], y[:n_train], X[n_train:], y[n_train:]


def _split(data: np.ndarray, train: bool, cut: float = TRAIN_CUT):
    n = data.shape[0]
    c = int(n * cut)
    part = data[:c] if train else data[c:n]
    return part[:, :-1].astype(np.float32), part[:, -1].astype(np.int64)


@dataclass
class MnistFederation:
    """Per-peer training shards plus the shared evaluation sets of the MNIST federation."""

    shards_X: list = field(default_factory=list)   # per peer: fp32 [n_i, 784] (train part)
    shards_y: list = field(default_factory=list)
    bad_X: np.ndarray | None = None                  # mnist_bad train part (poisoners)
    bad_y: np.ndarray | None = None
    test_X: np.ndarray | None = None                 # last 20% of mnist_test
    test_y: np.ndarray | None = None
    attack_X: np.ndarray | None = None               # last 20% of mnist_digit1
    attack_y: np.ndarray | None = None
    source: str = "synthetic"


def mnist_federation(num_peers: int, seed: int = 1234, data_dir: str | None = None,
                     n_train: int = 60000, n_test: int = 10000) -> MnistFederation:
    fed = MnistFederation()
    if data_dir and (Path(data_dir) / "mnist_test.npy").exists():
        d = Path(data_dir)
        fed.source = f"npy:{d}"
        for i in range(num_peers):
            X, y = _split(np.load(d / f"mnist{i}.npy"), True)
            fed.shards_X.append(X)
            fed.shards_y.append(y)
        fed.test_X, fed.test_y = _split(np.load(d / "mnist_test.npy"), False)
        fed.attack_X, fed.attack_y = _split(np.load(d / "mnist_digit1.npy"), False)
        fed.bad_X, fed.bad_y = _split(np.load(d / "mnist_bad.npy"), True)
        return fed
    Xtr, ytr, Xte, yte = synthetic_mnist(n_train, n_test, seed)
    Xtr, _, _ = standardize_cols(Xtr.astype(np.float64))
    Xte, _, _ = standardize_cols(Xte.astype(np.float64))
    rng = np.random.default_rng(seed)
    perm = rng.permutation(Xtr.shape[0])
    Xs, ys = Xtr[perm], ytr[perm]
    rows = Xs.shape[0] // num_peers
    for i in range(num_peers):
        sl = np.hstack([Xs[i * rows:(i + 1) * rows], ys[i * rows:(i + 1) * rows, None]])
        X, y = _split(sl, True)
        fed.shards_X.append(X)
        fed.shards_y.append(y)
    test = np.hstack([Xte, yte[:, None]])
    fed.test_X, fed.test_y = _split(test, False)
    d1 = np.hstack([Xtr[ytr == 1], ytr[ytr == 1][:, None]])   # mnist_digit1 (train rows, standardized)
    fed.attack_X, fed.attack_y = _split(d1, False)
    bad = d1.copy()
    bad[:, -1] = 7                                            # generate_poisoned
    fed.bad_X, fed.bad_y = _split(bad, True)
    return fed


# ------------------------------------------------------------------------------------ creditcard
@dataclass
class CreditData:
    X: np.ndarray        # [n, 25] standardized + bias (train split, 70%)
    y: np.ndarray        # +-1
    Xvalid: np.ndarray
    yvalid: np.ndarray


def creditcard(path: str | os.PathLike | None = None) -> CreditData:
    """``ML/code/utils.py:load_dataset('creditcard')`` (:88-121): drop the text row and the ID
    column, keep the label column as a feature (quirk Q3), 70/30 split, standardize, add bias."""
    import pandas as pd

    df = pd.read_csv(path or FILES / "creditcard.csv")
    nn, dd = df.shape
    credit = df.iloc[1:nn, 1:dd].values
    nn, dd = credit.shape
    datay = credit[:, dd - 1].astype(int)
    datay[datay == 0] = -1
    data = credit.astype(float)
    split = int(nn * 0.70)
    X, y = data[:split], datay[:split]
    Xv, yv = data[split:nn - 1], datay[split:nn - 1]
    X, mu, sigma = standardize_cols(X)
    Xv, _, _ = standardize_cols(Xv, mu, sigma)
    X = np.hstack([np.ones((X.shape[0], 1)), X])
    Xv = np.hstack([np.ones((Xv.shape[0], 1)), Xv])
    return CreditData(X, y.astype(np.float64), Xv, yv.astype(np.float64))


def credit_poisoned(cd: CreditData) -> CreditData:
    """``creditbad`` analogue (the reference ships a pre-made creditbad.csv): labels flipped."""
    return CreditData(cd.X.copy(), -cd.y, cd.Xvalid, cd.yvalid)


def synthetic_images(n: int, shape: tuple, n_classes: int, seed: int = 0, noise: float = 0.6):
    """Class-conditional synthetic images for the LFW / CIFAR sandboxes (their files are not in the
    reference either): each class is a smooth random prototype; samples are the prototype under a
    random brightness change plus pixel noise.  Returns float32 [n, prod(shape)] and int64 labels."""
    import torch
    import torch.nn.functional as F

    g = torch.Generator().manual_seed(seed)
    c, h, w = shape
    coarse = torch.rand((n_classes, c, max(2, h // 8), max(2, w // 8)), generator=g)
    protos = F.interpolate(coarse, size=(h, w), mode="bilinear", align_corners=False)
    y = torch.randint(0, n_classes, (n,), generator=g)
    gain = 0.8 + 0.4 * torch.rand((n, 1, 1, 1), generator=g)
    X = protos[y] * gain + noise * torch.randn((n, c, h, w), generator=g)
    return X.reshape(n, -1).numpy().astype(np.float32), y.numpy()


# ------------------------------------------------------------------------------------ LFW
LFW_SHAPE = (3, 62, 47)    # lfw_dataset.py: "batch shape for input x is (62, 47, 3)"
LFW_CLASSES = 2            # parse_lfw_maleness.py labels maleness (1 male / 0 female)


def lfw_federation(num_peers: int, seed: int = 1234, n_total: int = 5985) -> MnistFederation:
    """LFW-maleness-shaped federation for the ledger path (the reference's lfw pipeline,
    ML/Pytorch/data/lfw/parse_lfw_maleness.py + lfw_dataset.py).  The faces come from
    sklearn.fetch_lfw_people, which needs the network, so the images are synthetic class-conditional
    62x47x3 faces (synthetic_images) in [0, 1]; 75% train split into per-peer shards, the rest is
    the test set.  The "attack" set is the test faces of class 1 (a 1 -> 0 label flip is the
    binary analogue of the reference's 1 -> 7 poisoning); the poisoners' data is every class-1 train
    face relabelled 0."""
    X, y = synthetic_images(n_total, LFW_SHAPE, LFW_CLASSES, seed=seed, noise=0.9)
    X = np.clip(0.5 + 0.25 * X, 0.0, 1.0).astype(np.float32)
    cut = int(n_total * 0.75)
    fed = MnistFederation(source="synthetic-lfw")
    Xtr, ytr, Xte, yte = X[:cut], y[:cut], X[cut:], y[cut:]
    rows = max(1, Xtr.shape[0] // num_peers)
    for i in range(num_peers):
        lo = (i * rows) % max(1, Xtr.shape[0] - rows + 1)
        fed.shards_X.append(Xtr[lo:lo + rows])
        fed.shards_y.append(ytr[lo:lo + rows].astype(np.int64))
    fed.test_X, fed.test_y = Xte, yte.astype(np.int64)
    ones = yte == 1
    fed.attack_X, fed.attack_y = Xte[ones], yte[ones].astype(np.int64)
    tr1 = ytr == 1
    fed.bad_X, fed.bad_y = Xtr[tr1], np.zeros(int(tr1.sum()), np.int64)
    return fed


def dataset_dims(name: str) -> tuple[int, int, int]:
    """(num_params, num_features, num_classes) of the Biscotti model, SoftmaxModel(features, classes)
    (client_obj.py:20-29 builds a SoftmaxModel for every torch dataset).  mnist 784x10 = 7850 as in
    ML/Pytorch/datasets.py:22-52.  lfw: 8742 features x 2 maleness classes = 17486 -- the reference's
    own lfw numbers are inconsistent (get_num_params 18254 is its LFW CNN's count, get_num_classes 12
    does not match the maleness labels its partitioner writes), so the ledger runs the softmax on the
    labels the data actually has."""
    return {"mnist": (7850, 784, 10), "lfw": (8742 * LFW_CLASSES + LFW_CLASSES, 8742, LFW_CLASSES),
            "creditcard": (25, 25, 2)}[name]
