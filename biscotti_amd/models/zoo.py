"""Reference model definitions with the flat-vector interface the ledger uses.

Every model exposes ``reshape(flat) -> list[Tensor]`` (unflatten a parameter/gradient vector in
``named_parameters`` order) like the reference models, plus ``flatten_params`` / ``flatten_grads``
helpers (client.py:56-64,114-121 flatten W then b).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class _Flat(nn.Module):
    def reshape(self, flat) -> list[torch.Tensor]:
        flat = torch.as_tensor(np.asarray(flat), dtype=torch.float32)
        out, o = [], 0
        for p in self.parameters():
            n = p.numel()
            out.append(flat[o:o + n].view_as(p).clone())
            o += n
        return out

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def load_flat(self, flat) -> None:
        for p, t in zip(self.parameters(), self.reshape(flat)):
            p.data = t.to(p.device)


class SoftmaxModel(_Flat):
    """softmax_model.py:7-24 -- logits = x W^T + b; MNIST 784 -> 10 = 7850 parameters."""

    def __init__(self, D_in: int, D_out: int):
        super().__init__()
        self.linear = nn.Linear(D_in, D_out)
        self.D_in, self.D_out = D_in, D_out

    def forward(self, x):
        return self.linear(x.reshape(x.shape[0], self.D_in))


class SVMModel(_Flat):
    """svm_model.py:8-24 -- linear scorer trained with a multi-label margin loss."""

    def __init__(self, D_in: int, D_out: int):
        super().__init__()
        self.linear = nn.Linear(D_in, D_out)
        self.D_in, self.D_out = D_in, D_out

    def forward(self, x):
        return self.linear(x.reshape(x.shape[0], self.D_in))


class MNISTCNNModel(_Flat):
    """mnist_cnn_model.py:7-67 -- Conv(1->16, 5x5, pad 2) + ReLU + Linear(16*32*32? -> 10).

    The reference flattens a 16-channel 28x28 map padded to 32x32 into a 16384-wide linear layer."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 16, kernel_size=5, padding=4)
        self.fc = nn.Linear(16384, 10)

    def forward(self, x):
        x = x.reshape(x.shape[0], 1, 28, 28)
        x = F.relu(self.conv1(x))
        return self.fc(x.reshape(x.shape[0], -1))


class LFWCNNModel(_Flat):
    """lfw_cnn_model.py:8-28, layer for layer: conv3x3 3->18 (pad 1) + ReLU + maxpool 2, conv3x3
    18->36 (pad 1) + ReLU + maxpool 2, fc 5940->2 on 62x47x3 faces (36 x 15 x 11 = 5940).
    18,254 parameters -- the `get_num_params('lfw')` value of ML/Pytorch/datasets.py:22-23."""

    def __init__(self, n_classes: int = 2):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 18, kernel_size=3, stride=1, padding=1)
        self.conv2 = nn.Conv2d(18, 36, kernel_size=3, stride=1, padding=1)
        self.fc1 = nn.Linear(5940, n_classes)

    def forward(self, x):
        x = x.reshape(x.shape[0], 3, 62, 47)
        x = F.max_pool2d(F.relu(self.conv1(x)), kernel_size=2, stride=2)
        x = F.max_pool2d(F.relu(self.conv2(x)), kernel_size=2, stride=2)
        return self.fc1(x.reshape(x.shape[0], -1))


class CIFARCNNModel(_Flat):
    """cifar_cnn_model.py:8-31, layer for layer: conv3x3 3->20 with padding 3 (32x32 -> 36x36) + ReLU
    + maxpool(k=1, identity), fc 25920->10 (20 x 36 x 36 = 25920; the reference's ONE LAYER
    variant).  259,770 parameters."""

    def __init__(self, n_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 20, kernel_size=3, stride=1, padding=3)
        self.fc1 = nn.Linear(25920, n_classes)

    def forward(self, x):
        x = x.reshape(x.shape[0], 3, 32, 32)
        x = F.max_pool2d(F.relu(self.conv1(x)), kernel_size=1, stride=1)
        return self.fc1(x.reshape(x.shape[0], -1))


def flatten_params(model: nn.Module) -> np.ndarray:
    return torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]).double().numpy()


def flatten_grads(model: nn.Module) -> np.ndarray:
    return torch.cat([p.grad.detach().reshape(-1).cpu() for p in model.parameters()]).double().numpy()
