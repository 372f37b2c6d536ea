"""Model zoo (ML/Pytorch/*_model.py) and the batched per-peer learning tasks of the ledger.

* :class:`SoftmaxModel` -- one linear layer, THE Biscotti model (softmax_model.py:7-24)
* :class:`SVMModel`, :class:`MNISTCNNModel`, :class:`LFWCNNModel`, :class:`CIFARCNNModel`
  (svm_model.py, mnist_cnn_model.py, lfw_cnn_model.py, cifar_cnn_model.py) for the sandboxes
* :class:`SoftmaxTask` / :class:`LogisticTask` -- all virtual peers of a rank as batched tensors,
  stepping through the fused gfx950 kernels (ops/ml.py)
"""
from .zoo import CIFARCNNModel, LFWCNNModel, MNISTCNNModel, SoftmaxModel, SVMModel, flatten_grads, flatten_params
from .tasks import LogisticTask, SoftmaxTask, make_task

__all__ = ["SoftmaxModel", "SVMModel", "MNISTCNNModel", "LFWCNNModel", "CIFARCNNModel", "flatten_grads",
           "flatten_params", "SoftmaxTask", "LogisticTask", "make_task"]
