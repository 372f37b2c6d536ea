"""Host cost of reading a GPU-written pinned buffer (the recovery writes W_new into pinned memory; the block
build then reads it) vs pageable memory, and the block build from each."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from biscotti_amd.native import rt  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402


def T(f, n=200):
    for _ in range(5):
        f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t) / n * 1e6


dev = torch.device("cuda:0")
d = 7850
src = torch.randn(d, dtype=torch.float64, device=dev)
pin = torch.empty(d, dtype=torch.float64, pin_memory=True)
pag = np.random.randn(d)
R = rt()
fsm = R.RoundFSM(RunConfig(dataset="mnist", num_nodes=100).protocol(R), d)
fsm.begin_round([1] * 100)
nodes, cs = list(range(35)), [bytes(64)] * 35
out = {}


def gpu_write():
    pin.copy_(src, non_blocking=True)
    torch.cuda.synchronize()


def after_write(f):
    def g():
        gpu_write()
        t = time.perf_counter()
        f()
        return time.perf_counter() - t
    return g


def timed_after_write(f, n=200):
    ts = [after_write(f)() for _ in range(n)]
    return float(np.median(ts) * 1e6)


pv = pin.numpy()
out["read_pinned_after_gpu_write_us"] = timed_after_write(lambda: pv.sum())
out["copy_pinned_after_gpu_write_us"] = timed_after_write(lambda: pv.copy())
out["read_pinned_cached_us"] = T(lambda: pv.sum())
out["read_pageable_us"] = T(lambda: pag.sum())
out["block_from_pinned_after_gpu_write_us"] = timed_after_write(lambda: fsm.make_secagg_block(pv, nodes, cs, 1))
out["block_from_pageable_us"] = T(lambda: fsm.make_secagg_block(pag, nodes, cs, 1))
print(json.dumps(out))
