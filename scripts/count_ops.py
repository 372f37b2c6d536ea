"""Count the PyTorch ops and stream/event calls one engine round issues from the host thread
(each costs ~2-15 us of Python + dispatcher time; see scripts/host_op_costs.py).

    python scripts/count_ops.py [--rounds 10] [--config-set k=v ...]
"""
import argparse
import collections
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from biscotti_amd.parallel.comm import Comm  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402
from biscotti_amd.protocol.engine import BiscottiEngine  # noqa: E402

MAIN = threading.get_ident()
counts = collections.Counter()


class Count(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        if threading.get_ident() == MAIN:
            counts[str(func.overloadpacket.__name__)] += 1
        return func(*args, **(kwargs or {}))


def wrap(obj, name, label):
    f = getattr(obj, name)

    def w(*a, **k):
        if threading.get_ident() == MAIN:
            counts[label] += 1
        return f(*a, **k)
    setattr(obj, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    a = ap.parse_args()
    comm = Comm.init()
    wrap(torch.cuda.Event, "record", "Event.record")
    wrap(torch.cuda.Event, "synchronize", "Event.synchronize")
    wrap(torch.cuda.Stream, "wait_stream", "Stream.wait_stream")
    wrap(torch.cuda.Stream, "wait_event", "Stream.wait_event")
    wrap(torch.cuda, "current_stream", "current_stream")
    wrap(torch.cuda, "stream", "cuda.stream ctx")
    eng = BiscottiEngine(RunConfig(num_nodes=100, seed=0, max_iterations=10**9, host_threads=16, phase_sync=False),
                         comm)
    for _ in range(5):
        eng.run_round()
    torch.cuda.synchronize()
    with Count():
        for _ in range(a.rounds):
            eng.run_round()
    torch.cuda.synchronize()
    per = {k: round(v / a.rounds, 1) for k, v in counts.most_common()}
    print(json.dumps({"ops_per_round_total": round(sum(counts.values()) / a.rounds, 1), "by_op": per}))
    eng.close()


if __name__ == "__main__":
    main()
