"""Host-side cost (us per call) of the small PyTorch / HIP operations a round issues."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from biscotti_amd.utils import h2d  # noqa: E402
from biscotti_amd.utils import streams as S  # noqa: E402


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return round(dt / n * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(70 * 7850, device=dev)
    idx = list(range(70))
    arr = np.arange(3000, dtype=np.int32)
    s = torch.cuda.Stream()
    res = {
        "h2d_list70": per_call(lambda: h2d(idx, torch.int32, dev)),
        "h2d_np3000": per_call(lambda: h2d(arr, torch.int32, dev)),
        "h2d_list70_pin_memory": per_call(lambda: torch.as_tensor(idx, dtype=torch.int32).pin_memory().to(
            dev, non_blocking=True)),
        "streams.current": per_call(S.current),
        "streams.raw": per_call(S.raw),
        "streams.wait": per_call(lambda: S.wait(s, S.current())),
        "streams.use": per_call(lambda: S.use(s).__enter__() and None or S.use(torch.cuda.default_stream()).__enter__()),
        "stream_ctx": per_call(lambda: torch.cuda.stream(s).__enter__()),
        "torch_empty": per_call(lambda: torch.empty((70, 24), dtype=torch.int32, device=dev)),
        "torch_zeros": per_call(lambda: torch.zeros((70, 24), dtype=torch.int32, device=dev)),
        "event_record": per_call(lambda: torch.cuda.Event().record()),
        "current_stream": per_call(lambda: torch.cuda.current_stream()),
        "wait_stream": per_call(lambda: s.wait_stream(torch.cuda.current_stream())),
        "record_stream": per_call(lambda: x.record_stream(s)),
        "elementwise_add": per_call(lambda: x.add_(1.0)),
        "index_select": per_call(lambda: x.view(70, 7850).index_select(0, torch.arange(10, device=dev))),
        "pinned_empty": per_call(lambda: torch.empty((70, 24), dtype=torch.int32, pin_memory=True)),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
