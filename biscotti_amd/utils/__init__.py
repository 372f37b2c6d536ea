"""Logging in the reference's format and structured phase tracing.

Reference logging (DistSys/main.go:136-137): ``log.New(os.Stderr, "[peer] ",
log.Lshortfile|log.LUTC|log.Lmicroseconds)`` -> ``[peer] 21:03:12.123456 file.go:151: msg``.
The eval parsers key on lines such as ``"<id>:Train Error is %.5f in Iteration %d"``
(honest.go:151) and ``"<id>:Attack Rate is %.5f in Iteration %d"`` (:153); those are kept
verbatim.  Phase timings go to JSON lines (one record per round) instead of being reconstructed
from marker lines.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

import numpy as np


class _GoFormatter(logging.Formatter):
    def __init__(self, prefix: str):
        super().__init__()
        self.prefix = prefix

    def format(self, record: logging.LogRecord) -> str:
        t = time.gmtime(record.created)
        us = int((record.created % 1) * 1e6)
        return (f"{self.prefix}{t.tm_hour:02d}:{t.tm_min:02d}:{t.tm_sec:02d}.{us:06d} "
                f"{os.path.basename(record.pathname)}:{record.lineno}: {record.getMessage()}")


class _BatchingHandler(logging.Handler):
    """Writes formatted records in batches: one write + flush per `max_lines` records or
    `max_delay` seconds instead of one per record.  A round logs two lines; flushing each one to
    a pipe cost ~0.1 ms of the round's host critical path.  Flushed at exit and by flush()."""

    def __init__(self, stream=None, path: str | None = None, max_lines: int = 64, max_delay: float = 0.25):
        super().__init__()
        import atexit

        self.stream = open(path, "a") if path else (stream or sys.stderr)
        self.lines: list[str] = []
        self.max_lines, self.max_delay = max_lines, max_delay
        self.t_last = time.monotonic()
        atexit.register(self.flush)

    def emit(self, record: logging.LogRecord) -> None:
        try:
            self.lines.append(self.format(record))
            if len(self.lines) >= self.max_lines or time.monotonic() - self.t_last > self.max_delay:
                self.flush()
        except Exception:  # pragma: no cover
            self.handleError(record)

    def flush(self) -> None:
        if self.lines:
            out, self.lines = "\n".join(self.lines) + "\n", []
            try:
                self.stream.write(out)
                self.stream.flush()
            except ValueError:  # stream closed at interpreter teardown
                pass
        self.t_last = time.monotonic()


def fast_info(lg: logging.Logger, where: str, msg: str) -> None:
    """One INFO line in the reference's format without the logging machinery (LogRecord, findCaller's
    stack walk, Formatter): the per-round Train Error / Attack Rate lines cost ~15 us each through
    logging.info on the round's critical host thread.  `where` is the "file.py:line" the line names.
    Falls back to logging for handlers other than the batching one."""
    if not lg.isEnabledFor(logging.INFO):
        return
    h = lg.handlers[0] if lg.handlers else None
    if not isinstance(h, _BatchingHandler) or not isinstance(h.formatter, _GoFormatter):
        lg.info("%s", msg)
        return
    now = time.time()
    t = time.gmtime(now)
    h.lines.append(f"{h.formatter.prefix}{t.tm_hour:02d}:{t.tm_min:02d}:{t.tm_sec:02d}.{int((now % 1) * 1e6):06d} "
                   f"{where}: {msg}")
    if len(h.lines) >= h.max_lines or time.monotonic() - h.t_last > h.max_delay:
        h.flush()


def fast_info_at(lg: logging.Logger, where: str, msg: str, when: float) -> None:
    """fast_info with the line's timestamp given (wall-clock seconds): lines written after the fact for
    instants recorded earlier in the round (protocol/golog.py)."""
    if not lg.isEnabledFor(logging.INFO):
        return
    h = lg.handlers[0] if lg.handlers else None
    if not isinstance(h, _BatchingHandler) or not isinstance(h.formatter, _GoFormatter):
        lg.info("%s", msg)
        return
    t = time.gmtime(when)
    h.lines.append(f"{h.formatter.prefix}{t.tm_hour:02d}:{t.tm_min:02d}:{t.tm_sec:02d}.{int((when % 1) * 1e6):06d} "
                   f"{where}: {msg}")
    if len(h.lines) >= h.max_lines or time.monotonic() - h.t_last > h.max_delay:
        h.flush()


def flush_logs(lg: logging.Logger) -> None:
    for h in lg.handlers:
        h.flush()


def get_logger(name: str = "peer", path: str | None = None, level=logging.INFO) -> logging.Logger:
    lg = logging.getLogger(f"biscotti.{name}.{path or 'stderr'}")
    if not lg.handlers:
        h = _BatchingHandler(path=path) if path else _BatchingHandler(sys.stderr)
        h.setFormatter(_GoFormatter(f"[{name}] "))
        lg.addHandler(h)
        lg.propagate = False
    lg.setLevel(level)
    return lg


class _Phase:
    """One timed phase (a plain context manager: a generator-based one costs a few us per use, and
    a round enters ~25 phases on its critical host thread)."""

    __slots__ = ("timer", "name", "s")

    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        if self.timer.sync:
            self.timer.sync()
        self.s = time.perf_counter()
        return self

    def __exit__(self, *exc):
        tm = self.timer
        if tm.sync:
            tm.sync()
        t = tm.t
        t[self.name] = t.get(self.name, 0.0) + time.perf_counter() - self.s
        return False


class PhaseTimer:
    """Accumulates wall time per protocol phase; ``sync`` makes GPU work visible to the clock."""

    stamps = None

    def __init__(self, sync=None):
        self.t: dict[str, float] = {}
        self.sync = sync

    def phase(self, name: str) -> _Phase:
        return _Phase(self, name)

    def reset(self) -> dict[str, float]:
        out, self.t = self.t, {}
        return out


class _StampedPhase(_Phase):
    __slots__ = ("w",)

    def __enter__(self):
        super().__enter__()
        self.w = time.time() - (time.perf_counter() - self.s)   # wall clock of the same instant
        return self

    def __exit__(self, *exc):
        super().__exit__(*exc)
        end = self.w + (time.perf_counter() - self.s)
        st = self.timer.stamps
        first = st.get(self.name)
        st[self.name] = (first[0] if first else self.w, end)
        return False


class StampedPhaseTimer(PhaseTimer):
    """A PhaseTimer that also keeps each phase's wall-clock (first start, last end) of the current round in
    ``stamps`` (the reference's phase log lines are written from them, protocol/golog.py).  The plain timer
    pays nothing for this."""

    def __init__(self, sync=None):
        super().__init__(sync)
        self.stamps: dict = {}

    def phase(self, name: str) -> _Phase:
        return _StampedPhase(self, name)

    def take_stamps(self) -> dict:
        out, self.stamps = self.stamps, {}
        return out


class JsonlWriter:
    def __init__(self, path: str | None):
        self.f = open(path, "a") if path else None

    def write(self, rec: dict) -> None:
        if self.f:
            self.f.write(json.dumps(rec) + "\n")
            self.f.flush()

    def close(self) -> None:
        if self.f:
            self.f.close()


class _PinnedRing:
    """One pinned staging buffer for the round's small uploads, used as a ring: no pinned
    allocation per upload.  Space is reused only after a device synchronisation at the wrap-around
    (every few hundred rounds at ~20 KB/round), so no in-flight copy is ever overwritten."""

    SIZE = 8 << 20

    def __init__(self):
        import torch

        self.buf = torch.empty((self.SIZE,), dtype=torch.uint8, pin_memory=True)
        self.np = self.buf.numpy()
        self.off = 0

    def _put(self, arr) -> int:
        import torch

        nb = arr.nbytes
        if self.off + nb > self.SIZE:
            torch.cuda.synchronize()
            self.off = 0
        o = self.off
        self.off = (o + nb + 255) & ~255
        self.np[o:o + nb] = arr.reshape(-1).view(np.uint8)
        return o

    def upload(self, arr, dtype, device):
        """Stage `arr` and copy it into a fresh device tensor with ONE bare hipMemcpyAsync on the
        current stream (a framework-level pinned copy also records a host-allocator event per copy,
        ~20 us of host time on this stack)."""
        import torch

        from ..native import hip
        from . import streams as S

        o = self._put(arr)
        out = torch.empty(arr.shape, dtype=dtype, device=device)
        err = hip().bsc_h2d_async(out.data_ptr(), self.buf.data_ptr() + o, arr.nbytes, S.raw())
        if err != 0:
            raise RuntimeError(f"hipMemcpyAsync (h2d) failed with hipError {err}")
        return out


_ring = None
_NP_OF = {}


def h2d(data, dtype, device):
    """Small host -> device upload that does not block the host.

    ``torch.tensor(list, device=cuda)`` copies from pageable memory, which makes the host wait for
    everything already queued on the stream (e.g. a 0.6 ms MSM kernel) before it can continue.  A
    pinned staging buffer + ``non_blocking`` copy is stream-ordered instead: the host moves on and
    keeps launching work.  Uploads up to 1 MiB go through one preallocated pinned ring."""
    import torch

    global _ring
    if torch.device(device).type != "cuda":
        return torch.as_tensor(data, dtype=dtype)
    if not _NP_OF:
        _NP_OF.update({torch.int32: np.int32, torch.int64: np.int64, torch.float32: np.float32,
                       torch.float64: np.float64, torch.uint8: np.uint8})
    npdt = _NP_OF.get(dtype)
    arr = np.ascontiguousarray(data, dtype=npdt) if npdt is not None else None
    if arr is None or arr.nbytes > (1 << 20) or arr.nbytes == 0:
        return torch.as_tensor(data, dtype=dtype).pin_memory().to(device, non_blocking=True)
    if _ring is None:
        _ring = _PinnedRing()
    return _ring.upload(arr, dtype, device)


_PINNED: dict = {}


def pinned(key, shape, dtype, depth: int = 2):
    """A persistent pinned host buffer for read-backs, rotating over `depth` buffers per (key, shape,
    dtype): buffers written by bare copies (d2h_into) must never return to an allocator while a copy
    may be in flight, and a read-back may still be read while the next one is queued."""
    import torch

    k = (key, tuple(shape), dtype)
    ent = _PINNED.get(k)
    if ent is None:
        ent = _PINNED[k] = [[torch.empty(tuple(shape), dtype=dtype, pin_memory=True) for _ in range(depth)], 0]
    bufs, i = ent
    ent[1] = (i + 1) % len(bufs)
    return bufs[i]


def d2h_into(host, t) -> None:
    """Stream-ordered read-back of device tensor `t` into the pinned host tensor `host` (same shape
    and dtype) on the current stream: one bare hipMemcpyAsync (``host.copy_(t, non_blocking=True)``
    also records a host-allocator event, ~20 us of host time per copy on this stack)."""
    from ..native import hip
    from . import streams as S

    assert host.is_pinned() and not host.is_cuda and t.is_cuda and t.is_contiguous() and host.is_contiguous()
    assert host.dtype == t.dtype and host.numel() == t.numel()
    err = hip().bsc_d2h_async(host.data_ptr(), t.data_ptr(), t.numel() * t.element_size(), S.raw())
    if err != 0:
        raise RuntimeError(f"hipMemcpyAsync (d2h) failed with hipError {err}")


def h2d_many(items, device) -> list:
    """Several small uploads in ONE copy: [(data, dtype), ...] -> device tensors (views of one
    buffer).  Each hipMemcpyAsync costs ~20-30 us of host time on this stack, so a phase that needs
    five index tables pays that once."""
    import torch

    global _ring
    if torch.device(device).type != "cuda":
        return [torch.as_tensor(d, dtype=t) for d, t in items]
    if not _NP_OF:
        h2d([0], torch.int32, device)   # fills _NP_OF
    arrs = [np.ascontiguousarray(d, dtype=_NP_OF[t]) for d, t in items]
    offs, o = [], 0
    for a in arrs:
        offs.append(o)
        o = (o + a.nbytes + 15) & ~15
    if o == 0 or o > (1 << 20):
        return [h2d(d, t, device) for d, t in items]
    raw = np.zeros(o, np.uint8)
    for a, of in zip(arrs, offs):
        raw[of:of + a.nbytes] = a.reshape(-1).view(np.uint8)
    if _ring is None:
        _ring = _PinnedRing()
    dev = _ring.upload(raw, torch.uint8, device)
    return [dev[of:of + a.nbytes].view(t).view(a.shape) for a, of, (_, t) in zip(arrs, offs, items)]
