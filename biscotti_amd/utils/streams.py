"""Low-overhead HIP stream helpers for the round's host thread.

A round is host-bound (~200 small launches, copies and stream operations), and the public
``torch.cuda`` stream API costs more than the work it queues: ``current_stream()`` resolves the
device through several Python layers and builds a new ``Stream`` object every call (~3 µs),
``Stream.wait_stream`` creates and destroys an event each time (~10 µs), ``torch.cuda.stream(s)``
does both on entry and exit.  These helpers go straight to the ``torch._C`` stream calls, cache
the ``Stream`` objects (a process has a handful) and reuse one event per waiting stream pair.
(``scripts/host_op_costs.py`` measures the individual costs; ``scripts/count_ops.py`` counts them
per round.)
"""
from __future__ import annotations

import torch

_C = torch._C
_streams: dict = {}
_events: dict = {}


def current() -> torch.cuda.Stream:
    """The current stream of the current device (same object as ``torch.cuda.current_stream()``
    would describe, cached)."""
    key = _C._cuda_getCurrentStream(_C._cuda_getDevice())
    s = _streams.get(key)
    if s is None:
        s = _streams[key] = torch.cuda.Stream(stream_id=key[0], device_index=key[1], device_type=key[2])
    return s


def raw() -> int:
    """hipStream_t of the current stream (for the native launchers)."""
    return _C._cuda_getCurrentRawStream(_C._cuda_getDevice())


class use:
    """``with use(s):`` makes `s` the current stream (like ``torch.cuda.stream(s)``, same device)."""

    __slots__ = ("s", "prev")

    def __init__(self, s: torch.cuda.Stream):
        self.s = s

    def __enter__(self):
        self.prev = _C._cuda_getCurrentStream(_C._cuda_getDevice())
        s = self.s
        _C._cuda_setStream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *exc):
        p = self.prev
        _C._cuda_setStream(stream_id=p[0], device_index=p[1], device_type=p[2])
        return False


def wait(dst: torch.cuda.Stream, src: torch.cuda.Stream) -> None:
    """`dst` waits (on the device) for everything queued on `src` so far -- ``dst.wait_stream(src)``
    with a reused event: a stream wait binds to the event's latest record at enqueue time, so
    re-recording it for the next wait does not disturb waits already queued."""
    if dst.stream_id == src.stream_id and dst.device_type == src.device_type:
        return
    key = (dst.cuda_stream, src.cuda_stream)
    ev = _events.get(key)
    if ev is None:
        ev = _events[key] = torch.cuda.Event()
    ev.record(src)
    dst.wait_event(ev)


SPIN_S = 2e-4   # host waits spin this long, then poll with short sleeps (set_spin)


def set_spin(seconds: float) -> None:
    """How long host waits spin before they poll with sleeps -- these and the native round's waits
    (bsc_set_host_spin_ns).  The engine spins long with one rank per process (a sleeping thread wakes
    late; the GPU's one host thread has nothing else to do) and briefly with several (ranks sharing the
    CPU quota)."""
    global SPIN_S
    SPIN_S = float(seconds)
    try:
        from ..native import hip

        hip().bsc_set_host_spin_ns(int(seconds * 1e9))
    except (ImportError, OSError, AttributeError):
        pass


def host_wait(ev) -> None:
    """Wait on the host for a torch event: spin (the round's typical waits are tens to a few hundred us,
    and a sleeping thread wakes late), then poll with ~50 us sleeps, so a long wait -- ranks sharing a GPU,
    a collective waiting for a slow rank -- does not burn a core (docs/PERF.md, multi-rank host CPU)."""
    if ev.query():
        return
    import time

    t0 = time.perf_counter()
    while not ev.query():
        if time.perf_counter() - t0 > SPIN_S:
            time.sleep(5e-5)


def record(stream: torch.cuda.Stream | None = None) -> torch.cuda.Event:
    """A fresh event recorded on `stream` (default: the current stream), for host-side waits."""
    ev = torch.cuda.Event()
    ev.record(stream if stream is not None else current())
    return ev


# ---------------------------------------------------------------------------- cross-stream lifetimes
# A tensor used on a stream other than the one it was allocated on must not be reused before that
# stream is done with it.  `Tensor.record_stream` does that with an event recorded at every free
# and queried at later allocations (~14 per round here, and every allocation then pays the
# queries).  A round's cross-stream work is complete two rounds later (each stream's work of round
# r is waited on by the host through a read-back of round r or r+1), so the engine instead keeps such
# tensors referenced for two rounds: hold() during the round, rotate_holds() at its end.
_holds: list = [[]]


def hold(*tensors) -> None:
    _holds[-1].extend(tensors)


def rotate_holds(depth: int = 2) -> None:
    _holds.append([])
    while len(_holds) > depth + 1:
        _holds.pop(0)


def clear_holds() -> None:
    _holds[:] = [[]]
