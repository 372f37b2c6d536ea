"""Per-thread CPU attribution of this process (Linux /proc): which threads burn the host CPU of a rank --
the round's Python thread, the native crypto pool (``bsc-pool``) and job threads (``bsc-job``), the HIP
runtime, RCCL / gloo progress threads, OpenMP workers.  bench.py reports the CPU per thread group over
the timed rounds, per rank, so a multi-GPU run's host cost can be attributed (docs/PERF.md)."""
from __future__ import annotations

import os

_TICK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
_LABELS: dict = {}   # tid -> label of helper threads that inherited the process name (mark_new_threads)


def mark_new_threads(label: str) -> None:
    """Label every thread of this process that has no label yet and is not the main thread: called right
    after a library starts its helper threads (the HIP runtime at device init, RCCL / gloo at the first
    collective), so their CPU is attributed to that library instead of to the process name they inherit."""
    main = str(os.getpid())
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return
    for tid in tids:
        if tid != main and tid not in _LABELS:
            _LABELS[tid] = label


def snapshot() -> dict:
    """tid -> (thread name, CPU seconds) of every live thread of this process."""
    out = {}
    base = "/proc/self/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    main = str(os.getpid())
    for tid in tids:
        try:
            with open(f"{base}/{tid}/stat") as f:
                st = f.read()
            with open(f"{base}/{tid}/comm") as f:
                name = f.read().strip()
        except OSError:
            continue
        # fields after the ")" that closes the (possibly space-containing) name: utime, stime are 14, 15
        rest = st[st.rindex(")") + 2:].split()
        # the process's main thread (the round's host thread) apart from helper threads that inherited its
        # name (HIP runtime, RCCL proxy / socket threads, OpenMP workers)
        if tid == main:
            name = "main"
        elif tid in _LABELS and name in ("python", "python3", "pt_main_thread"):
            name = _LABELS[tid]
        out[tid] = (name, (int(rest[11]) + int(rest[12])) / _TICK)
    return out


def _group(name: str) -> str:
    """Thread groups: names are truncated to 15 characters and often numbered (``bsc-pool``,
    ``python``/``pt_main_thread``, ``HIP ...``, ``NCCL``/``rccl`` threads, ``gloo`` ...)."""
    n = name.rstrip("0123456789:-_ ")
    return n or name


def delta_by_group(a: dict, b: dict) -> dict:
    """CPU seconds per thread group between two snapshots (threads born in between count from 0)."""
    acc: dict = {}
    for tid, (name, t1) in b.items():
        t0 = a.get(tid, (name, 0.0))[1]
        g = _group(name)
        acc[g] = acc.get(g, 0.0) + max(0.0, t1 - t0)
    return dict(sorted(acc.items(), key=lambda kv: -kv[1]))
