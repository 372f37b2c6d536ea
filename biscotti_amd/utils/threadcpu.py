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


def _cgroup_dirs() -> list:
    """This process's cgroup-v2 directory and its ancestors up to /sys/fs/cgroup (a CFS quota may sit on
    any of them: on the GPU box the process's own group has no cpu controller, its parent has cpu.max)."""
    out = []
    try:
        rel = open("/proc/self/cgroup").read().strip().split("\n")[0].split(":", 2)[2]
    except (OSError, IndexError):
        rel = ""
    parts = [p for p in rel.split("/") if p]
    while True:
        out.append("/sys/fs/cgroup" + "".join("/" + p for p in parts))
        if not parts:
            return out
        parts.pop()


def cgroup_cpu_stat() -> dict:
    """CPU counters of the nearest cgroup that throttles this process: nr_periods, nr_throttled,
    throttled_usec (cgroup v2 cpu.stat, or v1 cpu,cpuacct).  A CFS quota (cpu.max) that the job's threads
    exhaust inside a 100 ms period stops EVERY thread of the group until the period ends -- a 10-100 ms
    stall of whichever rank holds a collective.  Empty when no such counters exist."""
    cands = [d + "/cpu.stat" for d in _cgroup_dirs()] + ["/sys/fs/cgroup/cpu/cpu.stat",
                                                         "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"]
    for p in cands:
        out = {}
        try:
            with open(p) as f:
                for ln in f:
                    k, _, v = ln.partition(" ")
                    if k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec"):
                        out[k] = int(v)
                    elif k == "throttled_time":   # v1: nanoseconds
                        out["throttled_usec"] = int(v) // 1000
        except (OSError, ValueError):
            continue
        if "nr_throttled" in out:
            return out
    return {}


def cgroup_delta(a: dict, b: dict) -> dict:
    return {k: b[k] - a.get(k, 0) for k in b}


def cpu_quota() -> float | None:
    """CPUs the tightest CFS quota over this process's cgroup and its ancestors allows (cpu.max), or None
    when unlimited / unknown."""
    best = None
    for d in _cgroup_dirs():
        try:
            q, per = open(d + "/cpu.max").read().split()[:2]
        except (OSError, ValueError):
            continue
        if q != "max":
            c = int(q) / int(per)
            best = c if best is None else min(best, c)
    if best is not None:
        return best
    try:   # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def pool_threads(local_ranks: int, world: int, cpus: float | None = None) -> int:
    """Native crypto pool size per rank so that every thread the node's local ranks keep busy fits the CPUs
    the job may use (the CFS quota, else the affinity mask): per rank, the round's host thread and the HIP
    runtime's threads take one CPU each and, with several ranks, RCCL's proxy / service threads two more
    (measured 1.2-2 cores per rank on the RCCL rehearsal, docs/PERF.md); the pool gets the rest, 2..16.  A
    pool that overshoots the quota gets every thread of the job throttled for the rest of the CFS period --
    the 50-280 ms multi-rank stalls of round 4."""
    if cpus is None:
        aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 16)
        q = cpu_quota()
        cpus = aff if q is None else min(aff, q)
    local = max(1, int(local_ranks))
    reserve = 2 + (2 if world > 1 else 0)
    return int(max(2, min(16, (int(cpus) - local * reserve) // local)))


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
