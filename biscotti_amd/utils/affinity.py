"""Host-thread placement next to the GPU.

The round is host-bound: one Python thread runs the protocol's critical path while the native pool
computes VRF outputs and signatures.  On a two-socket host (2 x 64 cores, SMT) the scheduler otherwise
moves that thread across sockets and onto SMT siblings of busy pool threads.  `pin_round_threads` puts
the calling (round) thread on a physical core of the GPU's own NUMA node and the native workers on
other physical cores of that node, within the job's CPU quota.  Only one rank per node is pinned (with
several local ranks each rank would need its own slice; they keep the scheduler's placement).
"""
from __future__ import annotations

import os


def _cpulist(text: str) -> list[int]:
    out: list[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_local_cpus(device_index: int) -> list[int]:
    """CPUs of the GPU's NUMA node (sysfs local_cpulist of its PCI function), [] if unknown."""
    import torch

    p = torch.cuda.get_device_properties(device_index)
    bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            return _cpulist(f.read())
    except OSError:
        return []


def physical_cores(cpus: list[int]) -> list[int]:
    """One CPU per physical core (the lowest SMT sibling present), in order."""
    seen, out = set(), []
    for c in sorted(cpus):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                key = min(_cpulist(f.read()))
        except OSError:
            key = c
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def pin_round_threads(device_index: int, ncpus: int, rt) -> dict | None:
    """Pin the calling thread to one physical core next to the GPU and the native workers to the next
    ncpus - 1 cores.  Returns the placement, or None when not applicable (unknown topology, several
    local ranks, or not asked for with BISCOTTI_PIN=1: an A/B on the 1-GPU box measured no difference,
    1.42 vs 1.43 ms/round over 5 runs each)."""
    if os.environ.get("BISCOTTI_PIN", "0") != "1" or not hasattr(os, "sched_setaffinity"):
        return None
    if int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > 1:
        return None
    allowed = os.sched_getaffinity(0)
    local = [c for c in gpu_local_cpus(device_index) if c in allowed]
    cores = physical_cores(local)
    if len(cores) < 4:
        return None
    n = max(2, min(ncpus, len(cores)))
    main, workers = cores[0], cores[1:n]
    rt.set_worker_cpus(workers)
    os.sched_setaffinity(0, {main})
    return {"main": main, "workers": workers}
