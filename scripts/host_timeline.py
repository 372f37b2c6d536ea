"""Host-side timeline of engine rounds: every PhaseTimer phase with its start/end (us from the
round's first phase), nested phases included, for a few steady-state rounds of the headline config.

    python scripts/host_timeline.py [--rounds 3] [--warm 20] [--set field=value ...] [--emulate-world N]
"""
import argparse
import dataclasses
import json
import os
import sys
import time
from contextlib import contextmanager

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd.parallel.comm import Comm  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402
from biscotti_amd.protocol.engine import BiscottiEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--wrap", default="", help="comma-separated engine methods (or task./crypto. methods) timed as events")
    ap.add_argument("--fsm-proxy", action="store_true", help="time every native RoundFSM call as an event (@fsm.name)")
    ap.add_argument("--emulate-world", type=int, default=0, help="rank 0 of an N-rank job (bench.py --emulate-world)")
    a = ap.parse_args()
    comm = Comm.emulated(a.emulate_world) if a.emulate_world > 1 else Comm.init()
    torch.set_num_threads(min(4, torch.get_num_threads()))
    kw = dict(num_nodes=100, seed=0, max_iterations=10**9, host_threads=16)
    types = {f.name: f.type for f in dataclasses.fields(RunConfig)}
    for item in a.set:
        k, v = item.split("=", 1)
        cur = getattr(RunConfig, k)
        kw[k] = (v.lower() in ("1", "true")) if isinstance(cur, bool) else type(cur)(v)
    eng = BiscottiEngine(RunConfig(**kw), comm)
    events = []
    jobs = []   # (kind, submit time, job): the native VRF / signature batches of the round
    R = eng.R

    class Spy:
        def __getattr__(self, k):
            return getattr(R, k)

        def vrf_prove_batch_async(self, *a, **kw):
            j = R.vrf_prove_batch_async(*a, **kw)
            jobs.append(("vrf%d" % len(a[0]), time.perf_counter(), j))
            return j

        def vrf_prove_set_async(self, *a, **kw):   # the early VRF outputs (head._early_vrf_submit)
            j = R.vrf_prove_set_async(*a, **kw)
            jobs.append(("vrfset", time.perf_counter(), j))
            return j
    eng.R = Spy()
    timer = eng.timer
    orig = timer.phase

    @contextmanager
    def phase(name):
        s = time.perf_counter()
        with orig(name):
            yield
        events.append((name, s, time.perf_counter()))
    timer.phase = phase

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def w(*a, **kw):
            s = time.perf_counter()
            try:
                return f(*a, **kw)
            finally:
                events.append(("@" + label, s, time.perf_counter()))
        setattr(obj, name, w)
    for m in filter(None, a.wrap.split(",")):
        if m.startswith("task."):
            wrap(eng.task, m[5:], m)
        elif m.startswith("crypto."):
            wrap(eng.crypto, m[7:], m)
        elif m.startswith("fsm."):
            wrap(eng.fsm, m[4:], m)
        elif m.startswith("native."):
            wrap(eng._native, m[7:], m)
        elif m.startswith("mod:"):   # mod:package.module.function (a module-level name the engine calls)
            import importlib
            mod, fn = m[4:].rsplit(".", 1)
            wrap(importlib.import_module(mod), fn, m[4:])
        else:
            wrap(eng, m, m)
    if a.fsm_proxy:   # pybind methods cannot be patched: the engine's FSM behind a timing proxy instead
        class FsmProxy:
            def __init__(self, o):
                object.__setattr__(self, "_o", o)

            def __getattr__(self, k):
                v = getattr(self._o, k)
                if not callable(v):
                    return v

                def f(*args, **kw):
                    s = time.perf_counter()
                    try:
                        return v(*args, **kw)
                    finally:
                        events.append(("@fsm." + k, s, time.perf_counter()))
                return f
        eng.fsm = FsmProxy(eng.fsm)
    for _ in range(a.warm):
        eng.run_round()
    torch.cuda.synchronize()
    out = []
    for _ in range(a.rounds):
        events.clear()
        jobs.clear()
        t0 = time.perf_counter()
        eng.run_round()
        rows = sorted(events, key=lambda e: e[1])
        t1 = time.perf_counter()
        time.sleep(0.01)   # let this round's jobs finish before reading their timings
        js = []
        for kind, ts, j in jobs:
            j.betas()
            q, run = j.timing_us()
            js.append((kind, round(1e6 * (ts - t0), 1), round(q, 1), round(run, 1)))
        out.append({"wall_us": round(1e6 * (t1 - t0), 1),
                    "phases": [(n, round(1e6 * (s - t0), 1), round(1e6 * (e - s), 1)) for n, s, e in rows],
                    "jobs (kind, submit_us, queued_us, run_us)": js})
        for _ in range(3):   # steady state again after the pause
            eng.run_round()
    print(json.dumps(out, indent=0))
    eng.close()


if __name__ == "__main__":
    main()
