"""Headline benchmark: Biscotti seconds per round (block commit) + final test accuracy,
MNIST softmax regression, 100 peers (BASELINE.json; reference 29.83 s/round at 87.7%).

    python bench.py --gpus N --steps K --warmup W [--config NAME]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Each step is one full protocol round with the reference defaults (3 verifiers, 3 aggregators,
2 noisers, epsilon 2, ns 70%, secure aggregation + Multi-Krum + DP noising on): local SGD of all
workers, BN256 commitments, noise, Krum + Schnorr signatures, Shamir shares with KZG-style
witnesses, miner aggregation, exact recovery, gob+SHA-256 block, evaluation.  Peers are packed as
virtual peers onto the N GPUs (strong scaling: 100 peers regardless of N).  Data: synthetic
MNIST-shaped digits (see biscotti_amd/data), zero-init model as in the reference.

``--config`` selects the other BASELINE.md rows (each compared with its own reference number):
fedsys, poison30, poison50_5v, churn10, scale40/60/80, secagg_off/verification_off/noising_off
(100-peer increments), mnist10_dp1 and credit4 (no published number).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import math
import sys
import time

import torch

BASELINE_S_PER_ROUND = 29.83   # nsdi-eval/scaleup/bis_baseline_100
BASELINE_ACC = 0.877

# name -> (RunConfig overrides, reference s/round or None, reference accuracy or None, extra refs, source)
# Reference accuracies are "last-10-round mean" where the reference only has a plotted curve
# (recovered from its PDF with scripts/extract_reference_curves.py -> profiles/reference_curves.json).
# The reference's 30%/50% poisoning tables (nsdi-eval/credit) are CREDITCARD runs (plot label
# "Validation Error", FedSys at 30% poison reaching err 0.00005 -- impossible for MNIST softmax);
# the MNIST 1->7 poisoning runs are eval/eval_poison (100/200 peers, -po 0.30 -ns 70 -ep 1.0).
PRESETS = {
    "headline": ({}, 29.83, 0.877, {}, "nsdi-eval/scaleup/bis_baseline_100"),
    "fedsys": ({"fedsys": True, "perc_samples": 35, "epsilon": 5.0}, 3.42, 0.9365, {},
               "nsdi-eval/scaleup/fed_baseline_100"),
    # MNIST 1->7 label flip (eval/eval_poison/runEval.sh:9), reference curves from the PDFs
    "poison30": ({"poisoning": 0.3, "epsilon": 1.0}, None, 1 - 0.0853, {"attack_rate": 0.0289},
                 "eval/eval_poison/mnist_poison_30_100{,_AR}.pdf (Biscotti - 30% Poison, last-10 mean)"),
    "poison30_200": ({"num_nodes": 200, "poisoning": 0.3, "epsilon": 1.0}, None, 1 - 0.0870, {"attack_rate": 0.0700},
                     "eval/eval_poison/mnist_poison_30_200{,_AR}.pdf (Biscotti - 30% Poison, last-10 mean)"),
    "fedsys_poison30": ({"fedsys": True, "perc_samples": 35, "poisoning": 0.3}, None, 1 - 0.1933,
                        {"attack_rate": 0.734},
                        "eval/eval_poison/mnist_poison_30_100{,_AR}.pdf (Federated Learning - 30% Poison)"),
    # creditcard label-flip poisoning, 50 peers (nsdi-eval/credit/*, last-10 mean validation error)
    "credit50_3v30": ({"num_nodes": 50, "dataset": "creditcard", "poisoning": 0.3}, 1.98, 1 - 0.0598, {},
                      "nsdi-eval/credit/bis_3v_30p"),
    "credit50_5v30": ({"num_nodes": 50, "dataset": "creditcard", "poisoning": 0.3, "num_verifiers": 5}, None,
                      1 - 0.0451, {}, "nsdi-eval/credit/bis_5v_30p"),
    "credit50_3v50": ({"num_nodes": 50, "dataset": "creditcard", "poisoning": 0.5}, None, 1 - 0.0905, {},
                      "nsdi-eval/credit/bis_3v_50p"),
    "poison50_5v": ({"num_nodes": 50, "dataset": "creditcard", "poisoning": 0.5, "num_verifiers": 5}, None,
                    1 - 0.0658, {}, "nsdi-eval/credit/bis_5v_50p"),
    "credit50_fed30": ({"fedsys": True, "num_nodes": 50, "dataset": "creditcard", "poisoning": 0.3,
                        "perc_samples": 35}, None, 1 - 0.0007, {}, "nsdi-eval/credit/fed_30p"),
    "credit50_fed50": ({"fedsys": True, "num_nodes": 50, "dataset": "creditcard", "poisoning": 0.5,
                        "perc_samples": 35}, None, 1 - 0.6310, {}, "nsdi-eval/credit/fed_50p"),
    "churn10": ({"churn": 0.1}, None, None, {}, "BASELINE.json config 5 (reference churn runs: 25-31 s/round)"),
    # process churn with state loss + rejoin (eval/eval_FT/runEval.sh: a node killed every 60/rate s,
    # restarted 5 s before the next kill), 50 MNIST peers as in nsdi-eval/churn.  Those logs' leader fired at
    # 5 shares ("As miner, I expect 5 shares", 60s.log:9686 -- 50 peers / 10, an older main.go), not at
    # NUM_SAMPLES/2 = 17: the presets use that threshold (miner_threshold=tenth); *_half keep the live rule
    "churn_kill4": ({"num_nodes": 50, "churn_kill_per_min": 4.0, "miner_threshold": "tenth"}, 30.92, 1 - 0.121, {},
                    "nsdi-eval/churn/15s.log"),
    "churn_kill2": ({"num_nodes": 50, "churn_kill_per_min": 2.0, "miner_threshold": "tenth"}, 26.27, 1 - 0.210, {},
                    "nsdi-eval/churn/30s.log"),
    "churn_kill1": ({"num_nodes": 50, "churn_kill_per_min": 1.0, "miner_threshold": "tenth"}, 25.71, 1 - 0.138, {},
                    "nsdi-eval/churn/60s.log"),
    "churn_kill05": ({"num_nodes": 50, "churn_kill_per_min": 0.5, "miner_threshold": "tenth"}, 25.44, 1 - 0.191, {},
                     "nsdi-eval/churn/120s.log"),
    "churn_kill1_half": ({"num_nodes": 50, "churn_kill_per_min": 1.0}, 25.71, 1 - 0.138, {},
                         "nsdi-eval/churn/60s.log (leader at NUM_SAMPLES/2, main.go:360: not the logs' rule)"),
    # the headline with the leader firing at N/8 shares (minBlockSize, main.go:348-352)
    "headline_eighth": ({"miner_threshold": "eighth"}, 29.83, 0.877, {},
                        "nsdi-eval/scaleup/bis_baseline_100 (leader at N/8 shares, main.go:348-352)"),
    # weak scaling: 100 peers per rank, reference defaults otherwise (the reference's scaling axis is the peer
    # count: nsdi-eval/increments/results.log:1-5, eval/eval_FedSys_scale); num_nodes = 100 x ranks
    "scale_weak": ({"peers_per_rank": 100}, None, None, {},
                   "nsdi-eval/increments/results.log:1-5 (peer-count axis; no published number at these sizes)"),
    # the long-parameter-vector ledger: LFW maleness softmax, d = 17486 (no reference number:
    # the reference's lfw pipeline is inconsistent, see data.dataset_dims)
    "lfw100": ({"dataset": "lfw"}, None, None, {}, "honest.go:211 'mnist/lfw for pytorch' (unpinned)"),
    # headline + the batched verifySecret audit of every aggregate (K13; not on the reference's path)
    "kzg_audit": ({"kzg_audit": "consistent"}, 29.83, 0.877, {}, "nsdi-eval/scaleup/bis_baseline_100 + K13 audit"),
    "scale40": ({"num_nodes": 40}, 23.87, None, {}, "nsdi-eval/increments/results.log:2"),
    "scale60": ({"num_nodes": 60}, 34.05, None, {}, "nsdi-eval/increments/results.log:3"),
    "scale80": ({"num_nodes": 80}, 48.07, None, {}, "nsdi-eval/increments/results.log:4"),
    # 200 peers (eval/eval_FedSys_scale runs FedSys up to 200; Krum inboxes of 140 updates)
    "scale200": ({"num_nodes": 200}, None, None, {}, "eval/eval_FedSys_scale (Biscotti at 200 peers: unpinned)"),
    "secagg_off": ({"secure_agg": False}, 50.63, None, {}, "nsdi-eval/increments/results.log:10"),
    "verification_off": ({"verification": False}, 19.95, None, {}, "nsdi-eval/increments/results.log:15"),
    "noising_off": ({"noising": False}, 53.10, None, {}, "nsdi-eval/increments/results.log:20"),
    "mnist10_dp1": ({"num_nodes": 10, "epsilon": 1.0}, None, None, {}, "BASELINE.json config 2"),
    "credit4": ({"num_nodes": 4, "dataset": "creditcard", "noising": False, "num_verifiers": 1,
                 "num_miners": 2, "num_noisers": 1, "epsilon": 0.0}, None, None, {}, "BASELINE.json config 1"),
}


def _host_threads() -> int:
    """Native crypto pool per rank: what the job's CPU quota leaves after every local rank's round thread,
    HIP runtime and RCCL threads (utils/threadcpu.pool_threads)."""
    import os

    from biscotti_amd.utils.threadcpu import pool_threads

    world = int(os.environ.get("WORLD_SIZE", "1"))
    return pool_threads(int(os.environ.get("LOCAL_WORLD_SIZE", str(world))), world)


def _pct(vals: list) -> tuple:
    v = sorted(vals)
    return (round(1e3 * v[len(v) // 2], 4), round(1e3 * v[-1], 4)) if v else (None, None)


def _pct_by_name(calls: list) -> dict:
    """{collective: {n, p50_ms, max_ms}} of the host time inside each collective call."""
    by: dict = {}
    for name, s in calls:
        by.setdefault(name, []).append(s)
    out = {}
    for name, v in sorted(by.items()):
        p50, mx = _pct(v)
        out[name] = {"n": len(v), "p50_ms": p50, "max_ms": mx}
    return out


def _phase_p50_max(round_phases: list) -> dict:
    """{phase: [median ms, worst-round ms]} over the timed rounds (phases a round did not enter count 0)."""
    keys = sorted({k for p in round_phases for k in p})
    return {k: list(_pct([p.get(k, 0.0) for p in round_phases])) for k in keys}


def _outliers(walls: list) -> dict:
    if not walls:
        return {}
    med = sorted(walls)[len(walls) // 2]
    return {"round_wall_p50_ms": round(1e3 * med, 4), "round_wall_max_ms": round(1e3 * max(walls), 4),
            "rounds_over_3x_median": sum(w > 3 * med for w in walls),
            "rounds_over_5x_median": sum(w > 5 * med for w in walls)}


def _spawn_ranks(n: int) -> int:
    """Run this same command under torch.distributed.run with n local ranks (127.0.0.1 rendezvous on a
    free port) as a child process; the parent only waits (it must not initialise the GPU)."""
    import os
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4")))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="headline", choices=sorted(PRESETS))
    ap.add_argument("--peers", type=int, default=None, help="override the preset's peer count")
    ap.add_argument("--set", action="append", default=[], metavar="FIELD=VALUE",
                    help="override any RunConfig field (sweeps), e.g. --set num_verifiers=5")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--seeds", type=int, default=1, help="accuracy over this many independent 100-round runs")
    ap.add_argument("--rounds", type=int, default=100, help="rounds the accuracy is quoted at (MAX_ITERATIONS)")
    ap.add_argument("--trace", default=None)
    ap.add_argument("--fedsys", action="store_true", help="same as --config fedsys")
    ap.add_argument("--emulate-world", type=int, default=0, metavar="N",
                    help="run rank 0 of an N-rank job alone on this GPU (other ranks' collective slots filled with "
                         "rank 0's data): the per-rank cost of an N-GPU job, never a scaling number")
    ap.add_argument("--phase-sync", action="store_true",
                    help="synchronise the GPU at every phase boundary (per-phase GPU attribution, slower)")
    ap.add_argument("--deterministic-time", action="store_true",
                    help="block timestamps = iteration + 1 (RunConfig.deterministic_time): a seed's chain, and so "
                         "its accuracy curve, is the same run to run (--seeds experiments)")
    a = ap.parse_args()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched without torchrun: start the N rank processes ourselves (one per GPU, RCCL over xGMI)
        # from this parent, which never touches the GPU, and exit with their status
        return _spawn_ranks(a.gpus)
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank number "
                         f"as {a.gpus} GPUs")
    if a.fedsys:
        a.config = "fedsys"
    over, ref_s, ref_acc, ref_extra, ref_src = PRESETS[a.config]
    over = dict(over)
    fedsys = over.pop("fedsys", False)
    per_rank_peers = over.pop("peers_per_rank", None)
    if per_rank_peers:   # weak scaling: the job's peers grow with its ranks (emulated ranks count)
        over["num_nodes"] = per_rank_peers * max(world, a.emulate_world, 1)

    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    if a.emulate_world > 1:
        if world != 1 or a.gpus != 1:
            raise SystemExit("--emulate-world runs one process on one GPU (--gpus 1, no torchrun)")
        comm = Comm.emulated(a.emulate_world)
    else:
        comm = Comm.init()
    if comm.device.type == "cuda":
        # the GPU path does little CPU tensor work; idle-spinning OpenMP workers would only steal the
        # cgroup CPU quota from the native crypto pool
        torch.set_num_threads(min(4, torch.get_num_threads()) if comm.world == 1 else 1)
    # lazy_eval: each round's two evaluation numbers are read back one round later (the kernels still run
    # inside the round); the accuracies below are read after drain()
    kw = dict(num_nodes=100, dataset="mnist", seed=a.seed, max_iterations=10**9, trace_file=a.trace,
              host_threads=_host_threads(), phase_sync=a.phase_sync, lazy_eval=True,
              deterministic_time=a.deterministic_time)
    kw.update(over)
    if a.peers:
        kw["num_nodes"] = a.peers
    types = {f.name: f.type for f in dataclasses.fields(RunConfig)}
    for item in a.set:
        k, v = item.split("=", 1)
        if k not in types:
            raise SystemExit(f"unknown RunConfig field {k!r}")
        cur = kw.get(k, getattr(RunConfig, k, None))
        kw[k] = (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v) if cur is not None \
            else v
    cfg = RunConfig(**kw)

    def build(c):
        if fedsys:
            from biscotti_amd.protocol.fedsys import FedSysEngine

            return FedSysEngine(c, comm)
        return BiscottiEngine(c, comm)

    t_setup = time.perf_counter()
    eng = build(cfg)
    sync = (lambda: torch.cuda.synchronize()) if eng.gpu else (lambda: None)
    sync()
    setup_s = time.perf_counter() - t_setup   # engine + HBM-resident tables (keygen/bootstrap analogue)
    for i in range(a.warmup):
        # the last warm-up round does not start the first timed round's front (engine._round_front): the timed
        # window holds exactly its own rounds' work
        eng.run_round(front=False) if i == a.warmup - 1 and hasattr(eng, "_round_front") else eng.run_round()
    comm.barrier()
    sync()
    import resource

    from biscotti_amd.utils import threadcpu

    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    th0 = threadcpu.snapshot()
    cg0 = threadcpu.cgroup_cpu_stat()
    comm.take_calls()
    t0 = time.perf_counter()
    last = None
    phases: dict = {}
    round_phases: list = []
    results = []
    walls = []
    seg0 = torch.cuda.memory_stats(comm.device).get("segment.all.allocated", 0) if eng.gpu else 0
    for k in range(a.steps):
        tr = time.perf_counter()
        # the run's end: the penultimate round's front launches the still-batched device VRF proofs and the last
        # round proves its own on the host (all inside the clock; drain() then waits less)
        last = eng.run_round(last=k == a.steps - 1, remaining=a.steps - k) if hasattr(eng, "_round_front") \
            else eng.run_round(last=k == a.steps - 1) if hasattr(eng, "drain") else eng.run_round()
        walls.append(time.perf_counter() - tr)
        results.append(last)
        round_phases.append(last.phases)
        for k, v in last.phases.items():
            phases[k] = phases.get(k, 0.0) + v
    t_drain = time.perf_counter()
    if hasattr(eng, "drain"):
        eng.drain()   # host work of the timed rounds still in flight (and their evaluations) inside the clock
    sync()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    drain_s = time.perf_counter() - t_drain
    drain_parts = dict(getattr(eng, "drain_parts_ms", None) or {})
    # device memory segments the caching allocator had to hipMalloc inside the timed window
    seg_new = (torch.cuda.memory_stats(comm.device).get("segment.all.allocated", 0) - seg0) if eng.gpu else 0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    th1 = threadcpu.snapshot()
    cg = threadcpu.cgroup_delta(cg0, threadcpu.cgroup_cpu_stat())
    calls = comm.take_calls()
    host_cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)   # every thread of this rank
    stats0 = {k: v for k, v in getattr(eng, "stats", {}).items() if isinstance(v, (int, float))}
    per_step = 1e3 / max(a.steps, 1)
    # this rank's host cost: CPU per thread group (the round's Python thread, the native crypto pool, RCCL /
    # gloo / HIP runtime threads), the round's phases and the engine's fast-path counters
    mine = {"rank": comm.rank, "host_cpu_ms_per_round": host_cpu * per_step,
            "thread_cpu_ms_per_round": {k: round(v * per_step, 3)
                                        for k, v in list(threadcpu.delta_by_group(th0, th1).items())[:10]},
            "phase_ms_per_round": {k: round(v * per_step, 4) for k, v in sorted(phases.items())},
            "engine_stats": stats0, "elapsed_s": elapsed,
            # stall attribution (docs/PERF.md, multi-rank stalls): the cgroup's CFS throttling over the timed window,
            # the host time inside each collective call, per-phase median / worst round, and the round outliers
            "cgroup_cpu_stat_delta": cg, "cpu_quota": threadcpu.cpu_quota(),
            "collective_ms": _pct_by_name(calls),
            "phase_ms_p50_max": _phase_p50_max(round_phases),
            "round_wall_ms": [round(1e3 * w, 3) for w in walls],
            **_outliers(walls)}
    per_rank = [mine]
    real_world = 1 if comm.emulating else comm.world
    if real_world > 1:
        import torch.distributed as dist

        per_rank = [None] * comm.world
        dist.all_gather_object(per_rank, mine)
    t = torch.tensor([elapsed], dtype=torch.float64, device=comm.device)
    if real_world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    s_per_round = elapsed / max(a.steps, 1)
    accs = [1.0 - r.test_error for r in results]
    attacks = [r.attack_rate for r in results]

    # accuracy is quoted the reference's way: after MAX_ITERATIONS = 100 rounds (untimed rounds finish
    # the run when warmup + steps < 100), final value and last-10 mean, over --seeds runs
    def finish(e, acc_l, att_l, done):
        rs = []
        while done < a.rounds:
            rs.append(e.run_round())
            done += 1
        if hasattr(e, "drain"):
            e.drain()
        acc_l.extend(1.0 - r.test_error for r in rs)
        att_l.extend(r.attack_rate for r in rs)
        return acc_l, att_l

    all_acc = [[None] * a.warmup + accs]
    all_att = [[None] * a.warmup + attacks]
    finish(eng, all_acc[0], all_att[0], a.warmup + a.steps)
    for k in range(1, a.seeds):
        if hasattr(eng, "close"):
            eng.close()
        e2 = build(dataclasses.replace(cfg, seed=a.seed + k, trace_file=None))
        acc_l, att_l = finish(e2, [], [], 0)
        all_acc.append(acc_l)
        all_att.append(att_l)
        eng = e2
    import statistics as st

    def ms(vals):
        vals = [v for v in vals if v is not None and v == v]
        if not vals:
            return None, None
        return float(st.mean(vals)), float(st.pstdev(vals)) if len(vals) > 1 else 0.0

    R = a.rounds
    finals = [l[R - 1] if len(l) >= R else l[-1] for l in all_acc]
    last10 = [st.mean([v for v in l[max(0, min(R, len(l)) - 10):min(R, len(l))] if v is not None]) for l in all_acc]
    att_final = [l[R - 1] if len(l) >= R else l[-1] for l in all_att]
    att10 = [st.mean([v for v in l[max(0, min(R, len(l)) - 10):min(R, len(l))] if v is not None]) for l in all_att]
    acc = finals[0]
    ok, why = eng.fsm.chain.verify() if not fedsys else (True, "")
    # contributors per committed block (updates in the block; the reference's churn logs show it as the stake
    # map's growth: stake_unit per contributor) and the stake total, for the churn comparisons
    blocks = len(eng.fsm.chain) - 1 if not fedsys else None
    contrib = (eng.stats.get("total_updates", 0) / max(1, eng.rounds_done)) if not fedsys else None
    stake_total = int(sum(dict(eng.fsm.stake).values())) if not fedsys else None
    from biscotti_amd.utils import flush_logs

    flush_logs(eng.log)   # buffered log lines go out before the result line
    if comm.rank == 0:
        headline = a.config == "headline"
        out = {
            "metric": ("sec/round (block commit) + final test acc, MNIST 100 peers" if headline else
                       f"sec/round + final test acc, {a.config}")
                      + (f" [emulated rank 0 of {comm.world}: per-rank cost, not a scaling number]"
                         if comm.emulating else ""),
            "value": s_per_round,
            "unit": "s/round",
            "n_gpus": real_world,
            "emulated_world": comm.world if comm.emulating else None,
            "device": comm.device.type,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * s_per_round,
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": s_per_round / ref_s if ref_s and not comm.emulating else None,
            "speedup_vs_baseline": ref_s / s_per_round if ref_s and not comm.emulating else None,
            "final_test_acc": acc,
            "test_acc_last10_mean": last10[0],
            "accuracy_rounds": R,
            "seeds": a.seeds,
            "final_test_acc_mean_std": ms(finals),
            "final_test_acc_per_seed": finals,
            "test_acc_last10_per_seed": last10,
            "test_acc_last10_mean_std": ms(last10),
            "setup_s": setup_s,
            "drain_ms": 1e3 * drain_s,          # inside the timed window: joins of the last rounds' work
            "drain_parts_ms": drain_parts,
            "device_segments_allocated_timed": seg_new,
            "round_wall_ms": [round(1e3 * w, 3) for w in walls],
            "host_cpu_ms_per_round": 1e3 * host_cpu / max(a.steps, 1),
            "thread_cpu_ms_per_round": mine["thread_cpu_ms_per_round"],
            "cgroup_cpu_stat_delta": mine["cgroup_cpu_stat_delta"],
            "cpu_quota": mine["cpu_quota"],
            "host_threads": cfg.host_threads,
            "collective_ms": mine["collective_ms"],
            "phase_ms_p50_max": mine["phase_ms_p50_max"],
            **_outliers(walls),
            "engine_stats": stats0,
            # per committed block: how deep in the leader's candidate arrival order its rows reached, of how many
            # candidates, and the leader's cap (the speculative horizon's input)
            "spec_depths": [list(x) for x in getattr(eng, "spec_depth_log", [])][:a.warmup + a.steps],
            "table_gb": (eng.crypto.eng.table_bytes() / 1e9) if hasattr(getattr(eng, "crypto", None), "eng") else 0.0,
            "b0": getattr(getattr(getattr(eng, "crypto", None), "eng", None), "b0", None),
            "baseline_test_acc": ref_acc,
            "baseline_source": ref_src,
            "rounds_total": eng.rounds_done if not fedsys else eng.iteration,
            "dtype": "fp32 model / fp64 ledger / exact BN256",
            "data": {"mnist": "synthetic: MNIST-shaped digits from sklearn's 8x8 real digits, augmented; zero-init model",
                     "lfw": "synthetic: class-conditional 62x47x3 faces, maleness labels; zero-init model"}
                    .get(cfg.dataset, "creditcard.csv shipped with the reference"),
            "config": {"name": a.config, "model": {"mnist": "softmax regression 784x10 (7850 params, SoftmaxModel)",
                                                   "lfw": "softmax regression 8742x2 (17486 params, SoftmaxModel)"}
                       .get(cfg.dataset, "logistic regression (25)"),
                       "peers": cfg.num_nodes, "global_batch": cfg.num_nodes * cfg.batch_size, "seq_len": 1,
                       "parallelism": (f"emulated rank 0 of dp{comm.world} (virtual peers: "
                                       f"{len(comm.peer_range(cfg.num_nodes))} on this GPU; collectives not timed)"
                                       if comm.emulating else
                                       f"dp{comm.world} (virtual peers: {math.ceil(cfg.num_nodes / comm.world)}/GPU)"),
                       "verifiers": cfg.num_verifiers, "aggregators": cfg.num_miners, "noisers": cfg.num_noisers,
                       "epsilon": cfg.epsilon, "ns_percent": cfg.perc_samples, "poisoning": cfg.poisoning,
                       "churn": cfg.churn, "secure_agg": cfg.secure_agg, "verification": cfg.verification,
                       "noising": cfg.noising, "fedsys": fedsys},
            "phase_ms_per_round": {k: 1e3 * v / max(a.steps, 1) for k, v in sorted(phases.items())},
            "phase_sync": bool(a.phase_sync),
            "chain_valid": bool(ok),
            "miner_threshold": getattr(cfg, "miner_threshold", None),
            "leader_cap": eng.fsm.leader_cap_size() if not fedsys else None,
            "contributors_per_block": contrib,
            "stake_total": stake_total,
            "stake_initial": cfg.num_nodes * cfg.default_stake,
            "chain_blocks": blocks,
            "deterministic_time": bool(cfg.deterministic_time),
        }
        if cfg.dataset == "mnist":
            out["final_attack_rate"] = att_final[0]
            out["attack_rate_last10_mean"] = att10[0]
            out["final_attack_rate_mean_std"] = ms(att_final)
            out["attack_rate_last10_mean_std"] = ms(att10)
            out["attack_rate_last10_per_seed"] = att10
        for k, v in ref_extra.items():
            out[f"baseline_{k}"] = v
        if real_world > 1:
            out["per_rank"] = per_rank
        print(json.dumps(out), flush=True)
    comm.barrier()
    if not fedsys:
        eng.close()
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
