"""FedSys: the reference's centralised federated-learning baseline (FedSys/*.go), on the same
virtual-peer / collective substrate as Biscotti.

Semantics kept from the reference:
  * star topology: peer 0 is the server (``amLeader``: port == basePort, FedSys/main.go:760-764);
    every other peer is a worker that takes one SGD step on the current global model
    (``computeUpdate``, FedSys/honest.go:165-181) -- no noise, commitments, committees or chain;
  * the server aggregates the first ``NUM_SAMPLES = int(N * ns / 100)`` updates to arrive
    (``processUpdate``, FedSys/main.go:530-584; -ns defaults to 35, main.go:212);
    with ``-rs`` it waits for all N-1 and draws ``RANDOM_SAMPLES`` of them WITH replacement
    (main.go:241-244, ``sampleUpdates`` FedSys/honest.go:130-163);
  * the new model is the plain SUM of the selected deltas added to W (``createNewModel``,
    honest.go:311-337) and is broadcast to every worker (``sendModel``, main.go:612-644);
  * poisoners (``-po``) train on the poisoned data; FedSys marks ids >= ceil(N(1-po)) (note the
    ``>=`` vs Biscotti's ``>``, quirk recorded in docs/QUIRKS.md);
  * creditcard uses EPSILON = 5 for its at-source DP noise (FedSys/main.go:42).

MI355X mapping: all workers' steps are one fused batched kernel per rank (the same K1 kernel as
Biscotti); the "RegisterUpdate" fan-in is one all_gather of the local delta slab, and every rank
applies the server's selection itself -- the "RegisterModel" broadcast is implied because the
aggregation is deterministic (the server's arrival order is a seeded permutation).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..native import rt
from ..parallel.comm import Comm
from ..utils import JsonlWriter, PhaseTimer, get_logger, h2d
from .config import RunConfig


@dataclass
class FedSysResult:
    iteration: int
    selected: list
    test_error: float
    attack_rate: float
    wall: float
    phases: dict = field(default_factory=dict)


class FedSysEngine:
    def __init__(self, cfg: RunConfig, comm: Comm | None = None):
        from ..data import dataset_dims
        from ..models import make_task

        self.cfg = cfg
        self.comm = comm or Comm()
        self.R = rt()
        self.dev = self.comm.device if cfg.device != "cpu" else torch.device("cpu")
        self.gpu = self.dev.type == "cuda"
        self.N = cfg.num_nodes
        self.local = self.comm.peer_range(self.N)
        self.maxlocal = self.comm.max_local(self.N)
        self.log = get_logger("peer", f"{cfg.log_dir}/log_{self.comm.rank}_{self.N}.log" if cfg.log_dir else None)
        self.trace = JsonlWriter(cfg.trace_file if self.comm.rank == 0 else None)
        self.timer = PhaseTimer(sync=(lambda: torch.cuda.synchronize(self.dev)) if self.gpu and cfg.phase_sync
                                else None)
        fc = self.R.FedSysConfig()
        fc.num_nodes, fc.perc_samples, fc.rand_sample, fc.poisoning = \
            self.N, cfg.perc_samples, cfg.rand_sample, cfg.poisoning
        fc.derive()
        self.fc = fc
        pc = cfg.protocol(self.R)
        self.d = dataset_dims(cfg.dataset)[0]
        probe = self.R.RoundFSM(pc, self.d)
        poisoned = {p for p in self.local if probe.is_poisoner(p, True)}   # FedSys: >= (Q4)
        self.task = make_task(cfg.dataset, self.local, self.N, self.dev, cfg.seed, poisoned=poisoned,
                              batch_size=cfg.batch_size, data_dir=cfg.data_dir, epsilon=cfg.epsilon,
                              colluders=set())
        self.W = torch.zeros(self.d, dtype=torch.float64, device=self.dev)
        self.iteration = 0
        self.history: list = []        # BlockData of every model the server broadcast

    def _seed(self, it: int) -> int:
        return (self.cfg.seed * 0x9E3779B97F4A7C15 + it * 0xBF58476D1CE4E5B9 + 0xF5D5) & (2**64 - 1)

    def run_round(self) -> FedSysResult | None:
        cfg, comm, tm = self.cfg, self.comm, self.timer
        if self.iteration > cfg.max_iterations:
            return None
        t0 = time.perf_counter()
        it = self.iteration
        workers = [p for p in self.local if p != 0]
        with tm.phase("local_step"):
            delta, _ = self.task.step(self.W, it, workers)
        with tm.phase("gather"):
            buf = torch.zeros((self.maxlocal, self.d), dtype=torch.float32, device=self.dev)
            if workers:
                lo = self.local.start
                buf.index_copy_(0, h2d([w - lo for w in workers], torch.long, self.dev), delta)
            allw = comm.all_gather(buf).reshape(-1, self.d)
        with tm.phase("aggregate"):
            submitted = list(range(1, self.N))
            sel = self.R.fedsys_select(self.fc, submitted, self._seed(it))
            rows = [r * self.maxlocal + (p - comm.peer_range(self.N, r).start)
                    for p in sel for r in [comm.owner(p, self.N)]]
            if rows:
                idx = h2d(rows, torch.long, self.dev)
                self.W = self.W + allw.index_select(0, idx).double().sum(0)   # createNewModel: plain sum
            bd = self.R.BlockData()
            bd.iteration = it
            bd.global_w = self.W.cpu().numpy()
            self.history.append(bd)
        with tm.phase("eval"):
            ev = self.task.evaluate(self.W)
        self.iteration += 1
        r = FedSysResult(it, list(sel), ev["test_error"], ev.get("attack_rate", float("nan")),
                         time.perf_counter() - t0, tm.reset())
        self.log.info("%d:Train Error is %.5f in Iteration %d", self.local.start, r.test_error, it)
        if cfg.dataset != "creditcard":
            self.log.info("%d:Attack Rate is %.5f in Iteration %d", self.local.start, r.attack_rate, it)
        self.trace.write({"iteration": it, "wall_s": r.wall, "selected": len(sel), "test_error": r.test_error,
                          **{f"t_{k}": v for k, v in r.phases.items()}})
        return r

    def model_digest(self) -> str:
        """SHA-256 of the gob encoding of the latest BlockData (what localTest.sh compares)."""
        if not self.history:
            return ""
        return self.R.sha256(self.history[-1].gob()).hex()
