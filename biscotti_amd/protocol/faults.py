"""Failure injection and recovery of the round engine: per-round availability churn, process churn with
state loss and chain-sync rejoin, network partitions, and chain resume from disk.

Reference: DistSys/blockNode.sh (iptables partition of one peer's port for 30 s),
DistSys/failAndRestartLocal.sh and eval/eval_FT/runEval.sh (kill / restart loop), the RegisterPeer
chain adoption (main.go:420-436,1000-1013, honest.go:679-685) and the FAIL_PROB crash
(main.go:1117-1120).  Every schedule is a function of the round seed, so every rank replicates it.
"""
from __future__ import annotations

import numpy as np


class FaultsMixin:
    def _resume(self, path: str) -> None:
        import os

        if not os.path.exists(path):
            return
        chain = self.R.Blockchain.load(path)
        self.fsm.chain = chain
        last = chain.latest()
        self.fsm.iteration = last.data.iteration
        if len(last.stake):
            self.fsm.stake = dict(last.stake)
        self.log.info("Resumed chain of %d blocks at iteration %d", len(chain), last.data.iteration)

    def _live_mask(self) -> list[int]:
        live = [1] * self.N
        if self.cfg.churn > 0:
            # per-round availability churn: a seeded fraction of the peers is unreachable this round
            seed = self.fsm.round_seed(7)
            perm = self.R.seeded_permutation(self.N, seed)
            k = int(round(self.cfg.churn * self.N))
            for p in perm[:k]:
                live[p] = 0
        if self.cfg.churn_kill_per_min > 0:
            self._crash_restart(live)
        if self._partitions:
            # DistSys/blockNode.sh: iptables drops the peer's port both ways for 30 s -- it neither
            # receives nor sends, i.e. it is offline for those rounds (and keeps its state)
            it = self.fsm.iteration + 1   # the round being opened (as in _crash_restart)
            for peer, first, rounds in self._partitions:
                if first <= it < first + rounds:
                    live[peer] = 0
        return live

    def _crash_restart(self, live: list) -> None:
        """Process churn with state loss (eval/eval_FT/runEval.sh, DistSys/failAndRestartLocal.sh): every
        60/rate seconds a random peer other than 0 is killed, stays down for 60/rate - 5 s and is
        restarted.  Seconds map to rounds through cfg.churn_round_s (the reference's churn runs took
        25-31 s per round).  A killed peer loses its state; the restarted process generates fresh
        VRF keys (myVRF.init at start-up, vrf.go:16-32) and rejoins through RegisterPeer: it adopts
        the longest chain it is offered after checking it (main.go:420-436,1000-1013,
        honest.go:679-685) -- here the blocks it missed are re-hashed and link-checked
        (Blockchain.verify_range) by the rank that hosts it.  Deterministic (round seed): every rank
        replicates the schedule."""
        from .engine import _seed_bytes

        cfg, fsm = self.cfg, self.fsm
        st = self._churn
        it = fsm.iteration + 1   # the round being opened
        # restarts due this round
        for p, back in list(st["down"].items()):
            if it >= back:
                del st["down"][p]
                view = st["view"].get(p, 1)
                height = len(fsm.chain)
                st["epoch"][p] = st["epoch"].get(p, 0) + 1
                st["rejoins"] += 1
                e = st["epoch"][p]
                self.vrf_noise_seed[p] = _seed_bytes(cfg.seed, f"vrf-noise-e{e}", p)
                self._seed_version = getattr(self, "_seed_version", 0) + 1   # native seed sets are rebuilt
                self.vrf_roles_seed[p] = _seed_bytes(cfg.seed, f"vrf-roles-e{e}", p)
                if p in self.local:
                    ok, why = fsm.chain.verify_range(max(0, view - 1), height)
                    if not ok:
                        raise RuntimeError(f"peer {p}: the chain offered at rejoin does not verify: {why}")
                    st["synced_blocks"] += height - view
                    self.log.info("%d:Rejoined at iteration %d: adopted a chain of %d blocks (%d verified)", p, it,
                                  height, height - view)
        # kills due this round
        st["acc"] += cfg.churn_kill_per_min * cfg.churn_round_s / 60.0
        down_rounds = max(1, int(np.ceil((60.0 / cfg.churn_kill_per_min - 5.0) / cfg.churn_round_s)))
        cand = [p for p in range(1, self.N) if p not in st["down"]]
        perm = self.R.seeded_permutation(len(cand), fsm.round_seed(11)) if cand else []
        j = 0
        while st["acc"] >= 1.0 and j < len(cand):
            p = cand[perm[j]]
            j += 1
            st["acc"] -= 1.0
            st["down"][p] = it + down_rounds
            st["view"][p] = len(fsm.chain)   # its chain at the moment it died
            st["kills"] += 1
        for p in st["down"]:
            live[p] = 0

    def _maybe_fail(self, it: int) -> None:
        """Fault injection (cfg.fail_at): this rank's process dies abruptly after committing block `it`
        (the reference's FAIL_PROB crash / failAndRestartLocal.sh kill); the surviving ranks' next
        collective fails and an elastic launcher restarts the job from the chain file."""
        f_it, f_rank = self.cfg.fail_point()
        if it != f_it or self.comm.rank != f_rank:
            return
        import os
        import sys

        from ..utils import flush_logs

        self.log.info("fault injection: rank %d exits after iteration %d", self.comm.rank, it)
        flush_logs(self.log)
        sys.stderr.flush()
        os._exit(17)
