"""Noising and verification of a round: the noiser lottery, DP noise, the verifier committee's Multi-Krum
(or RONI) and the verifiers' Schnorr signatures.

Reference: requestNoise / NoisedDelta (main.go:1513-1660, client_obj.py:97-98), VerifyUpdateKRUM
(krum.go:227-365: each verifier collects its own first KRUM_UPDATETHRESH arrivals and accepts the
n - floor(n/2) lowest Krum scores, client_obj.py:114-143), VerifyUpdateRONI (main.go:191-233), the
>= floor(nv/2) signature rule (main.go:1686), the leader's NUM_SAMPLES/2 cap (main.go:360) and
SchnorrSign (kyber.go:873-896).

Multi-Krum is a pure function of the noised updates, so every rank evaluates the whole committee on
identical inputs (deterministic kernels) instead of exchanging accept masks.  With the noise-aware
form the d-dimensional Gram is already in flight (head); several ranks exchange only each local
worker's commitment, noiser ids and noiser weights in ONE all_gather after the VRF outputs.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import bn256 as B
from ..ops import ml as K
from ..utils import d2h_into, h2d, h2d_many, pinned
from ..utils import streams as S
from .crypto_backends import _CommitTable

SIGN_THREADS = 4   # verifier signature batches: narrow, the pool's rest serves the VRF outputs


class VerifyMixin:
    # ------------------------------------------------------------------ noisers and noise
    def _select_noisers(self, fut_noise, stake, local_workers, index=None, after=None) -> dict:
        """Each worker's noisers from its own VRF output (getVRFNoisers, vrf.go:54-100).  Waits for the
        outputs only; the proofs finish on the native threads (or the device) and are joined later.
        index: positions of local_workers in the job's output list (an early job covers more peers).
        after: a block not committed yet whose stake the lottery uses (the speculative front)."""
        if fut_noise is None or not local_workers:
            return {}
        # the lottery reads the job's outputs natively (no 64-byte Python objects in between)
        idx = list(index) if index is not None else []
        nn = self.cfg.num_noisers
        if after is not None:
            sel = self.R.select_noisers_job_after(self.fsm, after, fut_noise, idx, local_workers, nn, self.N)
        elif stake is None:
            sel = self.fsm.select_noisers_job(fut_noise, idx, local_workers, nn, self.N)
        else:
            sel = self.R.select_noisers_job(stake, fut_noise, idx, local_workers, nn, self.N)
        self._noise_arr = (local_workers, sel)   # the same ids as an array, in local_workers order
        return dict(zip(local_workers, sel.tolist()))

    def _noise_scales(self, noisers: dict, ws: list) -> np.ndarray:
        """float32 [len(ws), nn]: each noiser's vector weight (getNoise's -sigma/sqrt(B)); 0 for colluding
        noisers (isCollusionAttack, main.go:1026-1057)."""
        ids = np.asarray([noisers[w] for w in ws], np.int64).reshape(len(ws), -1)
        sc = np.full(ids.shape, self.task.noise_scale(self.sigma), np.float32)
        if self.colluders:
            sc[np.isin(ids, np.fromiter(self.colluders, np.int64))] = 0.0
        return sc

    def _noise_ids_np(self, noisers: dict, local_workers: list):
        """(ids int32, weights fp32) [maxlocal, nn]: row w - lo holds local worker w's noisers and their
        weights (zeros elsewhere: rows that are in no inbox)."""
        nn_ = self.cfg.num_noisers
        nz = np.zeros((self.maxlocal, nn_), np.int32)
        sc = np.zeros((self.maxlocal, nn_), np.float32)
        if local_workers and noisers:
            # the rows of local_workers, cached per list (the round's head keeps one list object per round)
            c = getattr(self, "_noise_at", None)
            if c is None or c[0] is not local_workers:
                c = self._noise_at = (local_workers, np.asarray(local_workers, np.int64) - self.lo)
            at = c[1]
            arr = getattr(self, "_noise_arr", None)
            # the lottery's array (same ids, local_workers order) when it is this round's; else from the dict
            ids = arr[1].reshape(len(local_workers), -1) if arr is not None and arr[0] is local_workers else \
                np.asarray([noisers[w] for w in local_workers], np.int64).reshape(len(local_workers), -1)
            if ids.size and not (0 <= int(ids.min()) and int(ids.max()) < self.N):
                raise ValueError("noiser id out of range")
            nz[at] = ids
            if self.colluders:
                w = np.full(ids.shape, self.task.noise_scale(self.sigma), np.float32)
                w[np.isin(ids, self._colluder_arr())] = 0.0
                sc[at] = w
            else:
                sc[at] = self.task.noise_scale(self.sigma)
        return nz, sc

    def _colluder_arr(self) -> np.ndarray:
        arr = getattr(self, "_colluders_np", None)
        if arr is None:
            arr = self._colluders_np = np.fromiter(sorted(self.colluders), np.int64)
        return arr

    def _worker_rows(self, t: torch.Tensor, row_of: dict, ws: list) -> torch.Tensor:
        """Rows of t for the workers ws, in that order."""
        idx = [row_of[w] for w in ws]
        if idx == list(range(t.shape[0])):
            return t
        return t.index_select(0, h2d(idx, torch.long, self.dev))

    def _noise(self, delta, row_of, noisers, local_workers, it):
        """Noised deltas of the local workers in local_workers order (requestNoise + NoisedDelta,
        main.go:1513-1660): each worker's noisers' pre-sampled vectors averaged and added."""
        cfg = self.cfg
        delta = self._worker_rows(delta, row_of, local_workers) if local_workers else delta[:0]
        if not (cfg.noising and self.sigma > 0 and local_workers):
            return delta
        ids = [noisers[w] for w in local_workers]
        assert all(0 <= j < self.N for row in ids for j in row), "noiser id out of range"
        sc = h2d(self._noise_scales(noisers, local_workers), torch.float32, self.dev)
        if cfg.noise_independent:
            # ablation (not the reference): every (worker, noiser slot) draws its own vector, so no two
            # workers share noise -- isolates the effect of the noisers' shared pre-sampled vectors
            nn_ = len(ids[0]) if ids else 0
            nz = h2d([[self.N + w * nn_ + j for j in range(nn_)] for w in local_workers], torch.int32, self.dev)
            return K.dp_noise(delta, nz, sc, cfg.seed, it, table=None)
        nz = h2d(ids, torch.int32, self.dev)
        tbl = self.noise_rows.table if self.noise_rows is not None else None
        return K.dp_noise(delta, nz, sc, cfg.seed, it, table=tbl)

    # ------------------------------------------------------------------ committee Multi-Krum
    def _xrow_list(self, xrow) -> list:
        """peer -> row of the mapping xrow as a list (-1: no row), built once per mapping (RoundFSM.spec_plan)."""
        c = getattr(self, "_xrow_l", None)
        if c is None or c[0] is not xrow:
            xl = [-1] * self.N
            for p, r in xrow.items():
                xl[p] = r
            c = self._xrow_l = (xrow, xl)
        return c[1]

    def _krum_static(self, xrow, U, plan, live, inboxes, spec, arrivals=None) -> dict:
        """The part of a Krum launch that does not depend on the noisers (inbox rows, leader arrival
        ranks, speculative MSM row -> Krum row), uploaded in ONE copy.  run_round prepares it while
        the host still waits for the VRF outputs."""
        fsm = self.fsm
        vs = [v for v in plan.verifiers if v in inboxes]
        n = len(inboxes[vs[0]])
        # peer -> row of xrow as an array (-1: no row), built once per xrow mapping: the lookups below are
        # numpy gathers instead of per-element dict lookups on the round's host thread
        key = id(xrow)
        cached = getattr(self, "_xrow_np", None)
        if cached is None or cached[0] != key or cached[1] is not xrow:
            xa = np.full(self.N, -1, np.int64)
            xa[np.fromiter(xrow.keys(), np.int64)] = np.fromiter(xrow.values(), np.int64)
            cached = self._xrow_np = (key, xrow, xa)
        xa = cached[2]
        live_np = np.asarray(live, bool)
        inbox_np = xa[np.asarray([inboxes[v] for v in vs], np.int64)].astype(np.int32)
        rank = np.full(U, -1, np.int32)
        arr = np.asarray(arrivals if arrivals is not None else fsm.leader_arrivals(), np.int64)
        ok = live_np[arr] & (xa[arr] >= 0)
        rank[xa[arr[ok]]] = np.nonzero(ok)[0].astype(np.int32)
        ups = [(inbox_np, torch.int32), (rank, torch.int32)]
        if spec is not None:
            # speculative row -> selection row; -1 for rows that are no live worker (the pre-step's MSM
            # covers every local peer): their flags are cleared, so neither the MSM nor the sums use them
            wk = np.zeros(self.N, bool)
            pw = np.asarray(plan.workers, np.int64)
            wk[pw[live_np[pw]]] = True
            sw = np.asarray(spec[0], np.int64)
            src = np.where(wk[sw] & (xa[sw] >= 0), xa[sw], -1).astype(np.int32)
            ups.append((src, torch.int32))
        got = h2d_many(ups, self.dev)
        return {"U": U, "n": n, "clip": fsm.krum_clip(n), "need": len(plan.verifiers) // 2,
                "cap": fsm.leader_cap_size(), "inbox": got[0], "rank": got[1],
                "amap": got[2] if spec is not None else None}

    def _launch_krum(self, X, xrow, plan, live, inboxes, spec, box, pre=None, nz=None, sc=None, static=None):
        """Queue the committee's Multi-Krum (one Gram over the candidate rows X, every live verifier's
        selection on its own inbox, the >= floor(nv/2) vote and the leader's arrival cap) and, behind
        it, the device-side follow-up of the selection (_on_accept).  xrow: worker -> row of X.
        pre: the phase-1 Gram of _gram_rows (X is then None: the noised rows are assembled from it with
        the noisers' ids nz and weights sc, [U1, nn] device tensors).  Returns the callable giving
        (acc, node)."""
        U = X.shape[0] if X is not None else pre["U1"]
        st = static if static is not None and static["U"] == U else self._krum_static(xrow, U, plan, live, inboxes, spec)
        n, clip, need, cap = st["n"], st["clip"], st["need"], st["cap"]
        on_accept, flags = self._on_accept(spec, st["amap"], plan, live, box)
        if self.gpu and spec is not None and getattr(spec[1], "ev_flags", None) is not None:
            # the speculative rows' flags are set (side stream) before the selection writes them
            S.current().wait_event(spec[1].ev_flags)
        if pre is not None:
            if "ev" in pre and self.gpu:   # produced on the Gram stream
                S.current().wait_event(pre["ev"])
            box["flags_set"] = flags is not None
            return K.krum_committee_noise_async(pre, nz, sc, st["inbox"], n - clip, n - clip, need, st["rank"], cap,
                                                on_accept=on_accept, flags=flags)
        return K.krum_committee_async(X, st["inbox"], n - clip, n - clip, need, st["rank"], cap, on_accept=on_accept)

    def _on_accept(self, spec, amap_t, plan, live, box):
        """Device-side follow-up of the committee's selection: this rank's share rows' flags become the
        leader's block mask (rows outside it are cancelled) and the aggregation of the kept rows is
        queued -- on EVERY rank, with or without local rows, so the aggregation's collective lines up;
        its handle lands in box['sa'].  amap_t: device int32 [n speculative rows], speculative row -> Krum
        row (-1: dropped).  Returns (on_accept, flags): flags = (amap, alive) when the selection kernel
        itself should set the rows' flags (the fused native path), else None."""
        sp = spec[1] if spec is not None else None
        pred = self._predict_miners(plan, live) if self.gpu and self.cfg.secure_agg else None
        # the native aggregation behind the selection: every GPU round with a predictable miner layout and local
        # speculative rows (one rank) or any rows at all (several ranks: the collective lines up on every rank);
        # the rest takes the host-decided path after the approvals
        fused = pred is not None and self._native is not None and (sp is not None or self.comm.world > 1)

        def on_accept(node):
            with self.timer.phase("verify.queue_agg"):
                if fused:
                    # the round's iteration and the model it starts from: a speculative front runs before the
                    # previous block is committed (engine._spec_front_launch)
                    box["sa"] = self._spec_aggregate_native(sp, pred, node, amap_t, box.get("flags_set", False),
                                                            it=plan.iteration, W=box.get("W"))
                elif sp is not None:   # no aggregate behind the selection: cancel the rows the block drops
                    B.set_alive(node, amap_t, sp.alive)
                    sp.launch()
        # the fused path lets the noise-aware Krum's vote kernel set the speculative rows' flags itself
        flags = (amap_t, sp.alive) if fused and sp is not None and amap_t is not None else None
        return on_accept, flags

    def _verify(self, X: torch.Tensor, inbox: list, it: int, verifier: int) -> list[bool]:
        """One verifier's decision on its inbox rows X: RONI (VerifyUpdateRONI, main.go:191-233) or a
        stand-alone Krum (the committee path covers KRUM in run_round)."""
        cfg = self.cfg
        n = len(inbox)
        if cfg.defense == "RONI":
            # accept iff the update raises the verifier's training error by at most 0.02 (always accept
            # in the collusion experiment)
            if cfg.colluders > 0:
                return [True] * n
            base = self.task.train_error(self.W, verifier, it)
            return [self.task.train_error(self.W + X[i].double(), verifier, it) - base <= 0.02 for i in range(n)]
        clip = self.fsm.krum_clip(n)
        acc, _ = K.krum(X, n - clip, n - clip)
        return [bool(a) for a in acc.cpu().tolist()]

    # ------------------------------------------------------------------ the verification phase
    def _vgather(self):
        """The packed verification gather (ops/gather.py) for several ranks on GPUs with the noise-aware Krum,
        when its kernels' argument blocks hold this layout; None otherwise (the tensor path below)."""
        vg = self.__dict__.get("_vg")
        if vg is None:
            vg = False
            if self.gpu and self.comm.world > 1 and self._noise_krum():
                from ..ops.gather import VerifyGather

                nn_ = self.cfg.num_noisers
                if VerifyGather.fits(self.maxlocal, nn_, self.N):
                    U = self.comm.world * self.maxlocal + self.N
                    _, _, chunk, npairs = K.gram_split(U, self.comm.rank, self.comm.world)
                    vg = VerifyGather(self.comm, self.maxlocal, self.crypto.point_width, nn_, chunk, npairs, self.N,
                                      self.dev)
            self._vg = vg
        return vg or None

    def _gather_verify_packed(self, vg, head: dict, noisers: dict):
        """_gather_verify_inputs with the packed row: one pack kernel, the in-place all_gather, one unpack
        kernel (the workers' commitment rows land in pinned memory)."""
        pre = head["krum_pre"]
        nz_np, sc_np = self._noise_ids_np(noisers, head["local_workers"])
        if head["local_workers"]:
            rows = self.crypto.commit_rows_tensor(head["pending_commits"]).to(self.dev)
        else:   # no local worker this round (committee members, churn): every slot of the row is zeros
            rows = torch.zeros((1, self.crypto.point_width), dtype=torch.int32, device=self.dev)
        # slot j (local peer lo + j) -> its commitment row; the round's workers' flat rows: numpy gathers through
        # tables built once (no per-element Python loop on the round's thread)
        lw = np.asarray(head["local_workers"], np.int64)
        src = np.full(self.maxlocal, -1, np.int32)
        if lw.size:
            # the pre-step's rows are the local peers themselves (head.py: row_of = {w: w - lo})
            src[lw - self.lo] = (lw - self.lo) if head.get("row_is_slot") else \
                np.fromiter((head["row_of"][w] for w in head["local_workers"]), np.int64, lw.size)
        flat = self.__dict__.get("_flat_np")
        if flat is None:
            flat = self._flat_np = np.asarray([self.flat[p] for p in range(self.N)], np.int32)
        if self.gpu and "ev" in pre:   # the Gram slot is written on the Gram stream
            S.current().wait_event(pre["ev"])
        gram, nz, sc, host, ev = vg.exchange(pre["it"], rows.contiguous(), src, nz_np, sc_np,
                                             flat[np.asarray(head["workers"], np.int64)])
        pre["gram"] = gram
        pre.pop("split", None)
        head["commit_gather"] = (host, ev)
        return nz, sc

    def _gather_verify_inputs(self, head: dict, noisers: dict):
        """Several ranks, noise-aware Krum: ONE all_gather of every rank's [commitment rows | noiser ids
        | noiser weights] in the flat layout (each rank computed only its own workers' VRF outputs), the
        commitments' read-back queued right behind it.  Returns (nz, sc) [U1, nn] on the device."""
        pre = head.get("krum_pre")
        if pre is not None and pre.get("packed"):
            return self._gather_verify_packed(self._vgather(), head, noisers)
        nz_np, sc_np = self._noise_ids_np(noisers, head["local_workers"])
        nz_l, sc_l = h2d_many([(nz_np, torch.int32), (sc_np, torch.float32)], self.dev)
        parts = [self._local_commit_buf(head), nz_l, sc_l]
        pre = head.get("krum_pre")
        split = pre is not None and "split" in pre
        if split:
            # this rank's share of the Gram's tiles rides along (computed on the Gram stream)
            if self.gpu and "ev" in pre:
                S.current().wait_event(pre["ev"])
            parts.append(K.gram_slot(pre))
        got = self.comm.all_gather_packed(parts)
        if split:
            K.gram_adopt(pre, got[3])
        pw, nn_ = self.crypto.point_width, self.cfg.num_noisers
        g_commit = got[0].reshape(-1, pw)
        rows = g_commit.index_select(0, h2d([self.flat[w] for w in head["workers"]], torch.long, self.dev))
        if self.gpu:
            # (depth 4: the deferred signing reads these rows in the next round's VRF wait, commit_of.jac)
            host = pinned("commit_gather", rows.shape, rows.dtype, depth=4)
            d2h_into(host, rows.contiguous())
            head["commit_gather"] = (host, S.record())
        else:
            head["commit_gather"] = (rows, None)
        return got[1].reshape(-1, nn_).contiguous(), got[2].reshape(-1, nn_).contiguous()

    @staticmethod
    def _finish_verification(ver) -> dict:
        """The result of _verification_steps: ver is the stopped generator (resumed to its end here) or the
        StopIteration that already carries the result."""
        if isinstance(ver, StopIteration):
            return ver.value
        try:
            while True:
                next(ver)
        except StopIteration as done:
            return done.value

    def _verification_steps(self, head: dict, noisers: dict, noised, kst):
        """The verifier committee's decisions and signatures for this round, as a generator that stops once
        right after the Multi-Krum launch (the committee's selection and the aggregation behind it are queued on
        the device; engine._round_front can start a round this far ahead) and returns (StopIteration.value)
        approved workers, the commitment table, signatures (where a consumer reads them), the device
        aggregation box and the deferred signature join."""
        cfg, R, fsm, comm, tm = self.cfg, self.R, self.fsm, self.comm, self.timer
        plan, live, it = head["plan"], head["live"], head["plan"].iteration
        workers, local_workers, inboxes = head["workers"], head["local_workers"], head["inboxes"]
        row_of, spec, krum_pre = head["row_of"], head["spec"], head.get("krum_pre")
        pending_commits, fut_noise = head["pending_commits"], head["fut_noise"]
        self._cur_commits = pending_commits   # the early audit sums read its per-chunk commitments
        single = comm.world == 1
        commit_of = _CommitTable()
        g_commit = g_noised = g_delta = g_ts = None
        need_X = cfg.verification and bool(inboxes)
        noise_aware = krum_pre is not None

        def _materialize_commits():  # bound lazily: the first reader (signing or block) waits for the copy
            if commit_of.bound():
                return
            if single:
                if local_workers:
                    commit_of.fill_lazy(pending_commits.result, row_of)
                    if getattr(pending_commits, "value", 1) is None and getattr(pending_commits, "host", None) is not None:
                        commit_of.jac = (pending_commits.host, pending_commits.event)
            elif head.get("commit_gather") is not None:   # gathered with the noisers (noise-aware path)
                host, ev = head["commit_gather"]

                def load(host=host, ev=ev):
                    if ev is not None:
                        S.host_wait(ev)
                    return self.crypto.marshal_rows(host)
                commit_of.fill_lazy(load, {w: i for i, w in enumerate(workers)})
                if self.gpu and ev is not None:
                    # the gathered rows are device-layout Jacobian points: the block build and the signing marshal
                    # only the rows they use, natively (as with one rank's pre-step commitments)
                    commit_of.jac = (host, ev)
            elif workers:   # every worker's commitment: one batched marshal of the gathered rows
                sel = h2d([self.flat[w] for w in workers], torch.long, self.dev)
                commit_of.fill(self.crypto.marshal_rows(g_commit.index_select(0, sel)),
                               {w: i for i, w in enumerate(workers)})

        nz = sc = None
        if noise_aware and need_X and cfg.defense == "KRUM":
            if single:
                nz_np, sc_np = self._noise_ids_np(noisers, local_workers)
                if self.gpu and K.noise_tables_by_value(nz_np.size, len(next(iter(inboxes.values()), []))):
                    nz, sc = nz_np, sc_np   # host tables: they ride in the Krum kernel's arguments (no upload)
                else:
                    nz, sc = h2d_many([(nz_np, torch.int32), (sc_np, torch.float32)], self.dev)
            else:
                nz, sc = self._gather_verify_inputs(head, noisers)
        elif not single:
            # ONE all_gather carries every rank's commitments (device Jacobian rows), noised deltas (the
            # verifiers' input) and, on the plain path, deltas (the block payload) and clocks
            cr = self.crypto
            parts = [self._local_commit_buf(head)]
            if need_X or not cfg.secure_agg:
                parts.append(self._rows_buffer(noised, local_workers, self.d, torch.float32))
            if not cfg.secure_agg:
                parts.append(self._rows_buffer(self._worker_rows(head["delta"], row_of, local_workers)
                                               if local_workers else None, local_workers, self.d, torch.float32))
                # + each rank's clock: every rank builds the plain block with the leader's timestamp
                parts.append(torch.full((self.maxlocal, 1), self._now(it), dtype=torch.int64, device=self.dev))
            got = comm.all_gather_packed(parts)
            g_commit = got[0].reshape(-1, cr.point_width)
            g_noised = got[1].reshape(-1, self.d) if len(got) > 1 else None
            g_delta = got[2].reshape(-1, self.d) if len(got) > 2 else None
            g_ts = got[3][:, 0, 0] if len(got) > 3 else None
        if cfg.colluders > 0:  # privacy experiment bookkeeping (isCollusionAttack, main.go:1026-1057)
            thr = self.pc.collusion_thresh
            if any(v >= thr for v in plan.verifiers):
                self.stats["unmasked_updates"] += sum(1 for w in local_workers if all(j >= thr for j in noisers[w]))
        accepted_map: dict = {}
        signatures: dict = {}
        pending_signatures = None
        defer_sign = False
        box: dict = {"W": head.get("W")}   # W: set by a speculative front (the block it starts from is not committed)
        if need_X:
            vs = [v for v in plan.verifiers if v in inboxes]   # live verifiers, plan order
            nv = len(plan.verifiers)
            ni = len(inboxes[vs[0]])
            X, xrow = (noised, {w: i for i, w in enumerate(local_workers)}) if single else (g_noised, self.flat)
            if noise_aware:
                X, xrow = None, krum_pre["xrow"]
            if cfg.defense == "KRUM":
                # Multi-Krum is a pure function of the (gathered) noised deltas, so every rank evaluates the
                # whole committee itself (identical inputs, deterministic kernels)
                with tm.phase("verify.defense"):
                    wait = self._launch_krum(X, xrow, plan, live, inboxes, spec, box, pre=krum_pre, nz=nz, sc=sc,
                                             static=kst)
                yield "launched"
                with tm.phase("verify.defense"), tm.phase("verify.krum_wait"):
                    acc_t, node_t = wait()
                acc_np = acc_t.numpy().astype(np.uint8)   # [len(vs), ni]
                acc_row = {v: k for k, v in enumerate(vs)}
                if box.get("sa") is not None:   # the rows the device aggregation kept
                    node_np = node_t.numpy()
                    xc = getattr(self, "_xrow_np", None)
                    if xc is not None and xc[1] is xrow:   # numpy gather (the _krum_static table)
                        wk = np.asarray(workers, np.int64)
                        kept = set(wk[node_np[xc[2][wk]].astype(bool)].tolist())
                    else:
                        kept = {w for w in workers if node_np[xrow[w]]}
                    # a block row outside the (replicated) speculative candidates was never computed: the
                    # device aggregate is then incomplete and the host path tops it up
                    if not kept <= head["spec_cand"]:
                        kept = None
                        self.stats["spec_misses"] = self.stats.get("spec_misses", 0) + 1
                    box["sa"]["accepted"] = kept
            elif cfg.defense == "LSH":
                # LSH sieve (logistic_aggregator.py:7-29): like Krum a pure function of the (gathered)
                # noised updates, so every rank evaluates every verifier's inbox itself
                from ..ops.lsh import sieve_accept

                with tm.phase("verify.defense"):
                    acc_np = sieve_accept(X, [[xrow[w] for w in inboxes[v]] for v in vs], self.d,
                                          seed=self.fsm.round_seed(13)).astype(np.uint8)
                acc_row = {v: k for k, v in enumerate(vs)}
            else:
                # RONI: each verifier judges with its own data, so only its rank can decide; the accept
                # matrix [nv, ni] travels in one all_gather on several ranks
                mine = np.zeros((nv, ni), np.uint8)
                for v in vs:
                    if v in self.local:
                        rows_v = h2d([xrow[w] for w in inboxes[v]], torch.long, self.dev)
                        with tm.phase("verify.defense"):
                            ok = self._verify(X.index_select(0, rows_v), inboxes[v], it, v)
                        mine[plan.verifiers.index(v)] = np.asarray(ok, np.uint8)
                if single:
                    allm = mine
                else:
                    allm = comm.all_gather(torch.from_numpy(mine).to(self.dev)).cpu().numpy()
                    allm = np.stack([allm[comm.owner(v, self.N), plan.verifiers.index(v)] for v in plan.verifiers])
                acc_np = np.stack([allm[plan.verifiers.index(v)] for v in vs])
                acc_row = {v: k for k, v in enumerate(vs)}
            # vectorised over the [verifier, inbox slot] matrix (no per-element Python loop)
            inbox_arr = np.asarray([inboxes[v] for v in vs], np.int64)
            acc_b = np.asarray([acc_np[acc_row[v]] for v in vs], bool)
            for k, v in enumerate(vs):
                accepted_map[v] = inbox_arr[k][acc_b[k]].tolist()
            # the local verifiers sign their accepted commitments on native threads while the GPU computes
            # shares (main.go:1120-1140).  On the secure path nothing in the round reads the signatures
            # (Q5): their batch yields the host threads to the next round's VRF outputs and is joined one
            # round later; plain blocks carry them and --verify-signatures checks them, so there they are
            # joined before the block.
            defer_sign = (self._pipelined() and cfg.secure_agg and not cfg.verify_signatures
                          and fut_noise is not None)
            lk = [k for k, v in enumerate(vs) if v in self.local]
            local_vs = [vs[k] for k in lk]
            sig_np = np.zeros((nv, ni, 64), np.uint8)
            sign = {"prep": None, "job": None, "sl": None}
            if local_vs:
                _materialize_commits()
                rowmap = commit_of.row
                acc_l, inb_l = acc_b[lk], inbox_arr[lk]
                vidx = np.asarray([plan.verifiers.index(v) for v in local_vs], np.int64)
                sks = [self.sk[v] for v in local_vs]
                nonce_keys = [(v, it) for v in local_vs]

                def _prep_sign(after_vrf=None, sign=sign, threads=SIGN_THREADS):
                    # message i = row rows[i] of the commitment table, signed with sks[key_of[i]], nonce id =
                    # the worker; (sl_v, sl_j) = its (verifier, inbox slot) in the signature matrix
                    from .engine import _seed_bytes

                    sign["prep"] = None
                    kk, jj = np.nonzero(acc_l)            # (local verifier, inbox slot) of each signature
                    if kk.size:
                        ws = inb_l[kk, jj]
                        rmap = np.full(self.N, -1, np.int64)
                        rmap[list(rowmap)] = list(rowmap.values())
                        bases = [_seed_bytes(cfg.seed, f"nonce-{i}", v) for v, i in nonce_keys]
                        sign["sl"] = (vidx[kk], jj)
                        jac = getattr(commit_of, "jac", None)
                        if jac is not None and commit_of._table is None:
                            # the commitments are still the pre-step's Jacobian rows: the job marshals the signed
                            # ones on its own thread (the round's thread skips the table's ~30 us marshal)
                            S.host_wait(jac[1])
                            sign["job"] = R.schnorr_sign_rows_jac_async(jac[0].numpy().view(np.uint32),
                                                                        rmap[ws].tolist(), sks, kk.tolist(), bases,
                                                                        ws.tolist(), threads, after_vrf)
                        else:
                            sign["job"] = R.schnorr_sign_rows_async(commit_of.table, rmap[ws].tolist(), sks,
                                                                    kk.tolist(), bases, ws.tolist(), threads, after_vrf)
                sign["prep"] = _prep_sign
                if defer_sign:   # prepared in the next round's VRF wait, started once its outputs are known
                    self._pre_vrf_work.append(_prep_sign)
                else:
                    _prep_sign()

            def _join_signatures(sign=sign, sig_np=sig_np, vs=vs):
                with tm.phase("verify.sign_join"):
                    if sign["prep"] is not None:   # deferred and not prepared yet: start it now
                        self._pre_vrf_work = [f for f in self._pre_vrf_work if f is not sign["prep"]]
                        sign["prep"]()
                    if sign["job"] is not None:
                        sl_v, sl_j = sign["sl"]
                        sig_np[sl_v, sl_j] = sign["job"].result_array()
                    self.last_signatures = sig_np   # [nv, ni, 64]: this rank's verifiers' signatures
                    # the signatures travel to the workers (and on to the miners) only where a consumer
                    # reads them: plain blocks carry them, --verify-signatures checks them; on the secure
                    # path each rank keeps the ones its verifiers produced (Q5) as this matrix
                    if cfg.secure_agg and not cfg.verify_signatures:
                        return
                    gather = not single
                    sig_all = comm.all_gather(torch.from_numpy(sig_np).to(self.dev)).cpu().numpy() if gather \
                        else sig_np[None]
                    for v in vs:
                        if not gather and v not in self.local:
                            continue
                        vi = plan.verifiers.index(v)
                        o = comm.owner(v, self.N) if gather else 0
                        for w in accepted_map[v]:
                            j = inboxes[v].index(w)
                            signatures.setdefault(w, []).append(sig_all[o, vi, j].tobytes())
            pending_signatures = _join_signatures
            if not cfg.secure_agg or cfg.verify_signatures:
                pending_signatures()
                pending_signatures = None
            approved, _ = fsm.approve(accepted_map)
        else:
            approved, _ = fsm.approve({})
        _materialize_commits()
        return {"approved": approved, "commit_of": commit_of, "signatures": signatures, "box": box,
                "pending_signatures": pending_signatures, "defer_sign": defer_sign, "accepted_map": accepted_map,
                "gathered": (g_delta, g_noised, g_ts)}

    def _rows_buffer(self, rows: torch.Tensor | None, local_workers: list, width: int, dtype) -> torch.Tensor:
        """[maxlocal, width] buffer whose row (w - lo) holds local worker w's row of `rows` (given in
        local_workers order)."""
        buf = torch.zeros((self.maxlocal, width), dtype=dtype, device=self.dev)
        if local_workers and rows is not None:
            buf.index_copy_(0, h2d([w - self.lo for w in local_workers], torch.long, self.dev), rows)
        return buf
