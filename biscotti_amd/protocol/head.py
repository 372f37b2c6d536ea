"""Round head: everything a round needs that depends only on the latest block.

A head is opened as soon as the block that seeds it is committed (DistSys/main.go
prepareForNextIteration, :1062-1187): the live set and committee plan (stake lottery on the block
hash, vrf.go:103-182), the workers' noiser VRF outputs (vrf.go:54-100; each rank proves only the
peers it hosts), the local SGD step (client.py:38-65), the full-vector commitments
(honest.go:165-200), the speculative share MSM (kyber.go:484-646) and, for the noise-aware
committee Krum, the Gram of [every peer's delta; the noisers' pre-sampled vectors].

Cross-round pipelining (GPU; off with the ``no_pipeline`` ablation, which must not change the chain):
  * pre-step    the next round's local step + commitments (+ the Gram, gathered across ranks) are
                queued right behind the recovery of the model they start from
  * early VRF   the next round's noiser VRF outputs start when the block is built, before its audit
  * spec head   the next round's share MSM starts when the block is built, from fsm.successor(block)
"""
from __future__ import annotations

import torch

from ..ops import ml as K
from ..utils import h2d, h2d_many
from ..utils import streams as S

SPEC_GROUP_ROWS = 8   # speculative MSM rows per group, in leader arrival order (late cancellation)
# The leader's block closes at its first NUM_SAMPLES/2 approved arrivals (main.go:360): shares of candidates
# further down its arrival order are never aggregated.  The speculative MSM covers the candidates up to a
# horizon in that order -- the leader's cap plus SPEC_MARGIN, and at least SPEC_SLACK past the deepest block
# row of the last SPEC_WINDOW rounds (rejections push the block deeper; every candidate until SPEC_MIN_HISTORY
# blocks are known, more slack while the window fills) -- instead of every candidate (~94 at 100 peers, 2.7x the
# block); a block that reaches past it is topped up by the host path (spec_misses).
SPEC_MARGIN, SPEC_SLACK, SPEC_WINDOW, SPEC_MIN_HISTORY = 16, 8, 8, 3


class PlanView:
    """A native RoundPlan with its fields converted to Python once: every attribute read of the native
    object builds a new list (~1-3 us), and a round reads the plan's lists ~25 times."""

    __slots__ = ("iteration", "verifiers", "miners", "workers", "leader", "live", "done")

    def __init__(self, p):
        self.iteration, self.verifiers, self.miners, self.workers = p.iteration, p.verifiers, p.miners, p.workers
        self.leader, self.live, self.done = p.leader, p.live, p.done


class RoundHeadMixin:
    # ------------------------------------------------------------------ the head
    def _open_round(self, begun: tuple | None = None) -> dict:
        """Round head: live set, committee plan, the VRF outputs and the device work of the round that
        needs nothing but the latest block; consumed by run_round.  begun: (live, PlanView) of a round the FSM
        has begun already (a speculative front that was not adopted, engine._adopt_spec_front)."""
        cfg, R, fsm = self.cfg, self.R, self.fsm
        with self.timer.phase("head.plan"):
            if begun is not None:
                live, plan = begun
            else:
                live = self._live_mask()
                plan = PlanView(fsm.begin_round(live))
        head = {"live": live, "plan": plan}
        if plan.done:
            return head
        latest_hash = fsm.chain.latest_hash()
        workers = [w for w in plan.workers if live[w]]
        local_workers = [w for w in workers if w in self.local]
        # stake None: the noiser lottery reads the FSM's stake natively (unchanged until the block commits)
        head.update(workers=workers, local_workers=local_workers, stake=None)
        # noisers: each worker's own ECVRF over the latest block hash (vrf.go:54-100).  Only the 64-byte
        # outputs gate the round (noiser lottery -> noise -> Krum -> the selection that cancels speculative
        # MSM rows); every rank computes them for the peers it hosts only (the reference: each peer proves
        # its own), on host_threads - 1 native threads; the proofs nothing reads run on the device.
        with self.timer.phase("head.vrf_submit"):
            dev = self.vrf_dev is not None
            nthr = max(1, cfg.host_threads - 1) if self.gpu else cfg.host_threads
            ej, self._early_vrf = self._early_vrf, None
            fut_noise = None
            if ej is not None and local_workers and ej["hash"] == bytes(latest_hash) \
                    and ej["ver"] == getattr(self, "_seed_version", 0):
                # the outputs started when the block was built (_early_vrf_submit) over every local peer with
                # the current keys: adopted
                fut_noise = ej["job"]
                lo = self.lo
                head["vrf_index"] = [w - lo for w in local_workers]
                self.stats["early_vrf"] = self.stats.get("early_vrf", 0) + 1
            if ej is not None and fut_noise is not ej["job"]:
                # not adopted (a failed audit changed the block, or a restart its keys): joined later, not
                # here -- dropping a running job would wait for it
                self._stale_vrf.append(ej["job"])
            if fut_noise is None and local_workers:
                seeds = [self.vrf_noise_seed[w] for w in local_workers]
                fut_noise = R.vrf_prove_batch_async(seeds, latest_hash, nthr, None, dev)
                self.stats["vrf_outputs"] += len(seeds)
            fut_roles = None
            if cfg.roles_vrf_proof and not dev:  # getVRFRoles proves with the roles key too (result unused, Q7)
                roles = [self.vrf_roles_seed[p] for p in self.local if live[p]]
                if roles:
                    fut_roles = R.vrf_prove_batch_async(roles, latest_hash, 8, fut_noise)
        head.update(fut_noise=fut_noise, fut_roles=fut_roles)
        tm, it = self.timer, plan.iteration
        # the local step (and the commitments) may already be in flight: the native pre-step queued behind the
        # recovery of the model this head starts from, for every local peer.  The decision is the same on every
        # rank (the pre-step is queued at the same point everywhere): the Gram gather depends on it.
        pre, self._pre = self._pre, None
        use_pre = pre is not None and pre["it"] == it and pre["W"] is self.W
        with tm.phase("local_step"):
            if use_pre:
                self.stats["pre_steps"] = self.stats.get("pre_steps", 0) + 1
                S.current().wait_event(pre["ev"])   # the step ran on the Gram stream
                delta, qdelta = pre["delta"], pre["qdelta"]          # rows: every local peer
                row_of = {w: w - self.lo for w in local_workers}
            else:
                delta, qdelta = self.task.step(self.W, it, local_workers)
                row_of = {w: i for i, w in enumerate(local_workers)}
        with tm.phase("commit"):
            # every live verifier collects its own first krum_thresh arrivals (krum.go:284-322); only updates
            # that can end in the leader's block secret-share: the MSM runs speculatively on the CU-masked
            # side stream over every candidate, in leader arrival order, and the committee's selection
            # cancels the rows it rejects
            inboxes = {}
            sn, self._spec_next = self._spec_next, None
            if sn is not None and not (use_pre and pre is sn["pre"] and sn["hash"] == bytes(latest_hash)
                                       and sn["it"] == it and sn["verifiers"] == list(plan.verifiers)
                                       and sn["miners"] == list(plan.miners) and sn["workers"] == workers
                                       and all(live)):
                sn = None   # the committed block or the plan differs: the speculative MSM is not used
            if sn is not None:
                inboxes = sn["inboxes"]
            elif cfg.verification:
                for v, ib in zip(plan.verifiers, fsm.verifier_inboxes(workers)):
                    if live[v]:
                        inboxes[v] = list(ib)
            spec = None
            cand = set()
            if sn is not None:
                # launched at the previous block's build (_spec_head_launch), from this very plan
                cand, spec, head["arrivals"], head["cand_order"] = sn["cand"], sn["spec"], sn["arrivals"], sn.get("cand_order")
                if sn.get("kst") is not None:
                    head["kst"] = sn["kst"]   # Krum's static tables, built in the previous round's audit wait
                self.stats["spec_head"] = self.stats.get("spec_head", 0) + 1
            elif self.gpu and cfg.secure_agg:
                # replicated on every rank: the rows (of all ranks) whose shares are computed up front
                cand = self._block_candidates(plan, workers, inboxes)
                if local_workers:
                    arrivals = head["arrivals"] = fsm.leader_arrivals()   # once per round (Krum reuses it)
                    lo_rank = {w: i for i, w in enumerate(arrivals)}
                    spec_workers = sorted((w for w in local_workers if w in cand),
                                          key=lambda w: lo_rank.get(w, 1 << 30))
                    if spec_workers:
                        spec = (spec_workers, self.crypto.shares_async(qdelta, [row_of[w] for w in spec_workers],
                                                                       self.side_stream,
                                                                       group_rows=SPEC_GROUP_ROWS))
            # full-vector commitments on the background stream: their first consumer is the signing after
            # Krum, so noise + Krum on the main stream do not queue behind them
            pending_commits = pre["commits"] if use_pre else \
                self.crypto.commitments_async(qdelta, self.bg_stream if self.gpu else None)
        # noise-aware committee Krum: the d-dimensional part (the Gram of every peer's delta stacked over
        # the noisers' pre-sampled vectors of this iteration) depends only on this head, so it runs while
        # the host computes the VRF outputs; after the noisers are known only an O(n^2) assembly remains
        krum_pre = None
        if self._noise_krum() and inboxes and workers:   # replicated condition (the Gram gathers)
            with tm.phase("verify.pregram"):
                krum_pre = pre.get("gram") if use_pre else None
                if krum_pre is None:
                    # the pre-step's delta holds every local peer (no row selection needed)
                    krum_pre = self._gram_rows(delta, None if use_pre else row_of, it)
        head.update(delta=delta, qdelta=qdelta, pending_commits=pending_commits, inboxes=inboxes, row_of=row_of,
                    row_is_slot=use_pre, spec=spec, spec_cand=cand, krum_pre=krum_pre)
        if self.vrf_dev is not None:
            # the proofs nobody reads -- every noiser proof and the roles proofs -- go to the device prover
            # when the round runs (run_round's VRF wait), one launch per round on their own low-priority
            # stream: a timed window then contains exactly its rounds' proofs
            head["vrf_proofs"] = (local_workers, live, bytes(latest_hash))   # key rows built at the submit
        return head

    def _vrf_key_rows(self, local_workers: list, live) -> "np.ndarray":
        """The device prover's key rows of this round's proofs: every local worker's noiser proof, then every
        live local peer's roles proof (getVRFRoles, Q7) -- from per-peer row tables built once per key
        version (a churn restart draws new keys) instead of per-seed lookups every round."""
        import numpy as np

        ver = getattr(self, "_seed_version", 0)
        tab = getattr(self, "_vrf_rows_tab", None)
        if tab is None or tab[0] != ver:
            peers = list(self.local)
            tab = self._vrf_rows_tab = (ver, np.asarray(self.vrf_dev._rows([self.vrf_noise_seed[p] for p in peers]),
                                                        np.int32),
                                        np.asarray(self.vrf_dev._rows([self.vrf_roles_seed[p] for p in peers]), np.int32))
        lo = self.lo
        parts = [tab[1][np.asarray(local_workers, np.int64) - lo]] if local_workers else []
        if self.cfg.roles_vrf_proof:
            lv = np.asarray(live, bool)[lo:lo + len(self.local)]
            parts.append(tab[2][lv])
        return np.concatenate(parts) if parts else np.zeros(0, np.int32)

    def _block_candidates(self, plan, workers, inboxes) -> set:
        """Workers whose update can end in this round's block: without verification every live worker
        (capped to the leader's first arrivals); with it, every update some live verifier judges -- or
        every live worker when floor(nv/2) == 0 signatures suffice (the nv = 1 quirk, main.go:1686:
        updates no verifier saw are approved too)."""
        if not self.cfg.verification:
            return set(self.fsm.leader_cap(workers))
        if len(plan.verifiers) // 2 == 0:
            return set(workers)
        out: set = set()
        for ib in inboxes.values():
            out.update(ib)
        return out

    # ------------------------------------------------------------------ noise-aware Krum, phase 1
    def _noise_krum(self) -> bool:
        """The noise-aware committee Krum applies: every worker's noised update is its delta plus the mean
        of its noisers' pre-sampled vectors (client_obj.py:97-98), so Krum's Gram can be taken over
        [deltas; noise vectors] before the noisers are known.  Same answer on every rank."""
        cfg = self.cfg
        return bool(cfg.secure_agg and cfg.verification and cfg.defense == "KRUM" and cfg.noising
                    and self.sigma > 0 and cfg.num_noisers >= 1 and self.noise_rows is not None
                    and not cfg.noise_independent and self.comm.world * self.maxlocal + self.N <= K.KRUM_MAX_ROWS)

    def _gram_rows(self, delta: torch.Tensor, row_of: dict | None, it: int) -> dict:
        """Phase 1 of the noise-aware committee Krum over the flat peer layout: row r * maxlocal + j is
        rank r's j-th peer (self.flat), then the N noise rows of this iteration.  delta holds every
        local peer (row_of None, the pre-step) or the rows row_of names.  Several ranks: ONE all_gather
        of the [maxlocal, d] delta buffers (called at the same point on every rank)."""
        ml, d = self.maxlocal, self.d
        if row_of is None and delta.shape[0] == ml:
            buf = delta
        else:
            buf = torch.zeros((ml, d), dtype=torch.float32, device=self.dev)
            if row_of is None:
                buf[: delta.shape[0]] = delta
            elif row_of:
                ws = list(row_of)
                src = delta if [row_of[w] for w in ws] == list(range(delta.shape[0])) else \
                    delta.index_select(0, h2d([row_of[w] for w in ws], torch.long, self.dev))
                buf.index_copy_(0, h2d([w - self.lo for w in ws], torch.long, self.dev), src)
        comm = self.comm
        X = comm.all_gather(buf).reshape(-1, d) if comm.world > 1 else buf
        # several ranks: each computes 1/world of the Gram's tile pairs; the tiles travel with the
        # commitments + noiser ids in the verification all_gather (_gather_verify_inputs) -- on a GPU written
        # straight into this rank's row of the packed gather buffer (ops/gather.py)
        vg = self._vgather() if comm.world > 1 else None
        if vg is not None and S.current().stream_id != self.gram_stream.stream_id:
            # a discarded pre-step may still write this iteration's slot on the Gram stream
            S.wait(S.current(), self.gram_stream)
        nn = self._noise_gram_table()
        g = K.gram_stacked_async(X.contiguous(), self.noise_rows.rows(it),
                                 split=(comm.rank, comm.world) if comm.world > 1 else None,
                                 out=vg.gram_out(it) if vg is not None else None,
                                 nn=nn[it % 100] if nn is not None else None)
        g["xrow"] = self.flat
        g["it"] = it
        return g

    def _noise_gram_table(self):
        """GPU: the [100, N, N] Gram of each iteration's noise rows (NoiseRows.gram_table, built at setup), whose
        tiles the noise-aware Gram copies instead of computing; None on the CPU or with the
        noise_gram_each_round ablation."""
        if not (self.gpu and self.noise_rows is not None and self.noise_rows.table is not None) or \
                self.cfg.has("noise_gram_each_round"):
            return None
        return self.noise_rows.gram_table()

    # ------------------------------------------------------------------ cross-round pipelining
    def _pipelined(self) -> bool:
        return self.gpu and not self.cfg.has("no_pipeline")

    def _native_prestep_ok(self) -> bool:
        """The pre-step runs natively (NativeSecAgg, softmax tasks); the task and the slot ring are bound at the
        first use."""
        na = self._native
        if na is None or type(self.task).__name__ != "SoftmaxTask":
            return False
        if na.task is None:
            gs = self.gram_stream
            with S.use(gs):
                cnt = K._tile_counters(self.dev, 1024)
            # the noise table drives the pre-step's own Gram (one rank) or the multi-rank call's (_multi_gram)
            nk = self._noise_krum() and (self.comm.world == 1 or self._multi_gram)
            na.bind_task(self.task, gs, self.noise_rows.table if nk else None, cnt)
            if nk:
                na.set_nn_table(self._noise_gram_table())
        return True

    def _finish_pre(self, out: dict, it: int) -> dict:
        """A native pre-step's Gram: one rank -- computed in the call (its row map added here); several ranks --
        the deltas' all_gather and this rank's share of the Gram's tiles, on the Gram stream behind the step
        (every rank gets here at the same point of the round)."""
        if not self._noise_krum():
            out.pop("gram", None)
            return out
        if self.comm.world == 1:
            out["gram"]["xrow"] = self.flat
        else:
            with S.use(self.gram_stream):
                g = self._gram_rows(out["delta"], None, it)
                g["ev"] = S.record()
            out["gram"] = g
        return out

    def _spec_head_launch(self, block) -> None:
        """Launch the next round's speculative share MSM as soon as the block that seeds the next plan is
        built, before its audit is read and it is committed: the plan, inboxes and leader arrival order
        come from fsm.successor(block) (the FSM as it will be after the commit).  The MSM reads the
        pre-step's quantised updates (it waits for the step only, not for the audit).  The next head
        adopts it when the committed block and its plan match (they do unless the audit fails).  Local
        work only (no collective): each rank launches its own peers' rows."""
        cfg, pre = self.cfg, self._pre
        if self._shared_device and not cfg.has("spec_head_shared"):
            # several ranks on one GPU (rehearsals): speculative work only pays when the GPU would idle, and
            # here the other ranks' critical paths fill it (2-rank RCCL rehearsal: 14.6 vs 3.6 ms/round);
            # the spec_head_shared ablation forces it (the multi-rank GPU tests run the one-rank-per-GPU path)
            return
        if not (self._pipelined() and cfg.secure_agg and cfg.verification and cfg.churn == 0
                and cfg.churn_kill_per_min == 0 and not self._partitions and pre is not None
                and pre["W"] is self._W_next and self.local):
            return
        # successor FSM, its plan, inboxes, leader arrivals and this rank's candidates in arrival order: one
        # native call (RoundFSM.spec_plan)
        g = pre.get("gram")
        krum = g is not None and cfg.defense == "KRUM"
        # with the noise-aware Krum input, the same call also returns Krum's static tables (verify.py
        # _krum_static) for the successor plan: they go up in one copy below, off the next round's path
        # the candidates up to the horizon in the leader's arrival order (replicated on every rank)
        got = self.fsm.spec_plan(block, self.local.start, self.local.stop,
                                 self._xrow_list(g["xrow"]) if krum else [], g["U1"] if krum else 0,
                                 self._spec_horizon())
        if got is None:
            return
        plan, ibs, arrivals, spec_workers, cands = got[:5]
        order = got[-1]
        if not spec_workers and self.comm.world == 1:
            return
        # several ranks: the successor plan is kept even without local rows to launch (spec None), so every rank
        # makes the same speculative-front decision (engine._spec_front_launch: its collectives line up)
        sp = self._spec_msm_launch(pre, spec_workers) if spec_workers else None
        if not spec_workers:
            self.stats["spec_head_no_rows"] = self.stats.get("spec_head_no_rows", 0) + 1
        plan = PlanView(plan)
        workers = plan.workers
        inboxes = dict(zip(plan.verifiers, ibs))
        cand = set(cands)
        self._spec_next = {"plan": plan, "hash": bytes(block.hash), "it": plan.iteration, "verifiers": list(plan.verifiers),
                           "miners": list(plan.miners), "workers": workers, "inboxes": inboxes, "cand": cand,
                           "arrivals": arrivals, "spec": (spec_workers, sp) if spec_workers else None, "pre": pre,
                           "cand_order": order}
        if krum and ibs:
            n = len(ibs[0])
            up = h2d_many([(got[5], torch.int32), (got[6], torch.int32), (got[7], torch.int32)], self.dev)
            self._spec_next["kst"] = {"U": g["U1"], "n": n, "clip": self.fsm.krum_clip(n),
                                      "need": len(plan.verifiers) // 2, "cap": self.fsm.leader_cap_size(),
                                      "inbox": up[0], "rank": up[1], "amap": up[2]}

    def _spec_msm_launch(self, pre: dict, spec_workers: list):
        """The speculative share MSM over this rank's candidate rows (in the leader's arrival order) on the side
        stream, behind the pre-step that produced them."""
        cfg = self.cfg
        side = self.side_stream
        # the audit's commitment sums come from the pre-step's chunk commitments (the early audit sums of NativeSecAgg.after_select):
        # the MSM then computes the witness lanes only
        no_commit = getattr(pre["commits"], "ccom", None) is not None and cfg.kzg_audit == "off"
        lo = self.lo
        rows = [w - lo for w in spec_workers]
        self.stats["spec_rows"] = self.stats.get("spec_rows", 0) + len(rows)   # speculative MSM rows launched
        if self._native is not None:
            # one native call: wait for the step, launch with the rows in the kernel's arguments (resident output
            # ring); the plan's Python views are built after the launch
            sp = self._native.spec_msm(pre["qdelta"], rows, pre["ev"], no_commit, SPEC_GROUP_ROWS, self.upload_stream)
            sp.record(side)
        else:
            side.wait_event(pre["ev"])   # the step only (it ran on the Gram stream), not the audit on main
            # the row list goes up on an otherwise idle stream (not behind the audit on main or the Gram)
            with S.use(self.upload_stream):
                sp = self.crypto.shares_async(pre["qdelta"], rows, side, group_rows=SPEC_GROUP_ROWS,
                                              no_commit=no_commit)
        return sp

    def _spec_horizon(self) -> int:
        """How far down the leader's arrival order of candidates the speculative MSM reaches, -1: every candidate
        (replicated: the leader's cap and the committed blocks' depths are the same on every rank)."""
        cap = self.fsm.leader_cap_size()
        depths = getattr(self, "_spec_depths", None) or []
        if cap <= 0 or len(depths) < SPEC_MIN_HISTORY or self.cfg.has("spec_all_candidates"):
            return -1   # every candidate until a few blocks show how deep they reach
        if self.cfg.has("spec_tight"):
            return cap
        # a short history gets more slack: 2 rows per missing block of the window
        return max(cap + SPEC_MARGIN, max(depths) + SPEC_SLACK + 2 * (SPEC_WINDOW - len(depths)))

    def _note_block_depth(self, head: dict, node_list) -> None:
        """After a block: how far down the leader's candidate arrival order its rows reached (the horizon's
        input for the next rounds)."""
        order = head.get("cand_order")
        if not order or not node_list:
            return
        nl = set(node_list)
        d = 1 + max((i for i, w in enumerate(order) if w in nl), default=len(order))
        hist = self.__dict__.setdefault("_spec_depths", [])
        hist.append(d)
        del hist[:-SPEC_WINDOW]
        log = self.__dict__.setdefault("spec_depth_log", [])   # (depth, candidates, leader cap) per block, for bench
        if len(log) < 4096:
            log.append((d, len(order), self.fsm.leader_cap_size()))

    def _early_vrf_submit(self, block_hash) -> None:
        """Start the next round's noiser VRF outputs as soon as the block that seeds them is built, before
        its audit is read and it is committed, for every peer this rank hosts (its workers are not known
        yet).  The next head adopts the job when the committed block has this hash (it does unless the
        audit fails) and the keys match (a churn restart draws new ones)."""
        cfg = self.cfg
        # (getRoles draws every peer's noisers whether or not noise is added: main.go:507)
        if not (self._pipelined() and cfg.num_noisers > 0 and self.local):
            return
        ver = getattr(self, "_seed_version", 0)
        ss = getattr(self, "_seedset", None)
        if ss is None or ss[0] != ver:
            # every local peer's noise VRF seed, held natively (rebuilt when a churn restart draws new keys)
            ss = self._seedset = (ver, self.R.VrfSeedSet([self.vrf_noise_seed[p] for p in self.local]))
        job = self.R.vrf_prove_set_async(ss[1], bytes(block_hash), max(1, cfg.host_threads - 1), None,
                                         self.vrf_dev is not None)
        self.stats["vrf_outputs"] += len(self.local)
        # covers every local peer in order: peer p's output is entry p - lo
        self._early_vrf = {"hash": bytes(block_hash), "job": job, "ver": ver}

    # ------------------------------------------------------------------ commitments
    def _local_commit_rows(self, pending_commits, local_workers: list, row_of: dict) -> torch.Tensor:
        """Device commitment rows of the local workers in local_workers order.  The commitments are
        computed per row of qdelta (row_of: one row per local worker, or one per local peer when the
        pre-step computed them for every local peer)."""
        rows = self.crypto.commit_rows_tensor(pending_commits).to(self.dev)
        idx = [row_of[w] for w in local_workers]
        if idx == list(range(rows.shape[0])):
            return rows
        return rows.index_select(0, h2d(idx, torch.long, self.dev))

    def _local_commit_buf(self, head: dict) -> torch.Tensor:
        """[maxlocal, point width] buffer whose row (w - lo) holds local worker w's commitment (the
        flat-layout part of a gather)."""
        cr, lw = self.crypto, head["local_workers"]
        part = torch.zeros((self.maxlocal, cr.point_width), dtype=cr.point_dtype, device=self.dev)
        if lw:
            part.index_copy_(0, h2d([w - self.lo for w in lw], torch.long, self.dev),
                             self._local_commit_rows(head["pending_commits"], lw, head["row_of"]))
        return part
