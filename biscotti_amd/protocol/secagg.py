"""Secure aggregation and block building: share routing, the miners' sums, exact recovery, the aggregate
audit and the leader's block.

Reference: RegisterSecret / processShare (main.go:256-367), aggregateSecret (kyber.go:244-287), the
leader's node-list intersection and share gather (main.go:2046-2189,2237-2324), recoverSecret
(kyber.go:809-857) and createBlockSecAgg (honest.go:391-440); the plain path is RegisterUpdate +
createBlock (main.go:375-390, honest.go:346-388).

Share sums are additive, so each rank sums its own workers' share columns for all miners at once and
ONE all_gather (the reduce-scatter to the miners fused with the leader's gather) hands
every rank the per-rank partials; every rank then recovers the aggregate itself (exact integer
recovery on identical inputs), so all ranks build the leader's block bit for bit.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import bn256 as B
from ..ops import ml as K
from ..utils import d2h_into, h2d
from ..utils import streams as S
from .head import SPEC_GROUP_ROWS


class _Rows:
    """Share rows the host path aggregates on the GPU, in the shape of a speculative MSM's handle (NativeSpec): the
    rows' keep flags are set (alive), the tensors are final once `ev` has passed."""

    no_commit = False
    qdelta = None   # never the pre-step's rows: the audit sums come from the rows' commitment slots

    def __init__(self, pts, ys, alive, rows_t, ev):
        self.pts, self.ys, self.alive, self.rows_t, self.ev = pts, ys, alive, rows_t, ev
        self.rows = list(range(pts.shape[0]))

    def launch(self) -> None:
        return None


class SecAggMixin:
    # ------------------------------------------------------------------ device-side aggregation
    def _predict_miners(self, plan, live):
        """(contributing miners, share part of each) exactly as leader_view / route_shares report them
        whenever at least one update is approved: parts follow the live miners in address order
        (route_shares), the leader comes first and then plan.miners order (leader_view)."""
        if not live[plan.leader]:
            return None
        addr = self.fsm.addresses
        part, k = {}, 0
        for m in sorted(plan.miners, key=lambda m_: addr[m_]):
            if live[m]:
                part[m] = k
                k += 1
        contributing = [plan.leader] + [m for m in plan.miners if m != plan.leader and live[m]]
        if self.pc.shares_per_miner * len(contributing) < self.cfg.poly_size:
            return None   # too few live miners for a quorum (leader_view): the round's block is empty
        return contributing, part

    def _agg_index(self, contributing, part):
        """Resident index tensors of one miner layout (a handful recur: the parts are a permutation of
        0..M-1): chunk-commitment columns, witness columns, the contributing miners' share columns and
        their x-points, uploaded once."""
        # the indices depend only on the sequence of parts (which miner holds which share slice), not
        # on the miners' ids: M! layouts (6 for three miners) cover every round
        key = tuple(part[m] for m in contributing)
        hit = self._agg_idx.get(key)
        if hit is None:
            spm, T, nch = self.pc.shares_per_miner, self.T, self.nchunks
            base = np.arange(nch) * (T + 1)
            ycols = np.concatenate([spm * part[m] + np.arange(spm) for m in contributing])
            wc = np.concatenate([(base[:, None] + spm * part[m] + np.arange(spm)[None, :]).reshape(-1)
                                 for m in contributing])
            assert wc.max() < nch * (T + 1) and ycols.max() < T
            wts = K.recovery_weights((ycols - 10).tolist(), self.cfg.poly_size)
            parts = [base + T, wc, ycols, ycols - 10, np.asarray(wts["basis"])]
            idx = h2d(np.concatenate(parts).astype(np.int32), torch.int32, self.dev)
            offs = np.cumsum([0] + [len(x) for x in parts])
            A_dev = h2d(wts["A"].reshape(-1), torch.int64, self.dev)
            sl = [idx[offs[i]:offs[i + 1]] for i in range(5)]
            # the native round calls know the layout by an id (its columns, weights and outputs registered once)
            lid = self._native.add_layout(sl[0], sl[1], sl[2], sl[3], wts, A_dev, sl[4]) \
                if self._native is not None else None
            hit = (sl[:4], (ycols - 10).tolist(), (wts, A_dev, sl[4]), lid)
            if len(self._agg_idx) < 256:
                self._agg_idx[key] = hit
        return hit

    def _aggregate(self, pts, ys, rowsel, contributing, part, now) -> dict:
        """CPU (host crypto) secure aggregation of this rank's kept rows, combined over ranks, then exact recovery;
        GPU rounds aggregate through the native calls (_spec_aggregate_native).

        Every miner sums the shares it received (aggregateSecret, kyber.go:244-287) and the leader recovers from
        the miners' sums (kyber.go:809-857).  Each rank sums its own workers' share columns and ONE all_gather
        hands every rank all partials (share sums, chunk-commitment sums for the audit, the clocks); the witness
        sums stay per-rank partials (the KZG audit reads them when on).

        pts [R, nch, T+1, 64] / ys [R, nch, T] (None: no local rows); rowsel: a list of row indices.  Returns the
        handles _finish_secagg consumes."""
        assert not self.gpu, "GPU rounds aggregate natively"
        cfg, comm = self.cfg, self.comm
        T, nch, pw, pdt = self.T, self.nchunks, self.crypto.point_width, self.crypto.point_dtype
        audit = cfg.audit_aggregate
        kzg = cfg.kzg_audit != "off"
        (ccols, wcols, ycols_t, xs_t), xs_list, _, _ = self._agg_index(contributing, part)
        kzg_in = None   # this rank's (commitment sums, witness sums, share sums) for the KZG audit
        ys_part = cs_part = None
        if pts is not None and rowsel:
            flat = pts.view(pts.shape[0], nch * (T + 1), pw)
            rows_l = list(rowsel)
            ys_part = ys[rows_l].sum(0)
            if audit or kzg:
                cs_part = self.crypto.sum_rows(flat[rows_l][:, ccols.long()])
            if kzg:
                kzg_in = (cs_part, self.crypto.sum_rows(flat[rows_l][:, wcols.long()]),
                          ys_part.index_select(1, ycols_t.long()))
        if ys_part is None:   # no local rows: nothing to add
            ys_part = torch.zeros((nch, T), dtype=torch.int64)
        if audit and cs_part is None:   # no local rows: the neutral element (point at infinity)
            cs_part = torch.zeros((nch, pw), dtype=pdt)
        # ---- combine over ranks: ONE all_gather (share sums, commitment sums, clock)
        clock = None
        if comm.world > 1:
            parts = [ys_part.reshape(1, -1), torch.full((1, 1), now, dtype=torch.int64)]
            if audit:
                parts.append(cs_part.reshape(1, -1))
            got = comm.all_gather_packed(parts)
            ys_src = got[0].view(comm.world, nch, T)
            clock = got[1].reshape(comm.world)
            cs_tot = self.crypto.sum_rows(got[2].view(comm.world, nch, pw)) if audit else None
        else:
            ys_src = ys_part.reshape(1, nch, T)
            cs_tot = cs_part
        agg = ys_src.sum(0).index_select(1, ycols_t.long()).contiguous()   # [nch, npts]
        W_new, coeffs, status = K.recover(agg, xs_t.cpu(), cfg.poly_size, self.d, self.W, 10.0 ** cfg.precision)
        readback = self._d2h_async(status, W_new, *((clock,) if clock is not None else ()))
        audit_ok = self._audit(coeffs, cs_tot.reshape(1, nch, pw)) if audit else None
        out = {"W_new": W_new, "status": status, "agg": agg, "xs": list(xs_list), "audit_ok": audit_ok,
               "clock": clock, "now": now, "readback": readback}
        if kzg_in is not None:
            # each rank audits its own partial aggregate (verifySecret is linear in (C, W, y))
            cs_k, ws_k, y_k = kzg_in
            out["kzg_in"] = (cs_k, ws_k, agg if comm.world == 1 else y_k, xs_t)
        return out

    def _spec_aggregate_native(self, sp, pred, node, amap, flags_set: bool = False, it: int | None = None,
                               W=None) -> dict:
        """The GPU secure aggregation through the fused native calls (kernels/round.hip) -- behind the committee's
        selection (sp: the speculative MSM) or on the host-decided path (sp: _Rows) alike.  One rank: ONE call
        queues the rows' flags, the early audit sums, the miners' sums + exact recovery + read-back, the next
        round's pre-step and the audit; several ranks: one call up to this rank's partial sums in the packed
        send row, the all_gather (main stream), one call for the totals, recovery, read-back, pre-step and
        audit.  With the KZG audit on, this rank's partial aggregate (commitment, witness and share sums) is
        copied out of the resident buffers for it (_kzg_capture)."""
        cfg, comm, na = self.cfg, self.comm, self._native
        contributing, part = pred
        (_, _, ycols_t, xs_t), xs_list, _, lid = self._agg_index(contributing, part)
        kzg = cfg.kzg_audit != "off"
        run_audit = cfg.audit_aggregate
        audit = 1 if (run_audit or kzg) else 0   # the KZG audit reads the commitment sums too
        early = -1
        if sp is not None:
            sp.launch()
            pc = getattr(self, "_cur_commits", None)
            if audit and pc is not None and getattr(pc, "slot", None) is not None and pc.src is sp.qdelta:
                early, audit = pc.slot, 2   # the audit's sums from the pre-step's chunk commitments, early
            elif sp.no_commit and audit:
                raise RuntimeError("speculative MSM without commitment slots but no chunk commitments to audit with")
        if kzg and getattr(self, "_kzg_copied", None) is not None:
            S.current().wait_event(self._kzg_copied)   # the last aggregate's copies before its buffers are rewritten
        # it: the round being aggregated (default: the FSM's, begun); W: the model it starts from (default: the engine's)
        # -- a speculative front passes both, ahead of the previous block's commit (engine._spec_front_launch)
        it = self.fsm.iteration if it is None else it
        W = self.W if W is None else W
        nxt = it + 1
        # the next round's pre-step behind the recovery (softmax tasks: binds the task at the first use)
        pre_it = nxt if (self._pipelined() and getattr(self.task, "stateless_step", False)
                         and self._native_prestep_ok()) else -1
        now = self._now(it)
        sel = None if flags_set else node   # None: the vote kernel (or the host path) has set the rows' flags
        if comm.world == 1:
            W_new, pre = na.after_select(sel, amap, sp, early, self.upload_stream, lid, W, audit, pre_it,
                                         audit_now=run_audit)
            readback, clock = na.readback(), None
            if pre is not None:
                pre = self._finish_pre(pre, nxt)
        elif na.native_comm:
            # one call: partials, the all_gather, recovery, the next pre-step and its Gram's gather + tile pairs
            gram = self._multi_gram and pre_it >= 0
            W_new, k = na.agg_multi(sel, amap, sp, early, self.upload_stream, lid, now, W, audit, pre_it,
                                    run_audit, gram)
            pre = None
            if k >= 0:
                pre = na.multi_gram_pre(k, W_new, nxt, self.flat) if gram else \
                    self._finish_pre(na._pre_out(k, W_new, nxt), nxt)
            readback, clock = na.readback(clocks=True), True
        else:   # gloo ranks on GPUs (tests): the collective is torch's, between the two native calls
            na.select_partials(sel, amap, sp, early, self.upload_stream, lid, now, audit)
            comm.all_gather_into(na.recv, na.send)
            W_new, k = na.after_gather(lid, W, audit, pre_it, audit_now=run_audit)
            pre = self._finish_pre(na._pre_out(k, W_new, nxt), nxt) if k >= 0 else None
            readback, clock = na.readback(clocks=True), True
        if pre is not None:
            self._pre = pre
        out = {"W_new": W_new, "status": na.status, "agg": na.layout_agg(lid), "xs": list(xs_list),
               "audit_ok": na.audit(queue=False) if run_audit else None, "clock": clock, "now": now,
               "readback": readback, "contributing": list(contributing), "part": dict(part), "accepted": None,
               "node": node}
        if kzg:
            out["kzg_in"] = self._kzg_capture(lid, ycols_t, xs_t)
            out["kzg_events"] = [self._kzg_copied]   # the audit stream reads the copies (_kzg_adopt)
        return out

    def _kzg_capture(self, lid: int, ycols_t, xs_t):
        """This rank's partial aggregate for the KZG audit, copied (audit stream) out of the native round's resident
        buffers once the streams that wrote them are done: chunk-commitment sums, witness sums and share sums at
        the contributing points ([nch, npts]: the recovered aggregate on one rank, this rank's send-row partials
        on several).  The next aggregation waits for the copies (_kzg_copied) before rewriting the buffers."""
        na, nch = self._native, self.nchunks
        # a stream of its own: on the VRF prover's stream the copies (which the next aggregation waits for) queued
        # behind a whole ~2.2 ms prover launch
        st = self.__dict__.get("kzg_stream")
        if st is None:
            st = self.kzg_stream = torch.cuda.Stream(device=self.dev, priority=torch.cuda.Stream.priority_range()[0])
        for src in (S.current(), self.side_stream, self.upload_stream, self.witness_stream):
            S.wait(st, src)
        with S.use(st):
            if self.comm.world == 1:
                cs, ys = na.cs.clone(), na.layout_agg(lid).clone()
            else:
                row = na.send
                cs = row[: 96 * nch].view(torch.int32).view(nch, 24).clone()
                ys = row[96 * nch: 96 * nch + 8 * nch * self.T].view(torch.int64).view(nch, self.T) \
                    .index_select(1, ycols_t.long())
            ws = na.layout_ws(lid).clone()
            self._kzg_copied = S.record(st)
        return cs, ws, ys, xs_t

    def _native_rows_aggregate(self, pts, ys, rowsel: list, pred, ev) -> dict:
        """The host-decided path's GPU aggregation (no device selection, a speculative miss, a prediction mismatch):
        rows `rowsel` of the share tensors pts / ys (None: no local rows) through the same native calls, with the
        rows' flags set here instead of by the selection kernel."""
        rows = None
        if pts is not None and rowsel:
            keep = np.zeros(pts.shape[0], np.int32)
            keep[np.asarray(rowsel, np.int64)] = 1
            rows = _Rows(pts, ys, h2d(keep, torch.int32, self.dev),
                         h2d(np.arange(pts.shape[0], dtype=np.int32), torch.int32, self.dev), ev)
        return self._spec_aggregate_native(rows, pred, None, None, flags_set=True)

    # ------------------------------------------------------------------ read-backs and the audit
    def _d2h_async(self, *ts: torch.Tensor):
        """CPU: the tensors as numpy arrays behind a callable (the GPU path reads back natively)."""
        out = [t.numpy() for t in ts]
        return lambda: out

    def _audit(self, coeffs: torch.Tensor, csum: torch.Tensor):
        """CPU: the aggregate audit (recovered chunks vs the miners' summed chunk commitments) behind a callable
        giving ok int32 [n_miners, nchunks] (the GPU path runs it natively: bsc_round_audit)."""
        ok = self.crypto.check_aggregate(coeffs.cpu(), csum.cpu())
        return lambda: ok

    # ------------------------------------------------------------------ secure aggregation path
    def _secure_aggregation(self, plan, live, approved, qdelta, local_workers, row_of, commit_of,
                            signatures, spec=None, sa=None):
        cfg, R, fsm, tm = self.cfg, self.R, self.fsm, self.timer
        self._last_nodes = []
        if cfg.verify_signatures and cfg.verification:
            # miners reject shares without >= nv/2 valid verifier signatures (main.go:269-277, Q5)
            need = len(plan.verifiers) // 2
            approved = [w for w in approved
                        if sum(any(R.schnorr_verify(commit_of[w], self.pk[v], sg) for v in plan.verifiers)
                               for sg in signatures.get(w, [])) >= need]
        with tm.phase("shares"):
            # share routing + the leader's view natively (the routes never cross into Python)
            online, quorum, node_list, contributing, part_of = fsm.route_view(approved)
        if not (online and quorum):
            return None
        if sa is not None and sa.get("accepted") is not None and contributing == sa["contributing"] \
                and part_of == sa["part"] and set(node_list) == sa["accepted"]:
            # the device already aggregated exactly these workers' shares (queued behind the committee's
            # selection, before the host knew the approvals): recovery and audit are in flight
            self.stats["device_aggregations"] = self.stats.get("device_aggregations", 0) + 1
            with tm.phase("recover"):
                return self._finish_secagg(plan, node_list, commit_of, sa)
        # host-decided path (no device selection, RONI, or a prediction mismatch): the leader's block
        # carries lv.node_list only (its first NUM_SAMPLES/2 arrivals), so only those workers' shares are
        # computed; every rank takes this branch together (replicated decisions)
        with tm.phase("shares"):
            local_used = [w for w in node_list if w in self.local]
            sp2 = self._spec_topup(spec, local_used, row_of, qdelta)
        if sp2 is not None:
            # a speculative miss: the block's rows the MSM did not cover go into its ring slot behind its rows, the
            # slot's flags become the block's, and the aggregation reads them all (~2 ms recomputing every block row
            # with its commitment lanes before; docs/PERF.md, round 6)
            with tm.phase("recover"):
                agg = self._spec_aggregate_native(sp2, (contributing, part_of), None, None, flags_set=True)
                return self._finish_secagg(plan, node_list, commit_of, agg)
        with tm.phase("shares"):
            pts = ys = ev = None
            rowsel: list = []
            if local_used:
                spec_row = {w: i for i, w in enumerate(spec[0])} if spec is not None else {}
                # (an MSM run without its commitment slots cannot feed this path's audit sums: recompute)
                if spec is not None and all(w in spec_row for w in local_used) and not spec[1].no_commit:
                    sp = spec[1]
                    sp.launch()
                    pts, ys, ev = sp.pts, sp.ys, sp.ev
                    rowsel = [spec_row[w] for w in local_used]   # rows of the speculative tensors
                else:
                    sel = h2d([row_of[w] for w in local_used], torch.long, self.dev)
                    pts, ys = self.crypto.shares(qdelta.index_select(0, sel).contiguous())
                    rowsel = list(range(len(local_used)))
                    ev = S.record() if self.gpu else None
        with tm.phase("recover"):
            if self.gpu:
                agg = self._native_rows_aggregate(pts, ys, rowsel, (contributing, part_of), ev)
            else:
                agg = self._aggregate(pts, ys, rowsel, contributing, part_of, self._now(plan.iteration))
            return self._finish_secagg(plan, node_list, commit_of, agg)

    def _spec_topup(self, spec, local_used: list, row_of: dict, qdelta):
        """The host-decided aggregation's rows from the speculative MSM's ring slot, topped up with the block rows it did
        not cover (NativeSecAgg.spec_topup) -- GPU, native round, an MSM without commitment lanes over this very
        qdelta (the audit's sums then come from the pre-step's chunk commitments); None otherwise."""
        na = self._native
        if not (self.gpu and na is not None and spec is not None and local_used):
            return None
        sp = spec[1]
        if not (sp.no_commit and getattr(sp, "qdelta", None) is qdelta and hasattr(sp, "ev_flags")):
            return None
        used = set(local_used)
        keep = np.fromiter((w in used for w in spec[0]), np.int32, len(spec[0]))
        have = set(spec[0])
        extra = [row_of[w] for w in local_used if w not in have]
        sp2 = na.spec_topup(sp, keep, extra, SPEC_GROUP_ROWS, self.upload_stream, self.side_stream)
        if sp2 is None:
            return None
        S.current().wait_event(sp2.ev)   # the slot's flags and the new rows before the aggregation reads them
        self.stats["spec_topups"] = self.stats.get("spec_topups", 0) + 1
        return sp2

    def _finish_secagg(self, plan, node_list, commit_of, h):
        """Read back the recovered model (and the ranks' clocks), fall back to least squares for
        inconsistent chunks, build the block, then check the aggregate audit (running on the device
        meanwhile)."""
        cfg, R, fsm, tm = self.cfg, self.R, self.fsm, self.timer
        W_new, status, agg, xs, audit_ok = h["W_new"], h["status"], h["agg"], h["xs"], h["audit_ok"]
        with tm.phase("recover.readback"):
            got = h["readback"]()
            st, W_np = got[0], got[1]
            if h["clock"] is not None:
                now = int(got[2][self.comm.owner(plan.leader, self.N)])   # the leader's clock stamps the block
            else:
                now = h["now"]
        if not st.all():  # inconsistent shares: the reference's float64 least squares
            aggn, Wn = agg.cpu().numpy(), self.W.cpu().numpy()
            for k in np.nonzero(st == 0)[0]:
                c = R.recover_lstsq(xs, [int(v) for v in aggn[k]], cfg.poly_size - 1)
                for j, v in enumerate(c):
                    i = k * cfg.poly_size + j
                    if i < self.d:
                        W_np[i] = Wn[i] + v / 10.0 ** cfg.precision
            self.log.info("recovery fell back to least squares for %d chunks", int((st == 0).sum()))
        with tm.phase("recover.block"):
            jac = getattr(commit_of, "jac", None)
            if jac is not None and commit_of._table is None:
                # the commitments are still the pre-step's Jacobian rows: only the block's are marshalled (one
                # inversion, natively) -- the signing marshals the whole table later, off this path
                S.host_wait(jac[1])
                block = fsm.make_secagg_block_jac(W_np, node_list, jac[0].numpy().view(np.uint32),
                                                  [commit_of.row[w] for w in node_list], now)
            else:
                block = fsm.make_secagg_block(W_np, node_list, [commit_of[w] for w in node_list], now)
        self._W_next = W_new if st.all() and self.gpu else None
        # the next round's VRF outputs first (a native seed set: ~12 us to submit; started after the speculative
        # launch they were not ready at the next round's noiser lottery: vrf_join 0.04 -> 0.1 ms), then its
        # share MSM
        self._early_vrf_submit(block.hash)
        if self._W_next is not None:
            self._spec_head_launch(block)
            # and its front (noiser lottery, Krum launch, the aggregation behind the selection) before the audit wait
            self._spec_front_launch(block)
        if audit_ok is not None:
            if self._idle_work is not None:   # host-only work (no collective): overlap it with the audit
                self._idle_work()
                self._idle_work = None
            if self.gpu:
                # the next round's VRF batch has just started (_early_vrf_submit): this round's deferred
                # signature prep (its batch starts behind those outputs -- started in the read-back wait instead,
                # it slowed the outputs: vrf_join 0.03 -> 0.09 ms), the earlier rounds' evaluation read-backs and
                # the next round's host preparation fill the audit wait
                with tm.phase("recover.idle"):
                    sf = self._spec_front
                    # else (a front planned at the commit) run after the next round's front (run_round)
                    if not self._front_planned or sf is not None:
                        ej = sf["front"]["head"]["fut_noise"] if sf is not None else \
                            self._early_vrf["job"] if self._early_vrf is not None else None
                        work, self._pre_vrf_work = self._pre_vrf_work, []
                        for f in work:
                            f(ej)
                        # (after a speculative front the previous round's evaluation was queued just before: only
                        # the landed read-backs are taken)
                        self._resolve_evals(wait=sf is None)
                    self._prepare_next_in_wait()
            with tm.phase("recover.audit"):
                ok = audit_ok()
            if not ok.all():
                # a miner's sums do not commit to the recovered update: refuse it (the round ends like the
                # reference's missing-quorum path, with an empty block)
                self.stats["audit_failures"] += 1
                self.log.info("aggregate audit failed for %d (miner, chunk) pairs in iteration %d: empty block",
                              int((ok == 0).sum()), plan.iteration)
                return None
        self._last_nodes = node_list
        if cfg.kzg_audit != "off":
            self._kzg_adopt(h, plan.iteration)   # only aggregates that end in the chain are audited
            if self._kzg_pending:
                self._kzg_poll()
        return block

    def _prepare_next_in_wait(self) -> None:
        """Host work of the NEXT round that is ready before this round's audit is read: the host marshal of
        its commitments (the pre-step's commitment MSM has usually landed by now; never waited for here)
        and Krum's static tables for the successor plan the speculative MSM was launched from.  Both are
        used only if the next head adopts the pre-step / the speculative plan (the committed block matches)."""
        pre, sn = self._pre, self._spec_next
        pc = pre.get("commits") if pre is not None else None
        if pc is not None and getattr(pc, "value", 1) is None and pc.event.query():
            pc.result()
        if sn is None or sn.get("kst") is not None or pre is None or sn.get("pre") is not pre:
            return
        g = pre.get("gram")
        cfg = self.cfg
        if g is None or not (cfg.verification and cfg.defense == "KRUM" and sn["inboxes"]):
            return
        sn["kst"] = self._krum_static(g["xrow"], g["U1"], sn["plan"], [1] * self.N, sn["inboxes"], sn["spec"],
                                      sn["arrivals"])

    # ------------------------------------------------------------------ plain aggregation path
    def _plain_aggregation(self, plan, live, approved, delta_w, noised, local_workers, commit_of, signatures,
                           gathered=(None, None, None)):
        """RegisterUpdate path (-sa=false): the leader miner's block carries every routed update in full.
        delta_w / noised: the local workers' rows in local_workers order.  With several ranks the deltas,
        noised deltas and clocks already travelled in the verification all_gather, so every rank builds
        the leader's block itself (no broadcast)."""
        fsm, comm, tm = self.fsm, self.comm, self.timer
        self._last_nodes = []
        with tm.phase("aggregate"):
            routes = fsm.route_updates(approved)
            leader = plan.leader
            if not live[leader] or not routes.get(leader):
                return None
            ups = list(routes[leader])
            now = self._now(plan.iteration)
            if comm.world == 1:
                idx = {w: i for i, w in enumerate(local_workers)}
                sel = h2d([idx[w] for w in ups], torch.long, self.dev)
                dsrc, nsrc = delta_w, noised
            else:
                dsrc, nsrc, ts = gathered
                sel = h2d([self.flat[w] for w in ups], torch.long, self.dev)
                now = int(ts[comm.owner(leader, self.N)])
            dv = dsrc.index_select(0, sel).double().cpu().numpy()
            nv = nsrc.index_select(0, sel).double().cpu().numpy()
            blk = fsm.make_plain_block_arrays(self.W.cpu().numpy(), ups, dv, nv, [commit_of[w] for w in ups],
                                              [signatures.get(w, []) for w in ups], now)
            self._last_nodes = ups
            return blk
