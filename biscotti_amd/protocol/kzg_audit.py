"""Batched verifySecret audit of every committed aggregate (K13; kyber.go:650-673, defined but never
called on the reference's path).

verifySecret is linear in (C, W, y), so each rank checks its own partial aggregate: a random linear
combination over every (chunk, share point) of KZG_BATCH_ROUNDS rounds (device sums, kzg.hip) and
ONE host three-pairing product per batch (pairing.cpp, prepared G2 lines).  Only aggregates that end
in the chain are audited (staged when the block is adopted, not when the aggregate is queued), and a
failed batch is re-checked round by round so failures are attributed to the right iterations.
Failures are counted and logged; they never block the chain.
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils import streams as S

KZG_BATCH_ROUNDS = 16   # rounds whose audits share one pairing product (sums of independent RLCs)


class KzgAuditMixin:
    def _kzg_init(self, cfg) -> None:
        self._kzg_pending: list = []   # launched audits (device) or checked ones (CPU)
        self._kzg_stage: list = []     # rounds waiting for the next device launch
        if cfg.kzg_audit != "off":
            self.stats.update(kzg_checks=0, kzg_failures=0)
            # G2 side = (g2key[0], g2key[1]) = (G2, s G2)
            self._kzg_g2 = (self.R.g2_generator(), self._commit_key_g2_1(cfg.commit_key))
            self._kzg_rng = np.random.default_rng([cfg.seed, self.comm.rank, 0x6B7A67])

    def _commit_key_g2_1(self, path):
        """s G2 -- commitKey.json's Skey of Id 1 (publicKey.go:26-61), or 2 G2 for the generated key."""
        if path:
            import base64
            import json
            with open(path) as f:
                for ln in f:
                    if ln.strip():
                        rec = json.loads(ln)
                        if rec.get("Id") == 1:
                            return base64.b64decode(rec["Skey"])
            raise ValueError(f"{path}: no commit key record with Id 1")
        return self.R.g2_mul(self.R.g2_generator(), 2)

    # ---------------------------------------------------------------- staging (adopted aggregates only)
    def _kzg_adopt(self, agg: dict, it: int) -> None:
        """The aggregate `agg` (from _aggregate) is in the chain: stage its audit.  Device path: the
        audit stream waits for the events recorded where the sums were produced (not for work queued
        since), then the inputs join the batch."""
        kin = agg.get("kzg_in")
        if kin is None:
            return
        cs_k, ws_k, y_k, xs = kin
        if not self.gpu:
            self._kzg_host(cs_k, ws_k, y_k, agg["xs"], it)
            return
        st = self.vrf_stream
        for ev in agg["kzg_events"]:
            st.wait_event(ev)
        for t in (cs_k, ws_k, y_k, xs):
            t.record_stream(st)
        with S.use(st):
            self._kzg_queue(cs_k, ws_k, y_k, xs, it)

    def _kzg_queue(self, csum, wsum, ys, xs_t, it) -> None:
        """Stage one round's aggregate for the device RLC sums (on the audit stream, current here);
        KZG_BATCH_ROUNDS rounds with the same share-point layout go into ONE launch and one pairing
        product, read back and checked later (_kzg_poll), off the round's critical path."""
        npts = ys.shape[1]
        spm = self.pc.shares_per_miner
        if self._kzg_stage and self._kzg_stage[0]["npts"] != npts:
            self._kzg_launch()
        wperm = wsum.index_select(0, self.crypto.eng.kzg_order(npts, spm))   # (chunk, point) order
        self._kzg_stage.append({"cs": csum, "ws": wperm, "ys": ys, "xs": xs_t, "npts": npts, "it": it})
        if len(self._kzg_stage) >= KZG_BATCH_ROUNDS:
            self._kzg_launch()

    def _kzg_rlc(self, st: list):
        """Queue the RLC sums of the staged rounds `st` on the audit stream: (pinned host copy, event)."""
        with S.use(self.vrf_stream):
            cat = (lambda k: torch.cat([e[k] for e in st])) if len(st) > 1 else (lambda k: st[0][k])
            npts = st[0]["npts"]
            pts = self.crypto.eng.kzg_rlc(cat("cs"), cat("ws"), cat("ys"), torch.stack([e["xs"] for e in st]),
                                          npts, self.cfg.kzg_audit == "literal",
                                          int(self._kzg_rng.integers(0, 2**63)))
            host = torch.empty((3, 24), dtype=torch.int32, pin_memory=True)
            host.copy_(pts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.vrf_stream)
        return host, ev

    def _kzg_launch(self) -> None:
        st, self._kzg_stage = self._kzg_stage, []
        if not st:
            return
        host, ev = self._kzg_rlc(st)
        # the staged inputs stay alive until the batch is decided: a failed batch is re-checked per round
        self._kzg_pending.append({"its": [e["it"] for e in st], "ev": ev, "host": host, "job": None, "stage": st})

    def _kzg_host(self, cs, ws, ys, xs, it) -> None:
        """CPU path: the same random linear combination on the host (native threads), one round."""
        nch, npts = ys.shape
        spm = self.pc.shares_per_miner
        C = [bytes(c) for c in cs.numpy()]
        Wm = [bytes(w) for w in ws.numpy()]
        W = [Wm[(j // spm) * nch * spm + k * spm + j % spm] for k in range(nch) for j in range(npts)]
        bases = [self.R.g1_generator()] if self.cfg.kzg_audit == "literal" else \
            [self.crypto.key.point(self.cfg.poly_size * k) for k in range(nch)]
        pts = self.R.kzg_rlc_host(C, W, ys.numpy().reshape(-1), list(xs), bases,
                                  int(self._kzg_rng.integers(0, 2**63)), self.cfg.host_threads)
        self._kzg_pending.append({"its": [it], "ok": self.R.kzg_check(*pts, *self._kzg_g2)})

    def _kzg_recheck(self, e: dict) -> list:
        """A batch of several rounds failed: check each staged round on its own (device sums +
        pairing, waited for here) and return the iterations that fail individually."""
        bad = []
        for s in e["stage"]:
            host, ev = self._kzg_rlc([s])
            ev.synchronize()
            if not self.R.kzg_check_device_async(host.numpy().view(np.uint32), *self._kzg_g2).result():
                bad.append(s["it"])
        return bad

    def _kzg_poll(self, final: bool = False) -> None:
        """Start the pairing products of launches whose sums are back, and collect finished ones (all
        of them when final, the oldest when more than two are outstanding)."""
        if final and self._kzg_stage:
            self._kzg_launch()
        keep = []
        for i, e in enumerate(self._kzg_pending):
            must = final or len(self._kzg_pending) - i > 2
            if "ok" not in e and e["job"] is None and (must or e["ev"].query()):
                e["ev"].synchronize()
                e["job"] = self.R.kzg_check_device_async(e["host"].numpy().view(np.uint32), *self._kzg_g2)
            if "ok" not in e and e["job"] is not None and must:
                e["ok"] = e["job"].result()
            if "ok" in e:
                self.stats["kzg_checks"] += len(e["its"])
                if not e["ok"]:
                    bad = self._kzg_recheck(e) if len(e.get("stage") or ()) > 1 else e["its"]
                    self.stats["kzg_failures"] += len(bad)
                    if bad:
                        self.log.info("KZG audit (verifySecret, %s) failed for the aggregates of iterations %s",
                                      self.cfg.kzg_audit, bad)
            else:
                keep.append(e)
        self._kzg_pending = keep
