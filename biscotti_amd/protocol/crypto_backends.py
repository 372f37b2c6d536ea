"""Crypto backends of a round: host BN256 (CPU path) and the HBM-resident device engine (GPU path).

Both expose the same surface to the round engine -- asynchronous full-vector commitments
(createCommitment, kyber.go:533-562), shares + witnesses (createSharesAndWitnesses,
kyber.go:484-646), point-row sums (aggregateSecret, kyber.go:244-287) and the aggregate audit
(verifyCommitment on the recovered aggregate, kyber.go:564-577) -- so the engine never branches
on the device for crypto."""
from __future__ import annotations

import numpy as np
import torch

from ..native import rt
from ..ops import bn256 as B
from ..utils import d2h_into, h2d_many
from ..utils import streams as S


class _Ready:
    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


class _PendingCommitments:
    def __init__(self, host: torch.Tensor, event, jac: torch.Tensor | None = None):
        self.host, self.event, self.value = host, event, None
        self.jac = jac   # device Jacobian rows (multi-rank rounds gather these, not host marshals)
        self.ccom = self.ccom_event = self.src = None   # per-chunk commitments (chunked=True)

    def result(self) -> np.ndarray:
        if self.value is None:
            S.host_wait(self.event)
            self.value = rt().g1_marshal_jac_batch(self.host.numpy().view(np.uint32))
        return self.value


class HostCrypto:
    """CPU crypto backend (native host BN256): points travel as 64-byte marshals."""

    def __init__(self, key, poly: int, T: int, threads: int):
        self.key, self.poly, self.T = key, poly, T
        self.d = len(key)
        self.nchunks = (self.d + poly - 1) // poly
        self.threads = threads

    def commitments_async(self, qdelta: torch.Tensor, stream=None):
        return _Ready(self.commitments(qdelta))

    def commitments(self, qdelta: torch.Tensor) -> np.ndarray:
        q = qdelta.cpu().numpy()
        return np.stack([np.frombuffer(self.key.commit(q[i], 0), np.uint8) for i in range(q.shape[0])]) \
            if q.shape[0] else np.zeros((0, 64), np.uint8)

    def shares(self, qdelta: torch.Tensor):
        q = qdelta.cpu().numpy()
        n = q.shape[0]
        pts = np.zeros((n, self.nchunks, self.T + 1, 64), np.uint8)
        ys = np.zeros((n, self.nchunks, self.T), np.int64)
        for i in range(n):
            _, cc, y, wit = self.key.make_shares(q[i], self.poly, self.T)
            w = np.frombuffer(b"".join(wit), np.uint8).reshape(self.nchunks, self.T, 64)
            pts[i, :, : self.T] = w
            pts[i, :, self.T] = np.frombuffer(b"".join(cc), np.uint8).reshape(self.nchunks, 64)
            ys[i] = y
        return torch.from_numpy(pts), torch.from_numpy(ys)

    def sum_rows(self, pts: torch.Tensor) -> torch.Tensor:
        """[R, C, 64] -> [C, 64]"""
        return torch.from_numpy(rt().g1_sum_marshaled(pts.numpy()))

    # points travel as 64-byte kyber marshals on this backend
    point_width, point_dtype = 64, torch.uint8

    def commit_rows_tensor(self, pending) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(pending.result()))

    def marshal_rows(self, t: torch.Tensor) -> np.ndarray:
        return t.contiguous().numpy()

    def check_aggregate(self, coeffs: torch.Tensor, csum: torch.Tensor) -> np.ndarray:
        """ok[m, k]: commitment of recovered chunk k == miner m's summed chunk commitment (host)."""
        c, s = coeffs.numpy(), csum.numpy()
        ok = np.zeros((s.shape[0], self.nchunks), np.int32)
        for k in range(self.nchunks):
            L = min(self.poly, self.d - k * self.poly)
            ref = np.frombuffer(self.key.commit(np.ascontiguousarray(c[k, :L]), k * self.poly), np.uint8)
            ok[:, k] = [int(np.array_equal(ref, s[m, k])) for m in range(s.shape[0])]
        return ok


class _CommitTable(dict):
    """worker -> marshalled commitment (64 bytes), read from the round's uint8 [n, 64] table on first
    use: the signing reads the table rows natively, only the block's rows become bytes objects.  The
    table itself may be bound lazily (fill_lazy): its read-back is then waited for by its first reader
    (the block build or the signing), never in the middle of the verification phase."""

    def __init__(self):
        super().__init__()
        self._table, self.row, self._load = None, {}, None
        # (pinned [n, 24] device-layout Jacobian rows, their read-back event): set when the table is the
        # pre-step's commitments -- the block build then marshals only its own rows natively
        self.jac = None

    @property
    def table(self):
        if self._table is None and self._load is not None:
            self._table, self._load = self._load(), None
        return self._table

    def bound(self) -> bool:
        return self._table is not None or self._load is not None

    def fill(self, table: np.ndarray, row: dict) -> None:
        self._table, self.row = table, row

    def fill_lazy(self, load, row: dict) -> None:
        self._load, self.row = load, row

    def __missing__(self, w):
        v = self[w] = self.table[self.row[w]].tobytes()
        return v


class _SpecShares:
    """Speculative share/witness MSM of some workers' rows on a side stream.  `alive` (int32, one
    flag per row) is cleared for rows the verifiers reject; the MSM skips flagged rows, whether the
    flags were cleared before it started or while it runs.  Consumers wait on `ev`."""

    def __init__(self, eng, qdelta: torch.Tensor, rows: list, stream, deferred: bool = False, group_rows: int = 0,
                 no_commit: bool = False):
        self.eng, self.qdelta, self.rows, self.stream = eng, qdelta, rows, stream
        # no_commit: the chunk-commitment slots are not computed (the pre-step's chunk commitments feed the
        # audit); a consumer that needs them must not use these tensors
        self.no_commit = no_commit
        self.group_rows = 0 if deferred else group_rows
        # the row list and the all-ones flags in ONE upload (no fill kernel), on the caller's stream
        self.rows_t, self.alive = h2d_many([(rows, torch.int32), (np.ones(len(rows), np.int32), torch.int32)],
                                           qdelta.device)
        self.pts = self.ys = self.ev = None
        # deferred: launched once the selection has set the flags -> only the kept rows are computed,
        # packed densely over the grid
        self.deferred = deferred

    def launch(self) -> None:
        if self.ev is not None:
            return
        main = S.current()
        S.wait(self.stream, main)              # qdelta (and any flag updates) come from main
        with S.use(self.stream):
            self.pts, self.ys = self.eng.shares(self.qdelta, self.rows_t, commit_only=2 if self.no_commit else 0,
                                                check_rows=False, alive=self.alive, compact=self.deferred,
                                                group_rows=self.group_rows)
            self.ev = torch.cuda.Event()
            self.ev.record(self.stream)
        # used on the side stream / allocated there and used on main: kept for two rounds (S.hold)
        S.hold(self.qdelta, self.alive, self.rows_t, self.pts, self.ys)


class DeviceCrypto:
    """GPU crypto backend: HBM-resident tables, Jacobian points [.., 24] int32."""

    def __init__(self, key, poly: int, T: int, device):
        self.eng = B.DeviceCommitEngine(key, poly, T, device)
        self.d, self.poly, self.T, self.nchunks = self.eng.d, poly, T, self.eng.nchunks

    def commitments_async(self, qdelta: torch.Tensor, stream=None, chunked: bool = False):
        """Fixed-base MSM on device, queued download into pinned memory; result() waits for it and
        marshals on host with one batch inversion -> uint8 [n, 64].  The noise and Krum kernels
        queue behind the copy instead of waiting for the host to finish with the commitments.
        chunked: the per-chunk commitments C_k (the commitment lanes of the share MSM) are computed
        first and kept (pending.ccom [n, nch, 1, 24], ready at pending.ccom_event): the full
        commitment is their sum, and the aggregate audit sums them over the kept rows long before the
        share MSM ends (the early audit sums of NativeSecAgg.after_select)."""
        n = qdelta.shape[0]
        if n == 0:
            return _Ready(np.zeros((0, 64), np.uint8))
        main = S.current()
        stream = stream or main
        S.wait(stream, main)
        ccom = ccom_ev = None
        with S.use(stream):
            rows = self._arange(n, qdelta.device)
            if chunked:
                ccom, _ = self.eng.shares(qdelta.contiguous(), rows, commit_only=True, check_rows=False)
                ccom_ev = S.record(stream)
                jac = self.eng.commitments(ccom)
            else:
                jac = self.eng.commit_rows(qdelta.contiguous(), rows, check_rows=False)
            # pinned landing buffers are reused round to round (two in flight: the round head is
            # opened while the previous round's marshals may still be read)
            self._pin_i = (getattr(self, "_pin_i", 0) + 1) % 2
            key = (self._pin_i, tuple(jac.shape))
            host = self._pins.get(key) if hasattr(self, "_pins") else None
            if host is None:
                if not hasattr(self, "_pins"):
                    self._pins = {}
                host = self._pins[key] = torch.empty(jac.shape, dtype=jac.dtype, pin_memory=True)
            d2h_into(host, jac)
            ev = S.record(stream)
        S.hold(qdelta, jac)
        out = _PendingCommitments(host, ev, jac)
        if ccom is not None:
            S.hold(ccom)
            out.ccom, out.ccom_event, out.src = ccom, ccom_ev, qdelta
        return out

    def commitments(self, qdelta: torch.Tensor) -> np.ndarray:
        return self.commitments_async(qdelta).result()

    def _arange(self, n: int, device) -> torch.Tensor:
        if not hasattr(self, "_ar") or self._ar.numel() < n:
            self._ar = torch.arange(max(n, 256), dtype=torch.int32, device=device)
        return self._ar[:n]

    def shares(self, qdelta: torch.Tensor):
        rows = torch.arange(qdelta.shape[0], dtype=torch.int32, device=qdelta.device)
        return self.eng.shares(qdelta, rows, check_rows=False)   # arange: in range (and no stream sync)

    def shares_async(self, qdelta: torch.Tensor, rows: list, stream, launch: bool = True,
                     group_rows: int = 0, no_commit: bool = False) -> "_SpecShares":
        """Shares + witnesses of qdelta[rows] on `stream` (the caller's work keeps flowing on its own
        stream).  launch=False prepares the per-row flags only; launch() then starts the MSM after
        everything queued so far on the caller's stream (e.g. Krum's selection), so rows already
        rejected cost nothing."""
        sp = _SpecShares(self.eng, qdelta, rows, stream, deferred=not launch, group_rows=group_rows,
                         no_commit=no_commit)
        if launch:
            sp.launch()
        return sp

    def sum_rows(self, pts: torch.Tensor) -> torch.Tensor:
        """[R, C, 24] -> [C, 24]"""
        return B.sum_rows(pts.contiguous(), None, None)

    # points travel as Jacobian limbs [24] int32 on this backend
    point_width, point_dtype = 24, torch.int32

    def commit_rows_tensor(self, pending) -> torch.Tensor:
        S.current().wait_event(pending.event)   # produced on the background stream
        return pending.jac

    def marshal_rows(self, t: torch.Tensor) -> np.ndarray:
        return rt().g1_marshal_jac_batch(t.contiguous().cpu().numpy().view(np.uint32))

    def check_aggregate(self, coeffs: torch.Tensor, csum: torch.Tensor) -> torch.Tensor:
        return self.eng.check_chunks(coeffs, csum)
