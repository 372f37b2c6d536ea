"""Device-side BN256 G1 engine: fixed-base tables + batched share/commitment MSM on gfx950.

Replaces the reference's per-peer Go big.Int loops (DistSys/kyber.go:533-646) with HBM-resident
signed-window tables and one fused kernel per round phase (see csrc/kernels/msm.hip).

Tensor conventions (all on the GPU):
  * field elements: 8 x 32-bit Montgomery limbs stored in ``torch.int32`` (bit patterns)
  * affine points   [..., 16]  (x, y);  infinity = zeros
  * Jacobian points [..., 24]  (x, y, z); infinity <=> z == 0
"""
from __future__ import annotations

import numpy as np
import torch

from ..native import hip, rt
from ..utils import streams as S

TBL_ENTRIES = 128    # entries of an 8-bit signed window
B0_CHOICES = (14, 13, 12, 11, 10, 9, 8)   # first-window widths, widest that fits in HBM wins
_SCRATCH_BYTES = 1 << 31


def windows_for(b0: int) -> tuple[int, int]:
    """(NW, entries per base) for a B0-bit first window followed by 8-bit windows covering int64."""
    nw = 1 + -(-(65 - b0) // 8)
    return nw, (1 << (b0 - 1)) + (nw - 1) * TBL_ENTRIES


def table_bytes_for(d: int, poly: int, total_shares: int, b0: int) -> int:
    nchunks = (d + poly - 1) // poly
    return (d + nchunks * (poly - 1) * total_shares) * windows_for(b0)[1] * 64


def choose_b0(d: int, poly: int, total_shares: int, device, fraction: float = 0.6) -> int:
    """Widest first window whose tables fit in `fraction` of the free device memory.

    BSC_TABLE_B0 overrides.  On a 288 GB MI355X the MNIST key (d = 7850) gets B0 = 14: ~91 GB of
    tables and one mixed addition for every |coefficient| <= 8192."""
    import os
    env = os.environ.get("BSC_TABLE_B0")
    if env:
        return int(env)
    free, total = torch.cuda.mem_get_info(device)
    # processes sharing one GPU (several ranks / per-peer processes per device) split the budget evenly
    # up front, so they all pick the same B0 instead of each taking 60 % of what is left.  The count
    # comes from Comm.init (ranks with the same host and device UUID); one rank per GPU -> no split
    from ..parallel.comm import ranks_per_device

    per_gpu = max(1, ranks_per_device())
    budget = min(fraction * free, (fraction if per_gpu == 1 else 0.66) * total / per_gpu) - _SCRATCH_BYTES
    for b0 in B0_CHOICES:
        if table_bytes_for(d, poly, total_shares, b0) <= budget:
            return b0
    return 8


def _stream() -> int:
    return S.raw()


def _ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "device kernels need contiguous GPU tensors"
    return t.data_ptr()


def _check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"HIP launch of {what} failed with hipError {err}")


def u32_tensor(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(device)


class DeviceCommitEngine:
    """Commitment key + witness-base tables resident on one GPU.

    poly: POLY_SIZE (10); total_shares: TOTAL_SHARES (21) -- x = i - 10 (kyber.go:588).
    """

    def __init__(self, commit_key, poly: int, total_shares: int, device="cuda", b0: int | None = None):
        self.device = torch.device(device)
        self.d = len(commit_key)
        self.poly = int(poly)
        self.T = int(total_shares)
        self.J = self.poly - 1
        self.b0 = int(b0) if b0 is not None else choose_b0(self.d, self.poly, self.T, self.device)
        self.nw, self.pb = windows_for(self.b0)
        self.nchunks = (self.d + self.poly - 1) // self.poly
        lib = hip()
        self.pk_aff = u32_tensor(commit_key.affine_mont_u32(), self.device)  # [d, 16]
        # witness bases B_{j,x}: [nchunks][J][T][24]
        self.wbases = torch.empty((self.nchunks, self.J, self.T, 24), dtype=torch.int32, device=self.device)
        _check(lib.bsc_witness_bases(_ptr(self.pk_aff), self.d, self.poly, self.T, _ptr(self.wbases), _stream()),
               "witness_bases")
        PB, T = self.pb, self.T
        self.tbl_pk = torch.empty((self.d, PB, 16), dtype=torch.int32, device=self.device)
        self.tbl_wb = torch.empty((self.nchunks, self.J, PB, T, 16), dtype=torch.int32, device=self.device)
        self._build_table(self.pk_aff, False, self.d, 1, (PB, 1, 0), self.tbl_pk)
        self._build_table(self.wbases, True, self.nchunks * self.J * T, T, (PB * T, T, 1), self.tbl_wb)
        del self.wbases
        torch.cuda.synchronize(self.device)

    def table_bytes(self) -> int:
        return (self.tbl_pk.numel() + self.tbl_wb.numel()) * 4

    def release(self) -> None:
        """Drop the device tables (engine shutdown); the engine is unusable afterwards."""
        self.tbl_pk = self.tbl_wb = self.wbases = None

    def _build_table(self, bases, jac: bool, nbases: int, inner: int, strides, table) -> None:
        lib = hip()
        runs = (1 << (self.b0 - 1)) // TBL_ENTRIES + self.nw - 1   # 128-entry runs per base
        per_base = TBL_ENTRIES * 32 * 4 * runs
        batch = max(inner, (_SCRATCH_BYTES // per_base) // inner * inner)
        scratch = torch.empty((min(batch, nbases) * runs * TBL_ENTRIES * 32,), dtype=torch.int32, device=self.device)
        for s0 in range(0, nbases, batch):
            nb = min(batch, nbases - s0)
            _check(lib.bsc_fb_table(_ptr(bases), int(jac), s0, nb, inner, self.b0, self.nw, *strides, _ptr(table),
                                    _ptr(scratch), _stream()), "fb_table")
        del scratch

    # ---------------------------------------------------------------- per-round kernels
    def shares(self, coeffs: torch.Tensor, rows: torch.Tensor, commit_only: bool = False, check_rows: bool = True,
               alive: torch.Tensor | None = None, compact: bool = False, group_rows: int = 0):
        """Fused chunk commitments (+ witnesses and share values unless commit_only).

        coeffs: int64 [P, d] quantized deltas; rows: int32 [n] rows of `coeffs` to process.
        alive: optional int32 [n] flags (1 = compute); a row whose flag is cleared while the kernel
        runs (set_alive) is skipped from then on and its outputs are left undefined.
        compact: the flags are final when the kernel starts -- the flagged rows are packed densely
        over the grid (a skipped row then costs no SIMD lanes, unlike the per-thread skip).
        group_rows: process the rows G at a time in list order (late cancellation then saves the
        rows not reached yet); 0 = all rows chunk-major at once.
        Returns (pts [n, nchunks, S, 24] Jacobian with S = 1 or T+1, ys [n, nchunks, T] or None).
        """
        assert coeffs.dtype == torch.int64 and coeffs.dim() == 2 and coeffs.shape[1] == self.d
        assert rows.dtype == torch.int32 and rows.dim() == 1
        n = rows.numel()
        if n and check_rows:  # .item() synchronises the stream: callers passing arange skip it
            assert int(rows.min()) >= 0 and int(rows.max()) < coeffs.shape[0], "row index out of range"
        commit_only = int(commit_only)   # 2: witnesses + share values only (slot T left unwritten)
        S = 1 if commit_only == 1 else self.T + 1
        pts = torch.empty((n, self.nchunks, S, 24), dtype=torch.int32, device=self.device)
        ys = None if commit_only == 1 else torch.empty((n, self.nchunks, self.T), dtype=torch.int64,
                                                       device=self.device)
        cidx = None
        if alive is not None:
            assert alive.dtype == torch.int32 and alive.numel() == n
            if compact and n:
                cidx = torch.empty((n + 1,), dtype=torch.int32, device=self.device)
                _check(hip().bsc_alive_compact(_ptr(alive), n, _ptr(cidx), _stream()), "alive_compact")
        _check(hip().bsc_shares_msm(_ptr(coeffs), self.d, _ptr(rows), n, _ptr(self.tbl_pk), _ptr(self.tbl_wb),
                                    self.poly, self.T, self.b0, self.nw, commit_only, _ptr(alive), _ptr(cidx),
                                    int(group_rows), _ptr(pts), _ptr(ys), _stream()),
               "shares_msm")
        return pts, ys

    def commit_rows(self, coeffs: torch.Tensor, rows: torch.Tensor, check_rows: bool = True) -> torch.Tensor:
        """Full-vector commitments sum_i c_i PK[i] of the given rows, Jacobian [n, 24] (commit phase)."""
        assert coeffs.dtype == torch.int64 and coeffs.dim() == 2 and coeffs.shape[1] == self.d
        assert rows.dtype == torch.int32 and rows.dim() == 1
        n = rows.numel()
        out = torch.empty((n, 24), dtype=torch.int32, device=self.device)
        if n == 0:
            return out
        if check_rows:
            assert int(rows.min()) >= 0 and int(rows.max()) < coeffs.shape[0], "row index out of range"
        nslab = (self.d + 1023) // 1024
        partial = torch.empty((n * nslab, 24), dtype=torch.int32, device=self.device)
        _check(hip().bsc_commit_rows(_ptr(coeffs), self.d, _ptr(rows), n, _ptr(self.tbl_pk), self.b0, self.nw,
                                     _ptr(partial), _ptr(out), _stream()), "commit_rows")
        return out

    def check_chunks(self, coeffs: torch.Tensor, csum: torch.Tensor) -> torch.Tensor:
        """Aggregate audit: ok[m, k] = 1 iff the chunk commitment of the recovered coefficients
        coeffs[k] (int64 [nchunks, poly]) equals miner m's summed chunk commitment csum[m, k]
        (Jacobian int32 [nm, nchunks, 24]) -- verifyCommitment (kyber.go:564-577) on the aggregate."""
        assert coeffs.dtype == torch.int64 and tuple(coeffs.shape) == (self.nchunks, self.poly)
        assert csum.dtype == torch.int32 and csum.dim() == 3 and tuple(csum.shape[1:]) == (self.nchunks, 24)
        coeffs, csum = coeffs.contiguous(), csum.contiguous()
        nm = csum.shape[0]
        ok = torch.empty((nm, self.nchunks), dtype=torch.int32, device=self.device)
        _check(hip().bsc_chunk_check(_ptr(coeffs), self.d, self.poly, _ptr(self.tbl_pk), self.b0, self.nw, _ptr(csum),
                                     nm, self.nchunks, _ptr(ok), _stream()), "chunk_check")
        return ok

    def kzg_rlc(self, csum: torch.Tensor, wsum: torch.Tensor, ys: torch.Tensor, xs: torch.Tensor, spm: int,
                literal: bool, seed: int) -> torch.Tensor:
        """G1 side of the batched verifySecret audit (kzg.hip): (L1, A, L2) Jacobian int32 [3, 24] with
        e(L1, g2_0) e(-A, g2_1) e(L2, G2) == 1 iff (whp) every (chunk, share point) check holds.

        csum [nch, 24] chunk commitments; wsum [(npts/spm) * nch * spm, 24] witnesses (miner-major,
        chunk, share slot); ys int64 [nch, npts] share values at xs int32 [npts]; literal: pair y
        against G1 for every chunk (the reference's verifySecret, quirk Q9) instead of PK[poly*k].
        Several rounds: nch = rounds * nchunks stacked chunks, xs [rounds, npts], wsum in (chunk,
        point) order with spm = npts (kzg_order() gives that permutation of one round's sums)."""
        nch, npts = ys.shape
        assert csum.dtype == torch.int32 and tuple(csum.shape) == (nch, 24) and nch % self.nchunks == 0
        assert wsum.dtype == torch.int32 and tuple(wsum.shape) == (nch * npts, 24)
        assert ys.dtype == torch.int64 and xs.dtype == torch.int32 and xs.numel() == npts * (nch // self.nchunks)
        assert spm > 0 and npts % spm == 0 and (nch == self.nchunks or spm == npts)
        if literal:
            if getattr(self, "_g1_aff", None) is None:
                self._g1_aff = u32_tensor(rt().g1_affine_mont_u32(rt().g1_generator()), self.device)
            bases, stride = self._g1_aff, 0
        else:
            bases, stride = self.pk_aff, self.poly
        lib = hip()
        partial = torch.empty((lib.bsc_kzg_blocks(nch, npts), 72), dtype=torch.int32, device=self.device)
        out = torch.empty((3, 24), dtype=torch.int32, device=self.device)
        _check(lib.bsc_kzg_rlc(_ptr(csum.contiguous()), _ptr(wsum.contiguous()), _ptr(ys.contiguous()),
                               _ptr(xs.contiguous()), nch, npts, int(spm), _ptr(bases), stride, self.nchunks,
                               int(seed) & ((1 << 64) - 1), _ptr(partial), _ptr(out), _stream()), "kzg_rlc")
        return out

    def kzg_order(self, npts: int, spm: int) -> torch.Tensor:
        """Row permutation taking one round's witness sums from (miner, chunk, slot) to (chunk, point)
        order (int64 [nchunks * npts], cached): the layout several stacked rounds share."""
        key = (npts, spm)
        cache = self.__dict__.setdefault("_kzg_perm", {})
        if key not in cache:
            k = np.arange(self.nchunks)[:, None]
            j = np.arange(npts)[None, :]
            rows = (j // spm) * self.nchunks * spm + k * spm + j % spm
            cache[key] = torch.from_numpy(rows.reshape(-1).astype(np.int64)).to(self.device)
        return cache[key]

    def commitments(self, pts: torch.Tensor) -> torch.Tensor:
        """Full-vector commitment per row = sum of its chunk commitments. Returns Jacobian [n, 24]."""
        n, nch, S, _ = pts.shape
        out = torch.empty((n, 24), dtype=torch.int32, device=self.device)
        _check(hip().bsc_segment_sum(_ptr(pts), n, nch, S, S - 1, _ptr(out), _stream()), "segment_sum")
        return out


def sum_rows(pts: torch.Tensor, rows: torch.Tensor | None, cols: torch.Tensor | None,
             check: bool = True, row_mask: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = sum_r pts[rows[r], cols[i]] for a [R, C, 24] Jacobian tensor.

    check=False: the caller validated the index lists on the host before uploading them (the
    device-side max() would stall the host behind everything queued on the stream).
    row_mask: optional int32 [R] -- rows flagged 0 are left out (device-side selection)."""
    assert pts.dim() == 3 and pts.shape[2] == 24
    R, Cn, _ = pts.shape
    nrows = R if rows is None else rows.numel()
    ncols = Cn if cols is None else cols.numel()
    if rows is not None:
        assert rows.dtype == torch.int32 and (not check or nrows == 0 or int(rows.max()) < R)
    if cols is not None:
        assert cols.dtype == torch.int32 and (not check or ncols == 0 or int(cols.max()) < Cn)
    if row_mask is not None:
        assert row_mask.dtype == torch.int32 and row_mask.numel() == R
    out = torch.empty((ncols, 24), dtype=torch.int32, device=pts.device)
    _check(hip().bsc_sum_rows2(_ptr(pts), Cn, _ptr(rows), nrows, _ptr(cols), ncols, _ptr(row_mask), _ptr(out),
                               _stream()), "sum_rows2")
    return out


def set_alive(accept: torch.Tensor, src: torch.Tensor, alive: torch.Tensor) -> None:
    """alive[i] = accept[src[i]] for every speculative row i, 0 where src[i] < 0 (device-scope stores: a
    share MSM running on another stream sees them and skips the dropped rows).  accept: int32 over the
    selection's rows; src, alive: int32 [n speculative rows]."""
    n = alive.numel()
    assert accept.dtype == torch.int32 and src.dtype == torch.int32 and src.numel() == n
    assert alive.dtype == torch.int32
    _check(hip().bsc_set_alive(_ptr(accept), _ptr(src), n, _ptr(alive), _stream()), "set_alive")


def marshal_host(pts: torch.Tensor) -> "np.ndarray":
    """Jacobian [..., 24] on device -> kyber marshals uint8 [N, 64] on host, normalised with a single
    field inversion (Montgomery's batch trick) instead of one latency-bound inversion per point."""
    flat = pts.reshape(-1, 24).contiguous().cpu().numpy().view(np.uint32)
    return rt().g1_marshal_jac_batch(flat)


def marshal(pts: torch.Tensor) -> torch.Tensor:
    """Jacobian [..., 24] -> kyber marshal bytes uint8 [N, 64] (on device)."""
    flat = pts.reshape(-1, 24).contiguous()
    out = torch.empty((flat.shape[0], 64), dtype=torch.uint8, device=pts.device)
    _check(hip().bsc_marshal(_ptr(flat), flat.shape[0], _ptr(out), _stream()), "marshal")
    return out


def to_affine(pts: torch.Tensor) -> torch.Tensor:
    flat = pts.reshape(-1, 24).contiguous()
    out = torch.empty((flat.shape[0], 16), dtype=torch.int32, device=pts.device)
    _check(hip().bsc_to_affine(_ptr(flat), flat.shape[0], _ptr(out), _stream()), "to_affine")
    return out


def fp_op(a: torch.Tensor, b: torch.Tensor, op: int) -> torch.Tensor:
    """Element-wise field op on [n, 8] limb tensors (0 mul, 1 add, 2 sub, 3 inv, 4 from_mont)."""
    assert a.shape == b.shape and a.shape[-1] == 8
    out = torch.empty_like(a)
    _check(hip().bsc_fp_op(_ptr(a), _ptr(b), _ptr(out), a.shape[0], op, _stream()), "fp_op")
    return out


def point_op(a_aff: torch.Tensor, b_aff: torch.Tensor, ks: torch.Tensor, op: int) -> torch.Tensor:
    n = a_aff.shape[0]
    out = torch.empty((n, 24), dtype=torch.int32, device=a_aff.device)
    _check(hip().bsc_point_op(_ptr(a_aff), _ptr(b_aff), _ptr(ks), _ptr(out), n, op, _stream()), "point_op")
    return out


def host_commit_key(d: int, secret: int = 2):
    """Reference commitment key PK[i] = secret^i * G1 (DistSys/publicKey.go:26-61)."""
    return rt().CommitKey.generate(d, secret)


def cu_masked_stream(device, skip_every: int = 4):
    """A torch stream bound to (1 - 1/skip_every) of the device's CUs (hipExtStreamCreateWithCUMask).

    Long-running speculative MSMs go there so the protocol's critical-path kernels keep a quarter
    of the CUs to themselves.  Returns (stream, cus_used); the HIP stream lives for the process."""
    import ctypes

    used = ctypes.c_int(0)
    with torch.cuda.device(device):
        ptr = hip().bsc_stream_create_cumask(int(skip_every), ctypes.byref(used))
    if not ptr:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    return torch.cuda.ExternalStream(ptr, device=device), used.value


def set_wave_priorities(on: bool) -> None:
    """The round kernels' wave priority classes (kernels/wave_prio.h) on or off, process-wide."""
    _check(hip().bsc_wave_prio(1 if on else 0), "wave_prio")


class NativeSpec:
    """Handle of a speculative share MSM launched by NativeSecAgg.spec_msm (same surface as the engine's
    _SpecShares: the MSM is already running; `ev` marks its end on the side stream)."""

    def __init__(self, qdelta, rows, rows_t, alive, pts, ys, no_commit):
        from ..utils import streams as S

        self.qdelta, self.rows, self.rows_t, self.alive, self.pts, self.ys = qdelta, rows, rows_t, alive, pts, ys
        self.no_commit, self.deferred = no_commit, False
        self.ev = None
        self.ev_flags = None   # the rows' flags are set (the selection's writes wait for it)
        self._S = S

    def record(self, side) -> None:
        self.ev = self._S.record(side)

    def launch(self) -> None:   # already running
        return None


class NativeSecAgg:
    """The round's device choreography, enqueued natively (kernels/round.hip) through a context that holds every
    resident buffer: the recovered-model ring, the recovery / audit outputs and their pinned read-backs, one
    entry per miner layout (index columns, exact recovery weights, outputs), the pre-step's slot ring and the
    softmax task.  They are registered once (add_layout, bind_task), so a phase is ONE call with a handful of
    arguments -- the round's host thread is its critical path:

      after_select     one rank, behind the committee's selection: speculative rows' flags, early audit
                       sums, the miners' sums + exact recovery + read-back, the next round's pre-step, the audit
      select_partials  several ranks (one per GPU): flags, early audit sums and this rank's partial sums into
                       a packed send row; the caller all_gathers the rows (main stream) ...
      after_gather     ... and this call sums the ranks' partials, recovers, reads back (clocks included),
                       queues the pre-step and the audit
      prestep          the pre-step alone (first round, host-decided rounds)

    A recovered model never lands in the buffer it is computed from nor in one of the last two results
    (bsc_round_pick_W): aggregates that are computed and then dropped (speculative misses, failed audits,
    empty blocks) cannot overwrite the live model."""

    W_RING = 4
    # a slot is rewritten PRE_SLOTS pre-steps later; a round can queue two (a speculative aggregate that is
    # dropped, then the host path's), and its commitment table may be read lazily in the next round's VRF
    # wait (deferred signing): four slots keep every reader clear of the rewrite
    PRE_SLOTS = 4

    def __init__(self, eng: DeviceCommitEngine, main, side, bg, qscale: float, witness=None):
        self.eng, dev = eng, eng.device
        d, nch, poly = eng.d, eng.nchunks, eng.poly
        self.ctx = hip().bsc_round_create(main.cuda_stream, side.cuda_stream, bg.cuda_stream, _ptr(eng.tbl_pk), d, poly,
                                          eng.T, eng.b0, eng.nw, float(qscale))
        if not self.ctx:
            raise RuntimeError("bsc_round_create failed")
        if witness is not None:   # the miners' witness sums off the background stream (its commitments first)
            _check(hip().bsc_round_set_witness_stream(self.ctx, witness.cuda_stream), "round_set_witness_stream")
        self.W_ring = [torch.empty((d,), dtype=torch.float64, device=dev) for _ in range(self.W_RING)]
        self.coeffs = torch.empty((nch, poly), dtype=torch.int64, device=dev)
        self.status = torch.empty((nch,), dtype=torch.int32, device=dev)
        self.cs = torch.empty((nch, 24), dtype=torch.int32, device=dev)
        self.ok = torch.empty((1, nch), dtype=torch.int32, device=dev)
        self.h_status = torch.empty((nch,), dtype=torch.int32, pin_memory=True)
        self.h_W = torch.empty((d,), dtype=torch.float64, pin_memory=True)
        self.h_ok = torch.empty((2, nch), dtype=torch.int32, pin_memory=True)   # two audits in flight (bsc_round_audit)
        import ctypes

        ring = (ctypes.c_void_p * self.W_RING)(*[t.data_ptr() for t in self.W_ring])
        _check(hip().bsc_round_bind_outputs(self.ctx, ring, self.W_RING, _ptr(self.coeffs), _ptr(self.status),
                                            _ptr(self.cs), _ptr(self.ok), self.h_status.data_ptr(), self.h_W.data_ptr(),
                                            self.h_ok.data_ptr()), "round_bind_outputs")
        self._layouts: list = []   # keeps each layout's tensors alive
        self.world = 0            # several ranks: set by gather_buffers()
        self.h_clock = None
        self._out = (ctypes.c_int * 2)()
        self.task = None
        self.slots: list = []

    # ---------------------------------------------------------------- registration (once per run)
    def add_layout(self, ccols, wcols, ycols, xs, wts: dict, A_dev, basis_dev) -> int:
        """Register one miner layout (its index columns and exact recovery weights) with resident outputs;
        returns its id for the per-round calls."""
        nch, dev = self.eng.nchunks, self.eng.device
        npts, nwc = ycols.numel(), wcols.numel()
        agg = torch.empty((nch, npts), dtype=torch.int64, device=dev)
        ws = torch.empty((max(nwc, 1), 24), dtype=torch.int32, device=dev)
        lid = hip().bsc_round_add_layout(self.ctx, _ptr(ccols), _ptr(wcols), nwc, _ptr(ycols), _ptr(xs), npts, _ptr(A_dev),
                                         _ptr(basis_dev), wts["shift"], wts["inv_lo"], wts["inv_hi"], _ptr(agg), _ptr(ws))
        if lid < 0:
            raise RuntimeError("bsc_round_add_layout failed (too many layouts?)")
        self._layouts.append((ccols, wcols, ycols, xs, A_dev, basis_dev, agg, ws))
        return lid

    def layout_agg(self, lid: int) -> torch.Tensor:
        return self._layouts[lid][6]

    def layout_ws(self, lid: int) -> torch.Tensor:
        return self._layouts[lid][7]

    def bind_task(self, task, gram_stream, noise_table, gram_counters, kchunk: int = 512) -> None:
        """The softmax task's resident data and the pre-step's slot ring (PRE_SLOTS slots of step outputs, chunk
        and full commitments, the noise-aware Gram).  noise_table: the resident [N, 100, d] noise table for the
        one-rank pre-step's Gram (None: no Gram in the pre-step)."""
        eng, dev = self.eng, self.eng.device
        P, d = len(task.peers), eng.d
        U2 = noise_table.shape[0] if noise_table is not None else 0
        U = P + U2
        Tt = (U + 15) // 16
        npairs, nsplit = Tt * (Tt + 1) // 2, (d + kchunk - 1) // kchunk
        self.pid = torch.tensor(task.peers, dtype=torch.int32, device=dev)
        self.rows_ar = torch.arange(P, dtype=torch.int32, device=dev)
        self.task, self.P, self.U2, self.gram_stream = task, P, U2, gram_stream
        self.noise_table = noise_table
        _check(hip().bsc_round_bind_task(self.ctx, gram_stream.cuda_stream, _ptr(task.X), _ptr(task.y), _ptr(task.off),
                                         _ptr(task.ntrain), _ptr(self.pid), task.d_in, task.d_out, task.batch, P,
                                         task.seed & (2 ** 64 - 1), 100.0, 1e4, task.peers[0], _ptr(eng.tbl_wb),
                                         _ptr(self.rows_ar), noise_table.data_ptr() if noise_table is not None else None,
                                         U2, kchunk, _ptr(gram_counters)), "round_bind_task")

        def ev():
            e = torch.cuda.Event()
            e.record(gram_stream)   # materialise the handle (re-recorded natively)
            return e
        for _ in range(self.PRE_SLOTS):
            sl = {"delta": torch.empty((P, d), dtype=torch.float32, device=dev),
                  "qdelta": torch.empty((P, d), dtype=torch.int64, device=dev),
                  "loss": torch.empty((P,), dtype=torch.float32, device=dev),
                  "ccom": torch.empty((P, eng.nchunks, 1, 24), dtype=torch.int32, device=dev),
                  "jac": torch.empty((P, 24), dtype=torch.int32, device=dev),
                  "host": torch.empty((P, 24), dtype=torch.int32, pin_memory=True),
                  "part": torch.empty((nsplit, npairs, 256), dtype=torch.float64, device=dev),
                  "gram": torch.empty((npairs, 256), dtype=torch.float64, device=dev),
                  "ev": [ev() for _ in range(4)]}
            e_step, e_ccom, e_commit, e_gram = sl["ev"]
            k = hip().bsc_round_add_pre_slot(self.ctx, _ptr(sl["delta"]), _ptr(sl["qdelta"]), _ptr(sl["loss"]),
                                             _ptr(sl["ccom"]), _ptr(sl["jac"]), sl["host"].data_ptr(), _ptr(sl["part"]),
                                             _ptr(sl["gram"]), e_step.cuda_event, e_ccom.cuda_event,
                                             e_commit.cuda_event, e_gram.cuda_event)
            assert k == len(self.slots), "pre-step slot registration out of order"
            self.slots.append(sl)
        self._spec_ring_for(P)   # every local peer can be a speculative row
        torch.cuda.synchronize(dev)

    def set_nn_table(self, tab) -> None:
        """The pre-step's noise-aware Gram copies its noise x noise tiles from tab ([100, N, N] fp64, None: computes
        them): see NoiseRows.gram_table."""
        self.nn_tab = tab
        _check(hip().bsc_round_set_nn_table(self.ctx, _ptr(tab) if tab is not None else None), "round_set_nn_table")

    def _pre_out(self, k: int, W, it: int) -> dict:
        """The engine's pre-step dict of slot k (the step of every local peer from W for iteration it)."""
        from ..protocol.crypto_backends import _PendingCommitments

        sl = self.slots[k]
        e_step, e_ccom, e_commit, e_gram = sl["ev"]
        pc = _PendingCommitments(sl["host"], e_commit, sl["jac"])
        pc.ccom, pc.ccom_event, pc.src, pc.slot = sl["ccom"], e_ccom, sl["qdelta"], k   # early audit sums
        out = {"W": W, "it": it, "delta": sl["delta"], "qdelta": sl["qdelta"], "ev": e_step, "commits": pc, "slot": k}
        self.task.last_loss = sl["loss"]
        if self.noise_table is not None and self.world <= 1:
            out["gram"] = {"gram": sl["gram"], "U1": self.P, "U": self.P + self.U2,
                           "keep": (sl["delta"], self.noise_table, sl["part"]), "ev": e_gram}
        return out

    # ---------------------------------------------------------------- per-round calls
    def prestep(self, W, it: int, do_gram: bool = True) -> dict:
        """The pre-step alone: the local step of every local peer from W (Gram stream, behind main), the chunk +
        full commitments (background stream, read back) and, one rank with a noise table, the noise-aware Gram."""
        k = hip().bsc_round_prestep_slot(self.ctx, _ptr(W), int(it), int(do_gram))
        if k < 0:
            raise RuntimeError(f"bsc_round_prestep_slot failed ({k})")
        return self._pre_out(k, W, it)

    def after_select(self, node, amap, sp, early_slot: int, upload, layout: int, W, audit: int, pre_it: int,
                     audit_now: bool = True):
        """One rank: everything behind the committee's selection in one call (see the class docstring).
        Returns (W_new, pre dict or None)."""
        o = self._out
        err = hip().bsc_round_after_select(self.ctx, _ptr(node) if node is not None else None, _ptr(amap),
                                           _ptr(sp.alive), len(sp.rows),
                                           _ptr(sp.rows_t), sp.ev.cuda_event, _ptr(sp.pts), _ptr(sp.ys), int(early_slot),
                                           upload.cuda_stream, int(layout), _ptr(W), int(audit), int(pre_it), 1,
                                           int(audit_now), o)
        if err != 0:
            raise RuntimeError(f"bsc_round_after_select failed ({err})")
        W_new = self.W_ring[o[0]]
        return W_new, (self._pre_out(o[1], W_new, pre_it) if o[1] >= 0 else None)

    # ---------------------------------------------------------------- several ranks
    def gather_buffers(self, world: int):
        """Resident (send [row_bytes], recv [world, row_bytes]) uint8 buffers of the aggregation's packed
        all_gather (layout: kernels/round.hip, bsc_round_row_bytes)."""
        if self.world != world:
            eng = self.eng
            self.row_bytes = int(hip().bsc_round_row_bytes(eng.nchunks, eng.T))
            self.send = torch.zeros((self.row_bytes,), dtype=torch.uint8, device=eng.device)
            self.recv = torch.zeros((world, self.row_bytes), dtype=torch.uint8, device=eng.device)
            self.h_clock = torch.empty((world,), dtype=torch.int64, pin_memory=True)
            self.world = world
        return self.send, self.recv

    def select_partials(self, node, amap, sp, early_slot: int, upload, layout: int, clock: int, audit: int) -> None:
        """Several ranks, before the all_gather: flags, early audit sums and this rank's partial sums of its kept
        rows into the send row (sp None: no local rows -- zero partials)."""
        assert self.world > 1, "gather_buffers() first"
        n = len(sp.rows) if sp is not None else 0
        err = hip().bsc_round_select_partials(
            self.ctx, _ptr(node) if n and node is not None else None, _ptr(amap) if n else None, _ptr(sp.alive) if n else None, n,
            _ptr(sp.rows_t) if n else None, sp.ev.cuda_event if n else None, _ptr(sp.pts) if n else None,
            _ptr(sp.ys) if n else None, int(early_slot), upload.cuda_stream, int(layout), self.send.data_ptr(),
            int(clock), int(audit))
        if err != 0:
            raise RuntimeError(f"bsc_round_select_partials failed ({err})")

    def after_gather(self, layout: int, W, audit: int, pre_it: int, audit_now: bool = True):
        """Several ranks, behind the all_gather into recv: (W_new, pre-step slot k or -1); the pre dict needs
        the caller's Gram gather (the deltas cross ranks)."""
        o = self._out
        err = hip().bsc_round_after_gather(self.ctx, self.recv.data_ptr(), self.world, self.row_bytes, int(layout),
                                           _ptr(W), self.h_clock.data_ptr(), int(audit), int(pre_it), int(audit_now), o)
        if err != 0:
            raise RuntimeError(f"bsc_round_after_gather failed ({err})")
        return self.W_ring[o[0]], o[1]

    # ---------------------------------------------------------------- several ranks, native collectives
    native_comm = False   # the round's collectives run in the fused calls (comm_init)

    def comm_init(self, comm, timeout_s: float = 0.0) -> bool:
        """The round's own collectives (kernels/round.hip bsc_round_comm_init): RCCL ranks share ONE communicator
        of their own -- rank 0's unique id travels over the job's process group once -- on the Comm's comm stream
        (every collective of the round, native or torch's, then runs there in issue order); a rank emulating rank 0
        of a larger job fills the other ranks' slots by device copies.  False: gloo (the round's collectives stay
        torch's)."""
        if comm.world < 2 or self.native_comm:
            return self.native_comm
        import ctypes
        import os

        if comm.emulating:
            _check(hip().bsc_round_comm_init(self.ctx, None, comm.world, 0, None, 1, 0.0), "round_comm_init")
        elif comm.backend == "nccl":
            import torch.distributed as dist

            # the RCCL instance torch runs (its librccl), not a second copy of the library
            _check(hip().bsc_rccl_load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so").encode()),
                   "rccl_load")
            uid = [None]
            if comm.rank == 0:
                buf = (ctypes.c_ubyte * 128)()
                _check(hip().bsc_rccl_unique_id(buf), "rccl_unique_id")
                uid = [bytes(buf)]
            dist.broadcast_object_list(uid, src=0)
            ub = (ctypes.c_ubyte * 128).from_buffer_copy(uid[0])
            cs = comm._comm_stream()
            torch.cuda.synchronize(self.eng.device)
            _check(hip().bsc_round_comm_init(self.ctx, ub, comm.world, comm.rank, cs.cuda_stream, 0,
                                             float(timeout_s or 0.0)), "round_comm_init")
        else:
            return False
        self.native_comm = True
        self.crank, self.cworld = comm.rank, comm.world
        return True

    def bind_multi(self, maxlocal: int, num_nodes: int, vg=None) -> None:
        """The fused multi-rank calls' resident buffers: the aggregation's packed rows (gather_buffers), and with the
        packed verification row vg (ops/gather.py) the next noise-aware Gram's inputs -- this rank's padded delta
        rows, the gathered [world maxlocal, d] deltas, the split-K partials of its tile pairs."""
        from . import ml as K

        assert self.native_comm and self.world == self.cworld, "comm_init() and gather_buffers() first"
        eng, dev, d = self.eng, self.eng.device, self.eng.d
        U1 = self.cworld * maxlocal
        p0, p1, chunk, _ = K.gram_split(U1 + num_nodes, self.crank, self.cworld)
        nsplit = (d + 511) // 512
        self.multi = {"pad": torch.zeros((maxlocal, d), dtype=torch.float32, device=dev),
                      "X": torch.empty((U1, d), dtype=torch.float32, device=dev),
                      "part": torch.empty((nsplit, max(1, p1 - p0), 256), dtype=torch.float64, device=dev),
                      "U1": U1, "U": U1 + num_nodes, "split": (self.crank, chunk, p0, p1), "vg": vg}
        mu = self.multi
        _check(hip().bsc_round_bind_multi(self.ctx, self.send.data_ptr(), self.recv.data_ptr(), self.row_bytes,
                                          self.h_clock.data_ptr(), maxlocal, _ptr(mu["pad"]), _ptr(mu["X"]),
                                          _ptr(mu["part"]), U1, p0, p1,
                                          vg.recv[0].data_ptr() if vg is not None else None,
                                          vg.recv[1].data_ptr() if vg is not None else None,
                                          vg.row_bytes if vg is not None else 0), "round_bind_multi")
        torch.cuda.synchronize(dev)

    def agg_multi(self, node, amap, sp, early_slot: int, upload, layout: int, clock: int, W, audit: int, pre_it: int,
                  audit_now: bool, gram: bool):
        """Several ranks with native collectives, behind the committee's selection in ONE call: partial sums, the
        aggregation's all_gather, totals + recovery + read-back + the next pre-step + the audit and (gram) the next
        noise-aware Gram's deltas gather and tile pairs.  Returns (W_new, pre-step slot or -1)."""
        n = len(sp.rows) if sp is not None else 0
        o = self._out
        err = hip().bsc_round_agg_multi(
            self.ctx, _ptr(node) if n and node is not None else None, _ptr(amap) if n else None,
            _ptr(sp.alive) if n else None, n, _ptr(sp.rows_t) if n else None, sp.ev.cuda_event if n else None,
            _ptr(sp.pts) if n else None, _ptr(sp.ys) if n else None, int(early_slot), upload.cuda_stream, int(layout),
            int(clock), _ptr(W), int(audit), int(pre_it), int(audit_now), int(gram), o)
        if err != 0:
            raise RuntimeError(f"bsc_round_agg_multi failed ({err})")
        return self.W_ring[o[0]], o[1]

    def multi_gram_pre(self, k: int, W, it: int, xrow) -> dict:
        """The pre dict of slot k whose noise-aware Gram agg_multi queued (its tile pairs in this rank's slot of
        iteration it's verification row; the packed exchange completes it)."""
        out = self._pre_out(k, W, it)
        mu = self.multi
        rank, chunk, p0, p1 = mu["split"]
        npairs = ((mu["U"] + 15) // 16) * ((mu["U"] + 15) // 16 + 1) // 2
        out["gram"] = {"gram": None, "U1": mu["U1"], "U": mu["U"], "split": (rank, chunk, npairs), "packed": True,
                       "keep": (mu["X"], mu["part"]), "xrow": xrow, "it": it, "ev": self.slots[k]["ev"][3]}
        return out

    SPEC_SLOTS = 3
    ROWARG_MAX = 248   # kernels/msm.hip: speculative rows that travel in the MSM kernel's arguments

    def _spec_ring_for(self, cap: int) -> dict:
        """The speculative MSM's resident output ring (SPEC_SLOTS slots of cap rows: shares, share values, the
        device row list + the rows' flags, pinned row staging), registered with the native context -- from then
        on each pre-step sets the next slot's flags inside its step."""
        ring = self.__dict__.get("_spec_ring")
        if ring is not None and ring["cap"] >= cap:
            return ring
        import ctypes

        eng, dev = self.eng, self.eng.device
        ring = self._spec_ring = {"cap": cap, "k": -1, "slots": [
            {"pts": torch.empty((cap, eng.nchunks, eng.T + 1, 24), dtype=torch.int32, device=dev),
             "ys": torch.empty((cap, eng.nchunks, eng.T), dtype=torch.int64, device=dev),
             "rows": torch.empty((2 * cap,), dtype=torch.int32, device=dev),   # [row list | flags]
             "host": torch.empty((cap,), dtype=torch.int32, pin_memory=True)}
            for _ in range(self.SPEC_SLOTS)]}
        alive = (ctypes.c_void_p * self.SPEC_SLOTS)(*[sl["rows"].data_ptr() + 4 * cap for sl in ring["slots"]])
        _check(hip().bsc_round_set_spec_ring(self.ctx, alive, self.SPEC_SLOTS, cap), "round_set_spec_ring")
        return ring

    def spec_msm(self, qdelta, rows: list, ev_wait, no_commit: bool, group_rows: int, up) -> "NativeSpec":
        """The speculative share MSM of qdelta[rows] on the side stream, behind ev_wait (a torch event: the
        pre-step), in one native call with resident outputs (a ring of SPEC_SLOTS: a slot is rewritten three
        launches later, after its witness sums -- the native side waits for them).  The row list travels in
        the kernel's arguments; its device copy (for the early audit sums) goes up on `up`.  Returns the handle
        the engine's aggregation uses (pts, ys, alive, rows_t, ev)."""
        n = len(rows)
        ring = self._spec_ring_for(max(n, qdelta.shape[0]))
        k = ring["k"] = (ring["k"] + 1) % self.SPEC_SLOTS
        sl, cap = ring["slots"][k], ring["cap"]
        lp = sl.get("launch")
        if lp is None:   # the slot's pointers and event handles, resolved once (the launch sits on the round's path)
            ev_up, ev_flags = torch.cuda.Event(), torch.cuda.Event()
            ev_up.record(up)   # materialise the handles (re-recorded natively)
            ev_flags.record(up)
            lp = sl["launch"] = (sl["host"].numpy(), sl["host"].data_ptr(), _ptr(sl["pts"]), _ptr(sl["ys"]),
                                 _ptr(sl["rows"]), ev_up, ev_flags, ev_up.cuda_event, ev_flags.cuda_event,
                                 _ptr(self.eng.tbl_wb))
        h_np, h_ptr, pts_p, ys_p, rows_p, ev_up, ev_flags, ev_up_h, ev_flags_h, wb_p = lp
        h_np[:n] = rows
        _check(hip().bsc_round_spec_msm2(self.ctx, k, ev_wait.cuda_event if ev_wait is not None else None,
                                         qdelta.data_ptr(), h_ptr, n, wb_p, 2 if no_commit else 0, int(group_rows),
                                         pts_p, ys_p, rows_p, up.cuda_stream, ev_up_h, ev_flags_h), "round_spec_msm2")
        # the handle's views, after the launch
        sp = NativeSpec(qdelta, rows, sl["rows"][:n], sl["rows"][cap:cap + n], sl["pts"][:n], sl["ys"][:n], no_commit)
        sp.ev_flags = ev_flags
        return sp

    def spec_topup(self, sp: "NativeSpec", keep, extra: list, group_rows: int, up, side) -> "NativeSpec":
        """A speculative miss: the block's rows missing from sp's MSM (local peer rows `extra`) computed into the same
        ring slot behind its rows, with the slot's flags re-set from the host-decided block (keep: int32 per sp row).
        Returns the handle of all n + m rows (its event: the top-up's end on the side stream).  None when sp is not
        the live slot's handle or the slot is too small (the caller recomputes the rows)."""
        ring = self.__dict__.get("_spec_ring")
        if ring is None:
            return None
        n, m, cap = len(sp.rows), len(extra), ring["cap"]
        slot = next((k for k, sl in enumerate(ring["slots"]) if sl["pts"].data_ptr() == sp.pts.data_ptr()), -1)
        if slot < 0 or n + m > cap or m > 248 or n + m == 0:
            return None
        sl = ring["slots"][slot]
        kh = sl.get("keep")
        if kh is None:
            kh = sl["keep"] = torch.empty((cap,), dtype=torch.int32, pin_memory=True)
        kn = kh.numpy()
        kn[:n] = keep
        kn[n:n + m] = 1
        hn = sl["host"].numpy()
        hn[n:n + m] = extra
        ev_up = torch.cuda.Event()
        ev_up.record(up)   # materialise the handle (re-recorded natively)
        _check(hip().bsc_round_spec_topup(self.ctx, slot, kh.data_ptr(), n, sl["host"].data_ptr() + 4 * n, m,
                                          sp.qdelta.data_ptr(), _ptr(self.eng.tbl_wb), 2 if sp.no_commit else 0,
                                          int(group_rows), sl["pts"][n:].data_ptr(), sl["ys"][n:].data_ptr(),
                                          sl["rows"].data_ptr() + 4 * n, up.cuda_stream, ev_up.cuda_event),
               "round_spec_topup")
        out = NativeSpec(sp.qdelta, list(sp.rows) + list(extra), sl["rows"][:n + m], sl["rows"][cap:cap + n + m],
                         sl["pts"][:n + m], sl["ys"][:n + m], sp.no_commit)
        out.record(side)
        out.ev_up = ev_up
        return out

    def readback(self, clocks: bool = False):
        """Callable: waits for the recovery's read-back -> [status, W_new(, every rank's clock)] numpy views
        (pinned)."""
        def wait():
            _check(hip().bsc_round_wait(self.ctx, 0), "round_wait")
            out = [self.h_status.numpy(), self.h_W.numpy()]
            if clocks:
                out.append(self.h_clock.numpy())
            return out
        return wait

    def audit(self, queue: bool = True):
        """Queue the aggregate audit on main (queue=False: a fused call queued it already); returns the
        callable giving ok int32 [1, nchunks]."""
        if queue:
            _check(hip().bsc_round_audit(self.ctx, _ptr(self.coeffs), _ptr(self.cs), _ptr(self.ok),
                                         self.h_ok.data_ptr()), "round_audit")

        k = int(hip().bsc_round_audit_slot(self.ctx))   # this audit's slot: a later one may be queued before the read

        def result():
            _check(hip().bsc_round_wait(self.ctx, 2 + k), "round_wait")
            return self.h_ok[k:k + 1].numpy()
        return result

    def close(self) -> None:
        if self.ctx:
            hip().bsc_round_destroy(self.ctx)
            self.ctx = None
