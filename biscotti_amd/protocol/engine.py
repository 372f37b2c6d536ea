"""The Biscotti round engine (SPMD over ranks, virtual peers per rank).

One call of :meth:`BiscottiEngine.run_round` performs everything one reference iteration does
across all N peer processes (DistSys/main.go prepareForNextIteration -> messageSender ->
VerifyUpdateKRUM -> RegisterSecret -> startShareDeadlineTimer -> createBlockSecAgg -> sendBlock):

  1. roles        native FSM: stake lottery on the latest block hash; noisers by each worker's
                  own ECVRF output (batched over host threads)
  2. local step   fused gfx950 kernel for all local workers (softmax / logistic regression)
  3. commitments  fixed-base MSM (commit-only pass) for every online worker
  4. noising      counter-based DP noise averaged over each worker's noisers
  5. verification one packed all_gather of commitments + noised deltas; the committee's Multi-Krum
                  (one f64-MFMA Gram, every verifier's selection on its own inbox, the
                  >= floor(nv/2) vote and the leader's NUM_SAMPLES/2 arrival cap) replicated on
                  every rank; Schnorr signatures of the local verifiers on native threads
  6. secure agg.  share/witness MSM of exactly the kept rows (launched by the selection kernel,
                  packed densely over the grid); per-rank partial share sums for every miner; ONE
                  packed all_gather of the partial sums + chunk-commitment sums + clocks; exact
                  recovery + W update replicated on every rank; device audit of the aggregate
                  against the summed chunk commitments
  7. block        every rank builds the leader's block (gob + SHA-256) from identical inputs and
                  the leader's clock; empty blocks on the reference's timeout paths
  8. evaluation   test error / attack rate (logged in the reference's line format)

Every decision (roles, inbox, approvals, share routing, leader quorum, block contents) comes from
the native :class:`RoundFSM`, replicated identically on every rank.
"""
from __future__ import annotations

import hashlib
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..native import rt
from ..ops import bn256 as B
from ..ops import ml as K
from ..parallel.comm import Comm
from ..utils import JsonlWriter, PhaseTimer, d2h_into, flush_logs, get_logger, h2d, h2d_many, pinned
from ..utils import streams as S
from .config import RunConfig


def _seed_bytes(seed: int, tag: str, i: int) -> bytes:
    return hashlib.sha256(f"{seed}:{tag}:{i}".encode()).digest()


def _bytes_as(b: torch.Tensor, dtype) -> torch.Tensor:
    """Reinterpret a 1-D uint8 slice of a received buffer as `dtype` (copying only if the slice is
    not aligned for it)."""
    isz = torch.empty((), dtype=dtype).element_size()
    if b.storage_offset() % isz:
        b = b.clone()
    return b.view(dtype)


@dataclass
class RoundResult:
    iteration: int
    block_hash: bytes
    empty: bool
    node_list: list = field(default_factory=list)
    approved: list = field(default_factory=list)
    verifiers: list = field(default_factory=list)
    miners: list = field(default_factory=list)
    test_error: float = float("nan")
    attack_rate: float = float("nan")
    phases: dict = field(default_factory=dict)
    wall: float = 0.0
    inboxes: dict = field(default_factory=dict)        # live verifier -> the updates it judged
    approved_by_krum: list = field(default_factory=list)  # updates at least one verifier accepted


class _Ready:
    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


class _PendingCommitments:
    def __init__(self, host: torch.Tensor, event, jac: torch.Tensor | None = None):
        self.host, self.event, self.value = host, event, None
        self.jac = jac   # device Jacobian rows (multi-rank rounds gather these, not host marshals)

    def result(self) -> np.ndarray:
        if self.value is None:
            self.event.synchronize()
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
    use: the signing reads the table rows natively, only the block's rows become bytes objects."""

    def __init__(self):
        super().__init__()
        self.table, self.row = None, {}

    def fill(self, table: np.ndarray, row: dict) -> None:
        self.table, self.row = table, row

    def __missing__(self, w):
        v = self[w] = self.table[self.row[w]].tobytes()
        return v


class _SpecShares:
    """Speculative share/witness MSM of some workers' rows on a side stream.  `alive` (int32, one
    flag per row) is cleared for rows the verifiers reject; the MSM skips flagged rows, whether the
    flags were cleared before it started or while it runs.  Consumers wait on `ev`."""

    def __init__(self, eng, qdelta: torch.Tensor, rows: list, stream, deferred: bool = False, group_rows: int = 0):
        self.eng, self.qdelta, self.rows, self.stream = eng, qdelta, rows, stream
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
            self.pts, self.ys = self.eng.shares(self.qdelta, self.rows_t, check_rows=False, alive=self.alive,
                                                compact=self.deferred, group_rows=self.group_rows)
            self.ev = torch.cuda.Event()
            self.ev.record(self.stream)
        # used on the side stream / allocated there and used on main: kept for two rounds (S.hold)
        S.hold(self.qdelta, self.alive, self.rows_t, self.pts, self.ys)


class DeviceCrypto:
    """GPU crypto backend: HBM-resident tables, Jacobian points [.., 24] int32."""

    def __init__(self, key, poly: int, T: int, device):
        self.eng = B.DeviceCommitEngine(key, poly, T, device)
        self.d, self.poly, self.T, self.nchunks = self.eng.d, poly, T, self.eng.nchunks

    def commitments_async(self, qdelta: torch.Tensor, stream=None):
        """Fixed-base MSM on device, queued download into pinned memory; result() waits for it and
        marshals on host with one batch inversion -> uint8 [n, 64].  The noise and Krum kernels
        queue behind the copy instead of waiting for the host to finish with the commitments."""
        n = qdelta.shape[0]
        if n == 0:
            return _Ready(np.zeros((0, 64), np.uint8))
        main = S.current()
        stream = stream or main
        S.wait(stream, main)
        with S.use(stream):
            rows = self._arange(n, qdelta.device)
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
        return _PendingCommitments(host, ev, jac)

    def commitments(self, qdelta: torch.Tensor) -> np.ndarray:
        return self.commitments_async(qdelta).result()

    def _arange(self, n: int, device) -> torch.Tensor:
        if not hasattr(self, "_ar") or self._ar.numel() < n:
            self._ar = torch.arange(max(n, 256), dtype=torch.int32, device=device)
        return self._ar[:n]

    def shares(self, qdelta: torch.Tensor):
        rows = torch.arange(qdelta.shape[0], dtype=torch.int32, device=qdelta.device)
        return self.eng.shares(qdelta, rows)

    def shares_async(self, qdelta: torch.Tensor, rows: list, stream, launch: bool = True,
                     group_rows: int = 0) -> "_SpecShares":
        """Shares + witnesses of qdelta[rows] on `stream` (the caller's work keeps flowing on its own
        stream).  launch=False prepares the per-row flags only; launch() then starts the MSM after
        everything queued so far on the caller's stream (e.g. Krum's selection), so rows already
        rejected cost nothing."""
        sp = _SpecShares(self.eng, qdelta, rows, stream, deferred=not launch, group_rows=group_rows)
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


class BiscottiEngine:
    def __init__(self, cfg: RunConfig, comm: Comm | None = None):
        cfg.validate()
        self.cfg = cfg
        self.comm = comm or Comm()
        self.R = rt()
        self.dev = self.comm.device if cfg.device != "cpu" else torch.device("cpu")
        self.gpu = self.dev.type == "cuda"
        self.N = cfg.num_nodes
        self.pc = cfg.protocol(self.R)
        self.local = self.comm.peer_range(self.N)
        self.lo = self.local.start
        self.maxlocal = self.comm.max_local(self.N)
        # peer -> row in a [world * maxlocal] gathered buffer
        self.flat = {p: r * self.maxlocal + (p - self.comm.peer_range(self.N, r).start)
                     for r in range(self.comm.world) for p in self.comm.peer_range(self.N, r)}
        tag = f"{cfg.log_dir}/log_{self.comm.rank}_{self.N}.log" if cfg.log_dir else None
        self.log = get_logger("peer", tag)
        self.trace = JsonlWriter(cfg.trace_file if self.comm.rank == 0 else None)
        # phase_sync: synchronise the device at every phase boundary so GPU time lands in its phase
        # (diagnostics); off, phase times are host-side and the device pipeline runs undisturbed
        self.timer = PhaseTimer(sync=(lambda: torch.cuda.synchronize(self.dev))
                                if self.gpu and cfg.phase_sync else None)
        # ---- data / model
        from ..data import dataset_dims
        from ..models import make_task

        self.d = dataset_dims(cfg.dataset)[0]
        fsm_probe = self.R.RoundFSM(self.pc, self.d)
        poisoned = {p for p in self.local if fsm_probe.is_poisoner(p)}
        colluders = {p for p in range(self.N) if fsm_probe.is_colluder(p)}
        self.colluders = colluders
        self.task = make_task(cfg.dataset, self.local, self.N, self.dev, cfg.seed, poisoned=poisoned,
                              batch_size=cfg.batch_size, data_dir=cfg.data_dir, epsilon=cfg.epsilon,
                              colluders=colluders)
        # ---- ledger / protocol state
        self.fsm = fsm_probe
        if cfg.peers_file:
            with open(cfg.peers_file) as f:
                addrs = [ln.strip() for ln in f if ln.strip()]
            if len(addrs) >= self.N:
                self.fsm.addresses = addrs[: self.N]
        if cfg.resume and cfg.chain_file:
            self._resume(cfg.chain_file)
        if cfg.chain_file:
            # every rank has read the file before rank 0 rewrites it: genesis, or the verified
            # prefix of a resumed chain (a torn final record left by a crash is dropped here)
            self.comm.barrier()
            if self.comm.rank == 0:
                self.fsm.chain.save(cfg.chain_file)
        self.W = torch.from_numpy(np.array(self.fsm.chain.latest().data.global_w, dtype=np.float64)).to(self.dev)
        # ---- keys
        if cfg.commit_key:
            key = self.R.CommitKey.load(cfg.commit_key, self.d)
        else:
            key = self.R.CommitKey.generate(self.d, 2)  # publicKey.go: s = 2
        self.T = self.pc.total_shares
        if self.gpu:
            # protocol critical path on a high-priority stream; speculative share MSMs on a
            # low-priority one so they fill the GPU while the host waits for VRF proofs / Krum
            lo, hi = torch.cuda.Stream.priority_range()
            self.main_cus = 0
            if cfg.main_stream_exclusive and cfg.side_stream_skip_every > 0:
                # the critical path on exactly the CUs the MSM stream leaves free (no SIMD sharing)
                self.main_stream, self.main_cus = B.cu_masked_stream(self.dev, -cfg.side_stream_skip_every)
            else:
                self.main_stream = torch.cuda.Stream(device=self.dev, priority=hi)
            # speculative MSMs: a stream masked to 3/4 of the CUs (critical path keeps the rest)
            self.side_stream, self.side_cus = B.cu_masked_stream(self.dev, cfg.side_stream_skip_every) \
                if cfg.side_stream_skip_every > 0 else (torch.cuda.Stream(device=self.dev, priority=lo), 0)
            # work no consumer in the round waits for (the miners' witness sums) runs here
            # (a CU mask complementing the MSM's was measured slower and removed: docs/PERF.md)
            self.bg_stream = torch.cuda.Stream(device=self.dev, priority=lo)
            # long device work nothing in a round waits for -- the VRF proofs (kernels/vrf.hip) and the
            # KZG audit sums (kernels/kzg.hip), ~5 ms launches -- gets a stream of its own: on the
            # background stream it would hold up the next round's commitments
            self.vrf_stream = torch.cuda.Stream(device=self.dev, priority=lo) \
                if cfg.vrf_device or cfg.kzg_audit != "off" else None
            # the pre-step's Krum Gram (_queue_pre_step): beside the main stream, so the evaluation and
            # the audit queued there do not wait for it
            self.gram_stream = torch.cuda.Stream(device=self.dev, priority=lo)
            # small uploads that must not queue behind any round work (_spec_head_launch)
            self.upload_stream = torch.cuda.Stream(device=self.dev, priority=hi)
            torch.cuda.synchronize(self.dev)   # everything set up so far is visible to the new streams
            torch.cuda.set_stream(self.main_stream)
        self.crypto = DeviceCrypto(key, cfg.poly_size, self.T, self.dev) if self.gpu else \
            HostCrypto(key, cfg.poly_size, self.T, cfg.host_threads)
        self.nchunks = self.crypto.nchunks
        if cfg.pkey_file:
            ks = self.R.read_client_keys(cfg.pkey_file)
            self.sk = {i: ks[i][0] for i in range(self.N)}
            self.pk = {i: ks[i][1] for i in range(self.N)}
        else:
            self.sk, self.pk = {}, {}
            for i in range(self.N):
                s, p = self.R.client_key_from_entropy(_seed_bytes(cfg.seed, "client", i))
                self.sk[i], self.pk[i] = s, p
        # every peer's VRF seeds (the multi-rank noise-aware Krum replicates the noiser lottery, whose
        # outputs are publicly verifiable, on every rank); churn epochs are replicated too
        self.vrf_noise_seed = {i: _seed_bytes(cfg.seed, "vrf-noise", i) for i in range(self.N)}
        self.vrf_roles_seed = {i: _seed_bytes(cfg.seed, "vrf-roles", i) for i in range(self.N)}
        self.sigma = self.task.noise_sigma(cfg.epsilon)
        # every noiser's 100 pre-sampled noise vectors resident in HBM (314 MB for MNIST x 100 peers)
        self.noise_tbl = None
        if self.gpu and cfg.noising and cfg.noise_table and self.sigma > 0 and self.N * 100 * self.d * 4 <= (8 << 30):
            self.noise_tbl = K.noise_table(self.N, self.d, cfg.seed, self.dev)
        self.vrf_dev = None
        if self.gpu and cfg.vrf_device:
            from ..ops.vrf import DeviceVrfProver
            self.vrf_dev = DeviceVrfProver(self.dev, cfg.vrf_device_batch_rounds)
        self._side_work: list = []   # (event, tensors) of off-critical-path device work of this round
        self._agg_idx: dict = {}      # (contributing, parts) -> resident aggregation index tensors
        self._W_next = None          # device copy of the model a block under construction carries
        self._pre = None             # next round's local step + commitments, queued behind the recovery
        self._early_vrf = None       # next round's VRF outputs, started as soon as the block hash exists
        self._pinned: dict = {}      # persistent pinned read-back buffers (_d2h_async)
        self._evals: list = []       # (result, evaluation read-back) of rounds not resolved yet (lazy_eval)
        self._pre_vrf_work: list = []  # host work for the next round's VRF wait (deferred signature prep)
        self._sign_joins: list = []
        self._stale_vrf: list = []     # early VRF batches the next head did not adopt (joined by drain)
        self._spec_next = None        # next round's share MSM launched at block build (_spec_head_launch)  # deferred signature joins of the last rounds (secure path)
        self.stats = {"unmasked_updates": 0, "total_updates": 0, "audit_failures": 0}
        # batched verifySecret audit (K13): G2 side = (g2key[0], g2key[1]) = (G2, s G2)
        self._kzg_pending: list = []   # launched audits (device) or checked ones (CPU)
        self._kzg_stage: list = []     # rounds waiting for the next device launch
        if cfg.kzg_audit != "off":
            self.stats.update(kzg_checks=0, kzg_failures=0)
            self._kzg_g2 = (self.R.g2_generator(), self._commit_key_g2_1(cfg.commit_key))
            self._kzg_rng = np.random.default_rng([cfg.seed, self.comm.rank, 0x6B7A67])
        self._churn = {"down": {}, "view": {}, "epoch": {}, "acc": 0.0, "kills": 0, "rejoins": 0,
                       "synced_blocks": 0}
        self.stats["churn"] = self._churn
        self.rounds_done = 0
        self._partitions = cfg.partitions()
        self._head = None
        if self.gpu and cfg.secure_agg and 0 < cfg.num_miners <= 4:
            # every full-quorum miner layout's aggregation indices and exact recovery weights (~8 ms of
            # host work each, the parts are a permutation of 0..M-1) at setup, not in the first rounds
            # that meet them; layouts with offline miners are still built on first use
            import itertools

            M = cfg.num_miners
            for perm in itertools.permutations(range(M)):
                self._agg_index(list(range(M)), {i: perm[i] for i in range(M)})
        if self.vrf_dev is not None:
            # every peer's VRF key material (secret scalar, nonce prefix, public key: a fixed-base
            # multiplication each) derived and cached now -- the host batches and the device prover's
            # key table share the cache -- instead of inside the first rounds
            self.vrf_dev._rows(list(self.vrf_noise_seed.values()) + list(self.vrf_roles_seed.values()))
            # one proof now: the prover kernel's code object is loaded at its first launch (several ms),
            # which would otherwise land in the round that fills the first 16-round batch
            with S.use(self.vrf_stream):
                self.vrf_dev.prove([self.vrf_noise_seed[0]], [bytes(self.vrf_dev.ALPHA_LEN)])
            torch.cuda.synchronize(self.dev)
            self.vrf_dev.proofs = 0
        import atexit
        import weakref
        ref = weakref.ref(self)
        atexit.register(lambda: ref() is not None and ref().close())
        # everything allocated so far (torch, datasets, keys, tables) lives for the whole run: move it
        # out of the cyclic collector's generations, so an occasional full collection scans only
        # the rounds' garbage instead of pausing a round for ~0.1 s
        import gc
        gc.collect()
        gc.freeze()

    # ------------------------------------------------------------------ lifecycle
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

    def _kzg_queue(self, csum, wsum, ys, xs_t, it) -> None:
        """Stage this round's aggregate for the device RLC sums (on the audit stream, current here);
        kzg_batch_rounds rounds with the same share-point layout go into ONE launch and one pairing
        product, read back and checked later (_kzg_poll), off the round's critical path."""
        npts = ys.shape[1]
        spm = self.pc.shares_per_miner
        if self._kzg_stage and self._kzg_stage[0]["npts"] != npts:
            self._kzg_launch()
        wperm = wsum.index_select(0, self.crypto.eng.kzg_order(npts, spm))   # (chunk, point) order
        self._kzg_stage.append({"cs": csum, "ws": wperm, "ys": ys, "xs": xs_t, "npts": npts, "it": it})
        if len(self._kzg_stage) >= self.cfg.kzg_batch_rounds:
            self._kzg_launch()

    def _kzg_launch(self) -> None:
        st, self._kzg_stage = self._kzg_stage, []
        if not st:
            return
        with S.use(self.vrf_stream):
            cat = lambda k: torch.cat([e[k] for e in st]) if len(st) > 1 else st[0][k]
            npts = st[0]["npts"]
            pts = self.crypto.eng.kzg_rlc(cat("cs"), cat("ws"), cat("ys"), torch.stack([e["xs"] for e in st]),
                                          npts, self.cfg.kzg_audit == "literal",
                                          int(self._kzg_rng.integers(0, 2**63)))
            host = torch.empty((3, 24), dtype=torch.int32, pin_memory=True)
            host.copy_(pts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.vrf_stream)
        self._kzg_pending.append({"its": [e["it"] for e in st], "ev": ev, "host": host, "job": None})

    def _kzg_host(self, cs, ws, ys, xs, it) -> None:
        """CPU path: the same random linear combination on the host (native threads)."""
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
                    self.stats["kzg_failures"] += len(e["its"])
                    self.log.info("KZG audit (verifySecret, %s) failed for the aggregates of iterations %s",
                                  self.cfg.kzg_audit, e["its"])
            else:
                keep.append(e)
        self._kzg_pending = keep

    def _resolve_evals(self) -> None:
        """Read the queued evaluations of earlier rounds (lazy_eval) into their results and log them."""
        evs, self._evals = self._evals, []
        for res, f in evs:
            ev = f()
            res.test_error, res.attack_rate = ev["test_error"], ev["attack_rate"]
            self._log_round(res)

    def drain(self, final: bool = True) -> None:
        """Join work that belongs to rounds already returned: the last host VRF batch and, when
        final, the outstanding KZG audits and the device VRF proofs still queued or in flight."""
        if final:
            if self._kzg_pending or self._kzg_stage:
                self._kzg_poll(final=True)
            if self.vrf_dev is not None and getattr(self, "vrf_stream", None) is not None:
                self.vrf_dev.drain(self.vrf_stream)
                self.stats["vrf_device_proofs"] = self.vrf_dev.proofs
        if final:   # the last deferred signature batch (each round joins the previous one's)
            work, self._pre_vrf_work = self._pre_vrf_work, []
            for f in work:
                f(None)
            joins, self._sign_joins = self._sign_joins, []
            for join in joins:
                join()
        if final:
            self._resolve_evals()
        self._stale_vrf = [j for j in self._stale_vrf if not j.done()] if not final else []
        futs, self._pending_roles = getattr(self, "_pending_roles", None), None
        for fut in futs or ():
            if fut is not None:
                fut.wait()   # the proofs themselves are discarded: no Python objects built

    def close(self) -> None:
        """Join the pre-opened round's native VRF jobs and drain the device.  Idempotent; also
        registered with atexit so interpreter teardown never races native threads."""
        flush_logs(self.log)
        self.drain()
        head, self._head = self._head, None
        if head:
            for k in ("fut_noise", "fut_roles"):
                if head.get(k) is not None:
                    head[k].result()
        head = None  # drop the round's tensors while their streams are all still alive
        if self.gpu:
            torch.cuda.synchronize(self.dev)
            S.clear_holds()
        self._side_work = []
        self._agg_idx.clear()   # resident index tensors were used on the side stream destroyed below
        import gc
        gc.unfreeze()   # the engine's own reference cycles become collectable again (see __init__)
        if self.gpu and getattr(self, "side_stream", None) is not None:
            torch.cuda.synchronize(self.dev)
            torch.cuda.set_stream(torch.cuda.default_stream(self.dev))
            # the HBM-resident tables (up to ~90 GB) go now, not whenever the engine is collected
            if isinstance(self.crypto, DeviceCrypto):
                self.crypto.eng.release()
            self.noise_tbl = None
            if getattr(self, "side_cus", 0):
                # every tensor used on the CU-masked stream is gone (round locals, the head above):
                # flush the allocator's stream-use events, then release the stream before
                # interpreter teardown (the HIP runtime must not be left to destroy it at exit)
                gc.collect()
                torch.cuda.synchronize(self.dev)
                torch.cuda.empty_cache()
                B.hip().bsc_stream_destroy(self.side_stream.cuda_stream)
            if getattr(self, "main_cus", 0):
                B.hip().bsc_stream_destroy(self.main_stream.cuda_stream)
                self.main_cus = 0
            self.side_stream = None

    # ------------------------------------------------------------------ helpers
    def _now(self, iteration: int) -> int:
        return iteration + 1 if self.cfg.deterministic_time else int(time.time())

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

    def _rows_buffer(self, per_peer: dict, width: int, dtype) -> torch.Tensor:
        """[maxlocal, width] buffer whose row (peer - lo) holds that local peer's vector."""
        buf = torch.zeros((self.maxlocal, width), dtype=dtype, device=self.dev)
        for p, v in per_peer.items():
            buf[p - self.lo] = v
        return buf

    def _gathered_row(self, g: torch.Tensor, peer: int) -> torch.Tensor:
        r = self.comm.owner(peer, self.N)
        return g[r, peer - self.comm.peer_range(self.N, r).start]

    # ------------------------------------------------------------------ the round
    def _open_round(self) -> dict:
        """Round head: live set, committee plan and the asynchronous noiser / roles VRF proofs.

        It depends only on the latest block, so it is opened as soon as that block is committed
        (overlapping the previous round's evaluation and logging) and consumed by run_round."""
        cfg, R, fsm = self.cfg, self.R, self.fsm
        with self.timer.phase("head.plan"):
            live = self._live_mask()
            plan = fsm.begin_round(live)
        head = {"live": live, "plan": plan}
        if plan.done:
            return head
        latest_hash = fsm.chain.latest().hash
        workers = [w for w in plan.workers if live[w]]
        local_workers = [w for w in workers if w in self.local]
        head.update(workers=workers, local_workers=local_workers, stake=dict(fsm.stake))
        # noisers: each worker's own ECVRF over the latest block hash (vrf.go:54-100).  Only the
        # 64-byte outputs gate the round (the noiser lottery -> noise -> Krum -> the selection that
        # cancels speculative MSM rows), and they need nothing but the plan and the block hash: they
        # start first, on host_threads - 1 native threads (the launching thread keeps a core); the
        # proofs nothing reads run on the device (vrf_device) or after the outputs on the host.
        # Several ranks with the noise-aware Krum: every rank evaluates the committee over every
        # worker, so it needs every worker's noisers -- each rank replicates the (publicly verifiable)
        # VRF outputs instead of a gather after them; only the local proofs are produced here.
        mr_pre = (self.gpu and self.comm.world > 1 and cfg.secure_agg and cfg.verification and cfg.defense == "KRUM"
                  and cfg.noising and self.sigma > 0 and self.noise_tbl is not None and not cfg.noise_independent
                  and cfg.krum_pregram)
        vrf_workers = workers if mr_pre else local_workers
        head["vrf_workers"] = vrf_workers
        with self.timer.phase("head.vrf_submit"):
            seeds = [self.vrf_noise_seed[w] for w in local_workers]
            dev = self.vrf_dev is not None
            nthr = max(1, cfg.host_threads - 1) if self.gpu else cfg.host_threads
            vseeds = seeds if vrf_workers is local_workers else [self.vrf_noise_seed[w] for w in vrf_workers]
            ej, self._early_vrf = self._early_vrf, None
            fut_noise = None
            if ej is not None and vseeds and ej["hash"] == bytes(latest_hash):
                # the outputs started when the block was built (_early_vrf_submit): adopt them if they
                # cover these workers with the same keys
                pos = ej["pos"]
                if all(w in pos and ej["seeds"][pos[w]] == self.vrf_noise_seed[w] for w in vrf_workers):
                    fut_noise = ej["job"]
                    head["vrf_index"] = [pos[w] for w in vrf_workers]
                    self.stats["early_vrf"] = self.stats.get("early_vrf", 0) + 1
            if ej is not None and fut_noise is not ej["job"]:
                # not adopted (a failed audit changed the block, or a restart its keys): joined later,
                # not here -- dropping a running job would wait for it
                self._stale_vrf.append(ej["job"])
            if fut_noise is None:
                fut_noise = R.vrf_prove_batch_async(vseeds, latest_hash, nthr, None, dev) if vseeds else None
            fut_roles = None
            roles = [self.vrf_roles_seed[p] for p in self.local if live[p]] if cfg.roles_vrf_proof else []
            if roles and not dev:  # getVRFRoles proves with the roles key too (result unused, Q7)
                fut_roles = R.vrf_prove_batch_async(roles, latest_hash, cfg.roles_vrf_threads, fut_noise)
        head.update(fut_noise=fut_noise, fut_roles=fut_roles)
        # the local step, the commitments and the speculative shares depend only on the new global
        # model too: queue them now, behind nothing but the block that produced it
        tm, it = self.timer, plan.iteration
        # the local step (and the commitments) may already be in flight: queued behind the recovery of
        # the model this head starts from (_queue_pre_step), for every local peer
        pre, self._pre = self._pre, None
        use_pre = pre is not None and pre["it"] == it and pre["W"] is self.W and bool(local_workers)
        with tm.phase("local_step"):
            if use_pre:
                self.stats["pre_steps"] = self.stats.get("pre_steps", 0) + 1
                S.current().wait_event(pre["ev"])   # the step ran on the Gram stream
                qdelta, qrow = pre["qdelta"], {w: w - self.lo for w in local_workers}
                delta = pre["delta"]
                # with the pre-step's Krum Gram (rows = every local peer) nothing reads the workers'
                # delta rows alone; otherwise they are selected once here
                if len(local_workers) != delta.shape[0] and not (
                        pre.get("gram") is not None and self.comm.world == 1 and self._noise_krum()
                        and cfg.verification):
                    delta = delta.index_select(0, h2d([w - self.lo for w in local_workers], torch.long, self.dev))
            else:
                delta, qdelta = self.task.step(self.W, it, local_workers)
                qrow = None
        with tm.phase("commit"):
            # every live verifier collects its own first krum_thresh arrivals (krum.go:284-322); only
            # updates that can end in the leader's block secret-share: the MSM runs on the CU-masked
            # side stream, launched by the committee's selection (only the kept rows are computed) or,
            # with spec_msm, speculatively over every candidate (rows rejected later are cancelled)
            inboxes = {}
            sn, self._spec_next = self._spec_next, None
            if sn is not None and not (use_pre and pre is sn["pre"] and sn["hash"] == bytes(latest_hash)
                                       and sn["it"] == plan.iteration and sn["verifiers"] == list(plan.verifiers)
                                       and sn["miners"] == list(plan.miners) and sn["workers"] == workers
                                       and all(live)):
                sn = None   # the committed block or the plan differs: the speculative MSM is not used
            if sn is not None:
                inboxes = sn["inboxes"]
            elif cfg.verification:
                for v, ib in zip(plan.verifiers, fsm.verifier_inboxes(workers)):
                    if live[v]:
                        inboxes[v] = list(ib)
            # rows of delta (Krum, noise): the workers in order, or every local peer (unselected pre-step)
            row_of = {w: i for i, w in enumerate(local_workers)} if delta.shape[0] == len(local_workers) else \
                {w: w - self.lo for w in local_workers}
            qrow = qrow or row_of                                   # rows of qdelta (MSMs, commitments)
            spec = None
            cand = set()
            if self.gpu and cfg.secure_agg and sn is None:
                # replicated on every rank: the rows (of all ranks) whose shares are computed up front
                cand = self._block_candidates(plan, workers, inboxes)
                cap = fsm.leader_cap_size()
                if cfg.verification and cfg.spec_msm and cap > 0 and cfg.spec_group_rows <= 0:
                    # the block carries the first `cap` approved updates in leader arrival order, so the
                    # speculative MSM covers a prefix of that order with margin for rejections
                    k = min(len(cand), int(np.ceil(cfg.spec_margin * cap)) + 2)
                    cand = set([w for w in fsm.leader_arrivals() if w in cand][:k])
            if sn is not None:
                # launched at the previous block's build (_spec_head_launch), from this very plan
                cand, spec, head["arrivals"] = sn["cand"], sn["spec"], sn["arrivals"]
                self.stats["spec_head"] = self.stats.get("spec_head", 0) + 1
            elif self.gpu and cfg.secure_agg and local_workers:
                # speculative rows in leader arrival order: with spec_group_rows the MSM works through
                # them in that order, and once the committee's selection lands (set_alive) the rows
                # outside the leader's block are skipped when reached -- the block's rows are the first
                # approved arrivals, so by then most of them are done and no candidate is ever missing
                arrivals = head["arrivals"] = fsm.leader_arrivals()   # once per round (Krum's ranks reuse it)
                lo_rank = {w: i for i, w in enumerate(arrivals)}
                spec_workers = sorted((w for w in local_workers if w in cand), key=lambda w: lo_rank.get(w, 1 << 30))
                if spec_workers:
                    defer = cfg.verification and not cfg.spec_msm
                    spec = (spec_workers, self.crypto.shares_async(qdelta, [qrow[w] for w in spec_workers],
                                                                   self.side_stream, launch=not defer,
                                                                   group_rows=cfg.spec_group_rows))
            # full-vector commitments on the background stream: their first consumer is the signing
            # after Krum, so noise + Krum on the main stream do not queue behind them
            pending_commits = pre["commits"] if use_pre else \
                self.crypto.commitments_async(qdelta, self.bg_stream if self.gpu else None)
        # one rank, Multi-Krum over table noise: the d-dimensional part of the committee's Krum (the
        # Gram of the deltas stacked over the noisers' pre-sampled vectors of this iteration) depends
        # only on this head, so it runs now, while the host computes the workers' VRF outputs; after
        # the noisers are known only an O(n^2) assembly remains (ml.hip k_krum_rows_noise)
        krum_pre = None
        if self.comm.world == 1 and self._noise_krum() and inboxes and local_workers:
            with tm.phase("verify.pregram"):
                # adopted from the pre-step (rows = every local peer) or launched now (rows = workers)
                krum_pre = pre.get("gram") if use_pre else None
                if krum_pre is None:
                    krum_pre = K.gram_stacked_async(delta, self.noise_tbl[:, it % 100, :])
        elif mr_pre and inboxes and workers:
            # several ranks: ONE all_gather of the deltas right here (the first collective of the round),
            # then every rank runs the same phase-1 Gram over [every worker's delta; noise rows] while
            # the VRF outputs are computed -- the commitments travel later, off Krum's path
            with tm.phase("verify.pregram"):
                buf = torch.zeros((self.maxlocal, self.d), dtype=torch.float32, device=self.dev)
                if local_workers:
                    buf.index_copy_(0, h2d([w - self.lo for w in local_workers], torch.long, self.dev), delta)
                g = self.comm.all_gather(buf).reshape(-1, self.d)
                Xw = g.index_select(0, h2d([self.flat[w] for w in workers], torch.long, self.dev)).contiguous()
                krum_pre = K.gram_stacked_async(Xw, self.noise_tbl[:, it % 100, :])
                krum_pre["xrow"] = {w: i for i, w in enumerate(workers)}
                # the commitments' all_gather right behind it, from the background stream (it waits for
                # the commitments only), with an asynchronous read-back of the workers' rows: the
                # signing and the block read them without a device sync behind Krum's aggregation
                cr, bg = self.crypto, self.bg_stream
                with S.use(bg):
                    part = torch.zeros((self.maxlocal, cr.point_width), dtype=cr.point_dtype, device=self.dev)
                    if local_workers:
                        part.index_copy_(0, h2d([w - self.lo for w in local_workers], torch.long, self.dev),
                                         self._local_commit_rows(pending_commits, local_workers, qrow))
                    g = self.comm.all_gather(part).reshape(-1, cr.point_width)
                    rows_w = g.index_select(0, h2d([self.flat[w] for w in workers], torch.long, self.dev))
                    host = pinned("commit_gather", rows_w.shape, rows_w.dtype)
                    d2h_into(host, rows_w.contiguous())
                    head["commit_gather"] = (host, S.record(bg))
        head.update(delta=delta, qdelta=qdelta, pending_commits=pending_commits, inboxes=inboxes, row_of=row_of,
                    qrow=qrow, spec=spec, spec_cand=cand, krum_pre=krum_pre)
        if self.vrf_dev is not None:
            # the proofs nobody reads -- every noiser proof and the roles proofs -- on the device,
            # several rounds per launch on their own low-priority stream
            self.vrf_dev.submit(seeds + roles, latest_hash, self.vrf_stream)
        # one rank, Multi-Krum: the noise and committee-Krum kernels (and, behind the selection, the
        # whole device-side aggregation) depend only on this head, so they can be queued now as well
        if (cfg.early_krum and self.gpu and self.comm.world == 1 and cfg.secure_agg and cfg.defense == "KRUM"
                and inboxes and spec is not None and cfg.noising and self.sigma > 0 and fut_noise is not None):
            # (queued last: it waits for the VRF outputs on the host)
            with tm.phase("vrf_join"):
                noisers = self._select_noisers(fut_noise, head["stake"], local_workers, head.get("vrf_index"))
            with tm.phase("noise"):
                noised = None if krum_pre is not None else self._noise(delta, noisers, local_workers, it)
            with tm.phase("verify.launch"):
                box: dict = {}
                pg = krum_pre is not None and "row_peers" in krum_pre   # the pre-step's Gram: rows = local peers
                wait = self._launch_krum(noised, krum_pre["xrow"] if pg else row_of, plan, live, inboxes, spec, box,
                                         pre=krum_pre, noisers=noisers,
                                         local_workers=krum_pre["row_peers"] if pg else local_workers)
            head["early"] = {"noisers": noisers, "krum": wait, "box": box, "noised": noised}
        return head

    def _block_candidates(self, plan, workers, inboxes) -> set:
        """Workers whose update can end in this round's block: without verification every live worker
        (capped to the leader's first arrivals); with it, every update some live verifier judges --
        or every live worker when floor(nv/2) == 0 signatures suffice (the nv = 1 quirk,
        main.go:1686: updates no verifier saw are approved too)."""
        if not self.cfg.verification:
            return set(self.fsm.leader_cap(workers))
        if len(plan.verifiers) // 2 == 0:
            return set(workers)
        out: set = set()
        for ib in inboxes.values():
            out.update(ib)
        return out

    def _select_noisers(self, fut_noise, stake, local_workers, index=None) -> dict:
        """Each worker's noisers from its own VRF output (getVRFNoisers, vrf.go:54-100).  Waits for
        the outputs only; the proofs finish on the native threads and are joined at round end.
        index: positions of local_workers in the job's output list (an early job covers more peers)."""
        if fut_noise is None or not local_workers:
            return {}
        # the lottery reads the job's outputs natively (no 64-byte Python objects in between)
        sel = self.R.select_noisers_job(stake, fut_noise, list(index) if index is not None else [], local_workers,
                                        self.cfg.num_noisers, self.N)
        return dict(zip(local_workers, sel.tolist()))

    def _noise_scales(self, noisers: dict, ws: list) -> np.ndarray:
        """float32 [len(ws), nn]: each noiser's vector weight (getNoise's -sigma/sqrt(B)); 0 for
        colluding noisers (isCollusionAttack, main.go:1026-1057)."""
        ids = np.asarray([noisers[w] for w in ws], np.int64).reshape(len(ws), -1)
        sc = np.full(ids.shape, self.task.noise_scale(self.sigma), np.float32)
        if self.colluders:
            sc[np.isin(ids, np.fromiter(self.colluders, np.int64))] = 0.0
        return sc

    def _noise(self, delta, noisers, local_workers, it):
        """Noised deltas of the local workers (requestNoise + NoisedDelta, main.go:1513-1660): each
        worker's noisers' pre-sampled vectors averaged and added (HBM-resident table on the GPU)."""
        cfg = self.cfg
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
        return K.dp_noise(delta, nz, sc, cfg.seed, it, table=self.noise_tbl)

    def _sign_threads(self) -> int:
        """Threads of a signature batch: cfg.sign_threads (0: all but one of host_threads).  A narrow
        batch leaves most of the pool to the VRF outputs that gate the next round."""
        n = self.cfg.sign_threads
        return max(1, n if n > 0 else self.cfg.host_threads - 1)

    def _krum_static(self, xrow, U, plan, live, inboxes, spec, arrivals=None) -> dict:
        """The part of a Krum launch that does not depend on the noisers (inbox rows, leader arrival
        ranks, Krum row -> speculative MSM row), uploaded in ONE copy.  run_round prepares it while
        the host still waits for the VRF outputs."""
        fsm = self.fsm
        vs = [v for v in plan.verifiers if v in inboxes]
        n = len(inboxes[vs[0]])
        inbox_np = np.asarray([[xrow[w] for w in inboxes[v]] for v in vs], np.int32)
        rank = np.full(U, -1, np.int32)
        for r, w in enumerate(arrivals if arrivals is not None else fsm.leader_arrivals()):
            if live[w] and w in xrow:
                rank[xrow[w]] = r
        ups = [(inbox_np, torch.int32), (rank, torch.int32)]
        if spec is not None:
            amap = np.full(U, -1, np.int32)
            amap[[xrow[w] for w in spec[0]]] = np.arange(len(spec[0]), dtype=np.int32)
            ups.append((amap, torch.int32))
        got = h2d_many(ups, self.dev)
        return {"U": U, "n": n, "clip": fsm.krum_clip(n), "need": len(plan.verifiers) // 2,
                "cap": fsm.leader_cap_size(), "inbox": got[0], "rank": got[1],
                "amap": got[2] if spec is not None else None}

    def _launch_krum(self, X, xrow, plan, live, inboxes, spec, box, pre=None, noisers=None, local_workers=None,
                     static=None):
        """Queue the committee's Multi-Krum (one Gram over the candidate rows X, every live verifier's
        selection on its own inbox, the >= floor(nv/2) vote and the leader's arrival cap) and, behind
        it, the device-side follow-up of the selection (_on_accept).  xrow: worker -> row of X.
        pre: the phase-1 Gram of gram_stacked_async (X is then None: the noised rows are assembled
        from it with the noisers' ids and scales).  Returns the callable giving (acc, node)."""
        U = X.shape[0] if X is not None else pre["U1"]
        st = static if static is not None and static["U"] == U else self._krum_static(xrow, U, plan, live, inboxes, spec)
        n, clip, need, cap = st["n"], st["clip"], st["need"], st["cap"]
        ups = []
        if pre is not None:
            # one (noisers, scales) row per Gram row; rows of peers that are not workers this round
            # (the pre-step's Gram covers every local peer) are never in an inbox: zero weights
            ws = [w for w in local_workers if w in noisers]
            if len(ws) == len(local_workers):
                nz_np = np.asarray([noisers[w] for w in local_workers], np.int32)
                sc_np = self._noise_scales(noisers, local_workers)
            else:
                nn_ = len(noisers[ws[0]]) if ws else 1
                nz_np = np.zeros((len(local_workers), nn_), np.int32)
                sc_np = np.zeros((len(local_workers), nn_), np.float32)
                if ws:
                    at = np.asarray([i for i, w in enumerate(local_workers) if w in noisers])
                    nz_np[at] = np.asarray([noisers[w] for w in ws], np.int32)
                    sc_np[at] = self._noise_scales(noisers, ws)
            ups += [(nz_np, torch.int32), (sc_np, torch.float32)]
        inbox_t, rank_t, amap_t = st["inbox"], st["rank"], st["amap"]
        on_accept = self._on_accept(spec, amap_t, plan, live, box)
        if pre is not None:
            nz, sc = h2d_many(ups, self.dev)   # the noisers' ids and weights: ONE upload
            if "ev" in pre:   # produced on the Gram stream
                S.current().wait_event(pre["ev"])
            return K.krum_committee_noise_async(pre, nz, sc, inbox_t, n - clip, n - clip, need, rank_t, cap,
                                                on_accept=on_accept)
        return K.krum_committee_async(X, inbox_t, n - clip, n - clip, need, rank_t, cap, on_accept=on_accept)

    def _on_accept(self, spec, amap_t, plan, live, box):
        """Device-side follow-up of the committee's selection: this rank's share rows' flags become the
        leader's block mask (rows outside it are cancelled, or never computed when the MSM was
        deferred) and the aggregation of the kept rows is queued -- on EVERY rank, with or without
        local rows, so the aggregation's collective lines up; its handle lands in box['sa'].
        amap_t: device int32 [U], Krum row -> row of the speculative MSM (-1: none)."""
        sp = spec[1] if spec is not None else None
        pred = self._predict_miners(plan, live) if self.gpu and self.cfg.secure_agg else None

        def on_accept(node):
            with self.timer.phase("verify.queue_agg"):
                if sp is not None:
                    B.set_alive(node, amap_t, sp.alive)
                    sp.launch()   # no-op when the MSM already runs speculatively
                if pred is not None:
                    box["sa"] = self._spec_aggregate(spec, pred, node)
        return on_accept

    def run_round(self) -> RoundResult | None:
        cfg, R, fsm, comm = self.cfg, self.R, self.fsm, self.comm
        t_round = time.perf_counter()
        tm = self.timer
        with tm.phase("roles"):
            head, self._head = self._head or self._open_round(), None
            live, plan = head["live"], head["plan"]
            if plan.done:
                return None
            it = plan.iteration
            workers, local_workers, stake = head["workers"], head["local_workers"], head["stake"]
            fut_noise, fut_roles = head["fut_noise"], head["fut_roles"]
            delta, qdelta, pending_commits = head["delta"], head["qdelta"], head["pending_commits"]
            inboxes, row_of, spec = head["inboxes"], head["row_of"], head["spec"]
            qrow = head["qrow"]
        early = head.get("early")
        krum_pre = head.get("krum_pre")
        kst = None
        with tm.phase("pre_vrf"):
            # host work that does not need the VRF outputs, done while they are computed: the previous
            # round's signature batch (starts once these outputs are known) and Krum's static tables
            work, self._pre_vrf_work = self._pre_vrf_work, []
            for f in work:
                f(fut_noise)
            self._resolve_evals()
            if (self.gpu and krum_pre is not None and not early and cfg.verification and inboxes
                    and cfg.defense == "KRUM"):
                kst = self._krum_static(krum_pre["xrow"] if "xrow" in krum_pre else row_of, krum_pre["U1"], plan,
                                        live, inboxes, spec, head.get("arrivals"))
        with tm.phase("vrf_join"):
            noisers = early["noisers"] if early else self._select_noisers(fut_noise, stake,
                                                                           head.get("vrf_workers", local_workers),
                                                                           head.get("vrf_index"))
        with tm.phase("noise"):
            # with the phase-1 Gram the noised deltas are never materialised (only Krum reads them)
            noised = early["noised"] if early else (None if krum_pre is not None else
                                                    self._noise(delta, noisers, local_workers, it))
        # ---------------------------------------------------------------- verification
        with tm.phase("verify"):
            single = comm.world == 1
            commit_of = _CommitTable()
            g_commit = g_noised = g_delta = g_ts = None
            need_X = cfg.verification and bool(inboxes)

            def _materialize_commits():  # first use comes after the Krum kernels are queued
                if commit_of.table is not None:
                    return
                if single:
                    if local_workers:
                        commit_of.fill(pending_commits.result(), qrow)
                elif head.get("commit_gather") is not None:   # gathered in the head (mr_pre)
                    host, ev = head["commit_gather"]
                    ev.synchronize()
                    commit_of.fill(self.crypto.marshal_rows(host), {w: i for i, w in enumerate(workers)})
                elif workers:   # every worker's commitment: one batched marshal of the gathered rows
                    sel = h2d([self.flat[w] for w in workers], torch.long, self.dev)
                    commit_of.fill(self.crypto.marshal_rows(g_commit.index_select(0, sel)),
                                   {w: i for i, w in enumerate(workers)})
            mr_pre = not single and krum_pre is not None and "xrow" in krum_pre
            if not single and not mr_pre:
                # ONE all_gather carries every rank's commitments (device Jacobian rows), noised
                # deltas (the verifiers' input) and, on the plain path, deltas (the block payload)
                cr = self.crypto
                parts = [torch.zeros((self.maxlocal, cr.point_width), dtype=cr.point_dtype, device=self.dev)]
                if need_X or not cfg.secure_agg:
                    parts.append(torch.zeros((self.maxlocal, self.d), dtype=torch.float32, device=self.dev))
                if not cfg.secure_agg:
                    parts.append(torch.zeros((self.maxlocal, self.d), dtype=torch.float32, device=self.dev))
                    # + each rank's clock: every rank builds the plain block with the leader's timestamp
                    parts.append(torch.full((self.maxlocal, 1), self._now(it), dtype=torch.int64, device=self.dev))
                if local_workers:
                    lidx = h2d([w - self.lo for w in local_workers], torch.long, self.dev)
                    parts[0].index_copy_(0, lidx, self._local_commit_rows(pending_commits, local_workers, qrow))
                    if len(parts) > 1:
                        parts[1].index_copy_(0, lidx, noised)
                    if len(parts) > 2:
                        parts[2].index_copy_(0, lidx, delta)
                got = comm.all_gather_packed(parts)
                g_commit = got[0].reshape(-1, cr.point_width)
                g_noised = got[1].reshape(-1, self.d) if len(got) > 1 else None
                g_delta = got[2].reshape(-1, self.d) if len(got) > 2 else None
                g_ts = got[3][:, 0, 0] if len(got) > 3 else None
            if cfg.colluders > 0:  # privacy experiment bookkeeping (isCollusionAttack, main.go:1026-1057)
                thr = self.pc.collusion_thresh
                if any(v >= thr for v in plan.verifiers):
                    self.stats["unmasked_updates"] += sum(
                        1 for w in local_workers if all(j >= thr for j in noisers[w]))
            accepted_map: dict = {}
            signatures: dict = {}
            pending_signatures = None
            box = early["box"] if early else {}
            if need_X:
                vs = [v for v in plan.verifiers if v in inboxes]   # live verifiers, plan order
                nv = len(plan.verifiers)
                ni = len(inboxes[vs[0]])
                X, xrow = (noised, row_of) if single else (g_noised, self.flat)
                if krum_pre is not None and "xrow" in krum_pre:
                    X, xrow = None, krum_pre["xrow"]
                if cfg.defense == "KRUM":
                    # Multi-Krum is a pure function of the (gathered) noised deltas, so every rank
                    # evaluates the whole committee itself (identical inputs, deterministic kernels)
                    with tm.phase("verify.defense"):
                        wait = early["krum"] if early else self._launch_krum(
                            X, xrow, plan, live, inboxes, spec, box, pre=krum_pre, noisers=noisers, static=kst,
                            local_workers=krum_pre.get("row_peers", workers) if mr_pre or (
                                krum_pre is not None and "row_peers" in krum_pre) else local_workers)
                        if mr_pre and head.get("commit_gather") is None:
                            # the commitments' all_gather, queued behind Krum and its aggregation
                            cr = self.crypto
                            part = torch.zeros((self.maxlocal, cr.point_width), dtype=cr.point_dtype, device=self.dev)
                            if local_workers:
                                lidx = h2d([w - self.lo for w in local_workers], torch.long, self.dev)
                                part.index_copy_(0, lidx, self._local_commit_rows(pending_commits, local_workers,
                                                                                   qrow))
                            g_commit = comm.all_gather(part).reshape(-1, cr.point_width)
                        with tm.phase("verify.krum_wait"):
                            acc_t, node_t = wait()
                    acc_np = acc_t.numpy().astype(np.uint8)   # [len(vs), ni]
                    acc_row = {v: k for k, v in enumerate(vs)}
                    if box.get("sa") is not None:   # the rows the device aggregation kept
                        node_np = node_t.numpy()
                        kept = {w for w in workers if node_np[xrow[w]]}
                        # a block row outside the (replicated) speculative prefix was never computed:
                        # the device aggregate is then incomplete and the host path tops it up
                        if not kept <= head["spec_cand"]:
                            kept = None
                            self.stats["spec_misses"] = self.stats.get("spec_misses", 0) + 1
                        box["sa"]["accepted"] = kept
                else:
                    # RONI: each verifier judges with its own data, so only its rank can decide; the
                    # accept matrix [nv, ni] travels in one all_gather on several ranks
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
                # the local verifiers sign their accepted commitments on native threads while the GPU
                # computes shares (main.go:1120-1140); joined where first needed (plain blocks carry
                # them, --verify-signatures checks them) or at the end of the round
                # message i = row rows[i] of the commitment table, signed with sks[key_of[i]], nonce id =
                # the worker; (sl_v, sl_j) = its (verifier, inbox slot) in the signature matrix
                # on the secure path nothing in the round reads the signatures (Q5): their batch yields
                # the host threads to the next round's VRF outputs and is joined one round later
                defer_sign = (self.gpu and cfg.early_vrf and cfg.secure_agg and not cfg.verify_signatures
                              and fut_noise is not None)
                lk = [k for k, v in enumerate(vs) if v in self.local]
                local_vs = [vs[k] for k in lk]
                sig_np = np.zeros((nv, ni, 64), np.uint8)
                sign = {"prep": None, "job": None, "sl": None}
                if local_vs:
                    _materialize_commits()
                    table, rowmap = commit_of.table, commit_of.row
                    acc_l, inb_l = acc_b[lk], inbox_arr[lk]
                    vidx = np.asarray([plan.verifiers.index(v) for v in local_vs], np.int64)
                    sks = [self.sk[v] for v in local_vs]
                    nonce_keys = [(v, it) for v in local_vs]

                    def _prep_sign(after_vrf=None, sign=sign):
                        # message i = row rows[i] of the commitment table, signed with sks[key_of[i]], nonce
                        # id = the worker; (sl_v, sl_j) = its (verifier, inbox slot) in the signature matrix
                        sign["prep"] = None
                        kk, jj = np.nonzero(acc_l)            # (local verifier, inbox slot) of each signature
                        if kk.size:
                            ws = inb_l[kk, jj]
                            rmap = np.full(self.N, -1, np.int64)
                            rmap[list(rowmap)] = list(rowmap.values())
                            bases = [_seed_bytes(cfg.seed, f"nonce-{i}", v) for v, i in nonce_keys]
                            sign["sl"] = (vidx[kk], jj)
                            sign["job"] = R.schnorr_sign_rows_async(table, rmap[ws].tolist(), sks, kk.tolist(), bases,
                                                                    ws.tolist(), self._sign_threads(), after_vrf)
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
                        # the signatures travel to the workers (and on to the miners) only where a
                        # consumer reads them: plain blocks carry them, --verify-signatures checks them;
                        # on the secure path each rank keeps the ones its verifiers produced (Q5) -- as
                        # this matrix, with no per-signature objects
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
        # ---------------------------------------------------------------- aggregation + block
        # host work nothing before the block needs: one rank runs it while it waits for the aggregate
        # audit (_finish_secagg); several ranks run it after the block (its signature all_gather
        # must come at the same point on every rank)
        self._idle_work = pending_signatures
        if pending_signatures is not None and defer_sign:
            # joined at the next round's drain point instead of under this round's audit
            # (two rounds later: the batch starts behind the next round's VRF outputs)
            self._idle_work = None
            self._sign_joins.append(pending_signatures)
            while len(self._sign_joins) > 2:
                self._sign_joins.pop(0)()
        if cfg.secure_agg:
            block = self._secure_aggregation(plan, live, approved, delta, qdelta, local_workers, qrow,
                                             commit_of, signatures, spec, box.get("sa") if cfg.verification else None)
        else:
            block = self._plain_aggregation(plan, live, approved, delta, noised, local_workers, commit_of,
                                            signatures, (g_delta, g_noised, g_ts))
        with tm.phase("block"):
            if block is None:
                block = fsm.make_empty_block()
            r = fsm.commit_block(block)
            if r < 0:
                raise RuntimeError("block refused by the ledger")
            if cfg.chain_file and comm.rank == 0:
                R.Blockchain.append_to_file(cfg.chain_file, block)
            W_dev, self._W_next = self._W_next, None
            n_up = block.data.n_deltas
            if W_dev is not None and n_up:   # the recovered model is already on the device (same bits)
                self.W = W_dev
            elif n_up:
                self.W = torch.from_numpy(np.asarray(block.data.global_w, dtype=np.float64)).to(self.dev)
            eval_pending = self.task.evaluate_async(self.W)   # queued ahead of the next round's MSMs
        with tm.phase("next_head"):
            self._head = self._open_round()   # next round's committee + VRF proofs start now
        if self._idle_work is not None:  # every rank, same point: the collective stays aligned
            self._idle_work()
        lazy = cfg.lazy_eval and self.gpu
        with tm.phase("eval"):
            # lazy_eval: the evaluation kernels are queued (above) but their two numbers are read in
            # the next round's VRF wait (or by drain()); the round's result and log lines get them then
            ev = {"test_error": float("nan"), "attack_rate": float("nan")} if lazy else eval_pending()
        with tm.phase("vrf_drain"):
            # the noiser proofs (nothing in the round consumes them once the lottery has joined on
            # the VRF outputs) and the discarded roles proofs (Q7) finish on the native threads;
            # they are joined one round later (drain() joins the last ones), so the round does not
            # wait for them
            self.drain(final=False)
            self._pending_roles = (fut_noise, fut_roles)
        with tm.phase("side_join"):
            self._join_side_work()
        self.stats["total_updates"] += n_up
        res = RoundResult(iteration=it, block_hash=bytes(block.hash), empty=n_up == 0,
                          node_list=self._last_nodes, approved=list(approved), verifiers=list(plan.verifiers),
                          miners=list(plan.miners), test_error=ev["test_error"], attack_rate=ev["attack_rate"],
                          phases=tm.reset(), wall=time.perf_counter() - t_round, inboxes=dict(inboxes),
                          approved_by_krum=sorted(set().union(*accepted_map.values())) if accepted_map else [])
        if lazy:
            self._evals.append((res, eval_pending))
        else:
            self._log_round(res)
        self.rounds_done += 1
        S.rotate_holds()   # cross-stream tensors of two rounds ago are free to go
        if it == cfg.fail_at and comm.rank == cfg.fail_rank:
            # fault injection: this rank's process dies abruptly after committing block `it`
            # (the reference's FAIL_PROB crash / failAndRestartLocal.sh kill); the surviving ranks'
            # next collective fails and an elastic launcher restarts the job from the chain file
            self.log.info("fault injection: rank %d exits after iteration %d", comm.rank, it)
            import os
            import sys

            flush_logs(self.log)
            sys.stderr.flush()
            os._exit(17)
        return res

    # ------------------------------------------------------------------ off-critical-path work
    def _background(self, fn, *inputs):
        """Run `fn` on the background stream behind everything queued so far on the main stream.
        Nothing on the round's critical path reads the result; the main stream joins it
        (stream-ordered, no host wait) at the end of the round.  Without a GPU it runs inline."""
        if not self.gpu:
            return fn()
        main = S.current()
        bg = self.bg_stream
        S.wait(bg, main)
        with S.use(bg):
            out = fn()
            ev = S.record(bg) if self.cfg.join_background else None
        S.hold(*[t for t in inputs if isinstance(t, torch.Tensor)])
        self._side_work.append((ev, out))
        return out

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

    def _spec_aggregate(self, spec, pred, node) -> dict:
        """Queue the secure aggregation of the rows the committee's selection kept -- masked share-value
        sums, the cross-rank combination, exact recovery (main stream), the audit's commitment sums +
        check (side stream), the witness sums (background stream) -- right behind the selection
        kernels, before the host has read the selection.  Every rank queues it at the same point
        (the selection is replicated), so its collective lines up.  The host later adopts it if the
        approvals, miners and parts match (_secure_aggregation).  node: device int32 mask over the
        Krum rows (the leader's block)."""
        contributing, part = pred
        sp = spec[1] if spec is not None else None
        pts = ys = alive = None
        if sp is not None:
            sp.launch()
            pts, ys, alive = sp.pts, sp.ys, sp.alive
            S.current().wait_event(sp.ev)          # the MSM's shares
        agg = self._aggregate(pts, ys, alive, contributing, part, self._now(self.fsm.iteration))
        agg["contributing"], agg["part"], agg["accepted"], agg["node"] = list(contributing), dict(part), None, node
        return agg

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
            hit = (sl[:4], (ycols - 10).tolist(), (wts, A_dev, sl[4]))
            if len(self._agg_idx) < 256:
                self._agg_idx[key] = hit
        return hit

    def _aggregate(self, pts, ys, rowsel, contributing, part, now) -> dict:
        """Secure aggregation of this rank's kept rows, combined over ranks, then exact recovery.

        Every miner sums the shares it received (aggregateSecret, kyber.go:244-287) and the leader
        recovers from the miners' sums (kyber.go:809-857).  Share sums are additive, so each rank sums
        its own workers' share columns for all miners at once and ONE all_gather (the reduce-scatter
        to the miners fused with the leader's gather) hands every rank the totals; every
        rank then recovers the aggregate itself -- exact integer recovery on identical inputs, so all
        ranks build the leader's block bit for bit.  The chunk-commitment sums (identical for every
        miner: same node list) travel in the same buffer for the audit; the witness sums, which no
        consumer reads (the reference's leader never checks them), stay per-rank partials on the
        background stream.

        pts [R, nch, T+1, pw] / ys [R, nch, T] (None: no local rows); rowsel: device int32 mask [R]
        or a host list of row indices.  Returns the handles _finish_secagg consumes."""
        cfg, comm = self.cfg, self.comm
        T, nch, pw, pdt = self.T, self.nchunks, self.crypto.point_width, self.crypto.point_dtype
        audit = cfg.audit_aggregate
        kzg = cfg.kzg_audit != "off"
        (ccols, wcols, ycols_t, xs_t), xs_list, (wts, A_dev, basis_dev) = self._agg_index(contributing, part)
        kzg_in = None   # this rank's (commitment sums, witness sums, share sums) for the KZG audit
        main = S.current() if self.gpu else None
        # ---- this rank's partial sums
        single = comm.world == 1
        ys_part = None   # this rank's share sums (several ranks / host path); one rank fuses them below
        ys_fused = mask_fused = None   # one rank, GPU: the share sums are fused into the recovery kernel
        cs_part = None
        if pts is not None and (not isinstance(rowsel, list) or rowsel):
            flat = pts.view(pts.shape[0], nch * (T + 1), pw)
            if self.gpu:
                rows_t = None if not isinstance(rowsel, list) else h2d(rowsel, torch.int32, self.dev)
                mask = rowsel if rows_t is None else None
                if single:
                    ys_fused = ys
                    if mask is not None:
                        mask_fused = mask
                    else:
                        sel = np.zeros(ys.shape[0], np.int32)
                        sel[np.asarray(rowsel)] = 1
                        mask_fused = h2d(sel, torch.int32, self.dev)
                elif rows_t is None:
                    ys_part = (ys * mask.view(-1, 1, 1)).sum(0)
                else:
                    ys_part = ys.index_select(0, rows_t.long()).sum(0)
                ws_part = None
                if audit or kzg:
                    st = self.side_stream if comm.world == 1 else main
                    if st is not main:
                        S.wait(st, main)
                    with S.use(st):
                        cs_part = B.sum_rows(flat, rows_t, ccols, check=False, row_mask=mask)
                    if st is not main:
                        S.hold(pts, ccols, mask if mask is not None else rows_t)
                # the miners' witness sums: no consumer on the protocol path (background stream); the
                # KZG audit, when on, reads them from there
                ws_part = self._background(lambda: B.sum_rows(flat, rows_t, wcols, check=False, row_mask=mask),
                                           flat, wcols, mask if mask is not None else rows_t)
                if kzg:
                    kzg_in = (cs_part, ws_part, None if single else ys_part.index_select(1, ycols_t.long()))
            else:
                rows_l = list(rowsel)
                ys_part = ys[rows_l].sum(0)
                if audit or kzg:
                    cs_part = self.crypto.sum_rows(flat[rows_l][:, ccols.long()])
                if kzg:
                    kzg_in = (cs_part, self.crypto.sum_rows(flat[rows_l][:, wcols.long()]),
                              ys_part.index_select(1, ycols_t.long()))
        if ys_part is None and ys_fused is None:   # no local rows: nothing to add
            ys_part = torch.zeros((nch, T), dtype=torch.int64, device=self.dev)
        if audit and cs_part is None:   # no local rows: the neutral element (point at infinity)
            cs_part = torch.zeros((nch, pw), dtype=pdt, device=self.dev)
        # ---- combine over ranks: ONE all_gather (share sums, commitment sums, clock)
        clock = None
        if comm.world > 1:
            parts = [ys_part.reshape(1, -1), torch.full((1, 1), now, dtype=torch.int64, device=self.dev)]
            if audit:
                parts.append(cs_part.reshape(1, -1))
            got = comm.all_gather_packed(parts)
            ys_tot = got[0].view(comm.world, nch, T).sum(0)
            clock = got[1].reshape(comm.world)
            if audit:
                cs_all = got[2].view(comm.world, nch, pw)
                cs_tot = B.sum_rows(cs_all.contiguous(), None, None, check=False) if self.gpu else \
                    self.crypto.sum_rows(cs_all)
        else:
            ys_tot = ys_part
            cs_tot = cs_part
        if self.gpu:
            src = ys_fused if ys_fused is not None else ys_tot.reshape(1, nch, T).contiguous()
            W_new, coeffs, status, agg = K.recover_rows(src.contiguous(), mask_fused if ys_fused is not None else None,
                                                        ycols_t, xs_t, wts, A_dev, basis_dev, cfg.poly_size, self.d,
                                                        self.W, 10.0 ** cfg.precision)
        else:
            agg = ys_tot.index_select(1, ycols_t.long()).contiguous()   # [nch, npts]
            W_new, coeffs, status = K.recover(agg, xs_t.cpu(), cfg.poly_size, self.d, self.W, 10.0 ** cfg.precision)
        # the recovered model (and the clocks) are read back right behind the recovery, AHEAD of the
        # audit queued next on the same stream: the block is built while the audit still runs
        readback = self._d2h_async(status, W_new, *((clock,) if clock is not None else ()))
        if self.gpu and cfg.pre_step and getattr(self.task, "stateless_step", False):
            # every rank recovers the same W_new, so each one queues its own local peers' next step (on
            # the Gram stream, behind the recovery but not behind the audit queued next on main)
            self._pre = self._queue_pre_step(W_new, self.fsm.iteration + 1)   # fsm: the round being aggregated
        audit_ok = self._audit(coeffs, cs_tot.reshape(1, nch, pw)) if audit else None
        if kzg_in is not None:
            # each rank audits its own partial aggregate: verifySecret is linear in (C, W, y), so the
            # partial sums of honest shares satisfy it exactly like the total does
            cs_k, ws_k, y_k = kzg_in
            if self.gpu:
                y_k = agg if y_k is None else y_k
                bg = self.vrf_stream
                S.wait(bg, main)
                S.wait(bg, self.side_stream)
                S.wait(bg, self.bg_stream)
                with S.use(bg):
                    self._kzg_queue(cs_k, ws_k, y_k, xs_t, self.fsm.iteration)
                for t in (cs_k, ws_k, y_k, xs_t):
                    t.record_stream(bg)
            else:
                self._kzg_host(cs_k, ws_k, y_k, xs_list, self.fsm.iteration)
        return {"W_new": W_new, "status": status, "agg": agg, "xs": list(xs_list), "audit_ok": audit_ok,
                "clock": clock, "now": now, "readback": readback}

    def _spec_head_launch(self, block) -> None:
        """Launch the next round's speculative share MSM as soon as the block that seeds the next plan is
        built, before its audit is read and it is committed: the plan, inboxes and leader arrival order
        come from fsm.successor(block) (the FSM as it will be after the commit).  The MSM reads the
        pre-step's quantised updates (it waits for the step only, not for the audit).  The next head
        adopts it when the committed block and its plan match (they do unless the audit fails)."""
        cfg, pre = self.cfg, self._pre
        if not (cfg.spec_head and self.gpu and self.comm.world == 1 and cfg.secure_agg and cfg.verification
                and cfg.spec_msm and cfg.spec_group_rows > 0 and cfg.churn == 0 and cfg.churn_kill_per_min == 0
                and not self._partitions and pre is not None and pre["W"] is self._W_next and self.local):
            return
        shadow = self.fsm.successor(block)
        live = [1] * self.N
        plan = shadow.begin_round(live)
        if plan.done:
            return
        workers = list(plan.workers)
        inboxes = {v: list(ib) for v, ib in zip(plan.verifiers, shadow.verifier_inboxes(workers))}
        cand = set(workers) if len(plan.verifiers) // 2 == 0 else set().union(*inboxes.values())
        arrivals = shadow.leader_arrivals()
        lo_rank = {w: i for i, w in enumerate(arrivals)}
        spec_workers = sorted((w for w in workers if w in self.local and w in cand),
                              key=lambda w: lo_rank.get(w, 1 << 30))
        if not spec_workers:
            return
        side = self.side_stream
        side.wait_event(pre["ev"])   # the step only (it ran on the Gram stream), not the audit on main
        # the row list goes up on an otherwise idle stream (not behind the audit on main or the Gram)
        with S.use(self.upload_stream):
            sp = self.crypto.shares_async(pre["qdelta"], [w - self.lo for w in spec_workers], side,
                                          group_rows=cfg.spec_group_rows)
        self._spec_next = {"hash": bytes(block.hash), "it": plan.iteration, "verifiers": list(plan.verifiers),
                           "miners": list(plan.miners), "workers": workers, "inboxes": inboxes, "cand": cand,
                           "arrivals": arrivals, "spec": (spec_workers, sp), "pre": pre}

    def _early_vrf_submit(self, block_hash) -> None:
        """Start the next round's noiser VRF outputs as soon as the block that seeds them is built,
        before its audit is read and it is committed: for every peer whose output the next head can
        need (the local peers; every peer when each rank replicates the committee's Krum).  The next
        head adopts the job when the committed block has this hash (it does unless the audit fails)
        and the keys match (a churn restart draws new ones)."""
        cfg = self.cfg
        # (getRoles draws every peer's noisers whether or not noise is added: main.go:507)
        if not (self.gpu and cfg.early_vrf and cfg.num_noisers > 0):
            return
        peers = list(range(self.N)) if self.comm.world > 1 else list(self.local)
        seeds = [self.vrf_noise_seed[p] for p in peers]
        job = self.R.vrf_prove_batch_async(seeds, bytes(block_hash), max(1, cfg.host_threads - 1), None,
                                           self.vrf_dev is not None)
        self._early_vrf = {"hash": bytes(block_hash), "job": job, "seeds": seeds,
                           "pos": {p: i for i, p in enumerate(peers)}}

    def _local_commit_rows(self, pending_commits, local_workers: list, qrow: dict) -> torch.Tensor:
        """Device commitment rows of the local workers in local_workers order.  The commitments are
        computed per row of qdelta (qrow: one row per local worker, or one per local peer when the
        pre-step computed them for every local peer)."""
        rows = self.crypto.commit_rows_tensor(pending_commits).to(self.dev)
        idx = [qrow[w] for w in local_workers]
        if idx == list(range(rows.shape[0])):
            return rows
        return rows.index_select(0, h2d(idx, torch.long, self.dev))

    def _queue_pre_step(self, W: torch.Tensor, it: int) -> dict:
        """The next round's local step for EVERY local peer (its workers are not known before the next
        block's roles) and their commitments (background stream), queued right behind the recovery
        of W -- the GPU runs them while the host reads W back, builds and commits the block; the next
        head adopts them if that block carries W (same device tensor) and discards them otherwise."""
        # on the Gram stream, right behind the recovery: the audit queued on the main stream runs beside
        # it instead of in front of it; consumers on other streams wait for out["ev"]
        cfg = self.cfg
        main, gs = S.current(), self.gram_stream
        S.wait(gs, main)
        with S.use(gs):
            delta, qdelta = self.task.step(W, it, list(self.local))
            ev = S.record()
            out = {"W": W, "it": it, "delta": delta, "qdelta": qdelta, "ev": ev,
                   "commits": self.crypto.commitments_async(qdelta, self.bg_stream)}
        S.hold(delta, qdelta)
        if (cfg.pre_gram and self.comm.world == 1 and self._noise_krum() and self.local):
            # the noise-aware Krum's d-dimensional phase over EVERY local peer's delta (the workers are
            # not known yet) and this iteration's noise rows, on the same stream right behind the step:
            # done long before the noisers are drawn, and the main stream's evaluation does not wait
            with S.use(gs):
                g = K.gram_stacked_async(delta, self.noise_tbl[:, it % 100, :])
                g["ev"] = S.record()
            g["xrow"] = {p: p - self.lo for p in self.local}
            g["row_peers"] = list(self.local)
            out["gram"] = g
        return out

    def _noise_krum(self) -> bool:
        """The noise-aware committee Krum applies: Gram of [deltas; noise table rows] ahead of the VRF."""
        cfg = self.cfg
        return bool(self.gpu and cfg.secure_agg and cfg.verification and cfg.defense == "KRUM" and cfg.noising
                    and self.sigma > 0 and self.noise_tbl is not None and not cfg.noise_independent
                    and cfg.krum_pregram)

    def _d2h(self, *ts: torch.Tensor) -> list:
        """Several device tensors to host numpy arrays with ONE wait (pinned, stream-ordered copies)."""
        return self._d2h_async(*ts)()

    def _d2h_async(self, *ts: torch.Tensor):
        """Queue the copies now (on the current stream, behind what produced the tensors and ahead of
        anything queued later); the returned callable waits for them and gives numpy arrays."""
        if not self.gpu:
            out = [t.numpy() for t in ts]
            return lambda: out
        hs = []
        for i, t in enumerate(ts):
            # persistent pinned buffers per (slot, shape, dtype): a round reads its copies before the
            # next round queues new ones into the same buffer
            key = (i, tuple(t.shape), t.dtype)
            h = self._pinned.get(key)
            if h is None:
                h = self._pinned[key] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            d2h_into(h, t.contiguous())
            hs.append(h)
        ev = S.record()

        def wait():
            ev.synchronize()
            return [h.numpy() for h in hs]
        return wait

    def _audit(self, coeffs: torch.Tensor, csum: torch.Tensor):
        """Queue the aggregate audit (recovered chunks vs the miners' summed chunk commitments);
        returns a callable giving ok int32 [n_miners, nchunks].  On the GPU the check runs on the
        side stream while the host builds the block (gob + SHA-256)."""
        if not self.gpu:
            ok = self.crypto.check_aggregate(coeffs.cpu(), csum.cpu())
            return lambda: ok
        # the check needs the recovered coefficients (main) and the commitment sums (side stream);
        # by now the share MSM is done, so it runs on the main stream: high priority and every CU
        # (the CU-masked side stream would leave a quarter of the GPU idle on the critical path)
        main = S.current()
        if self.comm.world == 1:
            S.wait(main, self.side_stream)
        ok = self.crypto.check_aggregate(coeffs, csum)
        key = ("audit", tuple(ok.shape), ok.dtype)
        host = self._pinned.get(key)
        if host is None:
            host = self._pinned[key] = torch.empty(ok.shape, dtype=ok.dtype, pin_memory=True)
        d2h_into(host, ok.contiguous())
        ev = S.record(main)

        def result():
            ev.synchronize()
            return host.numpy()
        return result

    def _join_side_work(self) -> None:
        # the background work (the miners' witness sums) has no consumer in the protocol: its inputs
        # and outputs are stream-ordered on the background stream (record_stream), so the main stream
        # does not wait for it -- it overlaps the next round's head instead of the audit
        if self._side_work:
            if self.cfg.join_background:
                main = S.current()
                for ev, _ in self._side_work:
                    main.wait_event(ev)
            self._side_work.clear()

    # ------------------------------------------------------------------ verification defences
    def _verify(self, X: torch.Tensor, inbox: list, it: int, verifier: int, on_accept=None) -> list[bool]:
        cfg = self.cfg
        n = len(inbox)
        if cfg.defense == "RONI":
            # VerifyUpdateRONI (main.go:191-233): accept iff the update raises the verifier's
            # training error by at most 0.02 (always accept in the collusion experiment)
            if cfg.colluders > 0:
                return [True] * n
            base = self.task.train_error(self.W, verifier, it)
            return [self.task.train_error(self.W + X[i].double(), verifier, it) - base <= 0.02 for i in range(n)]
        clip = self.fsm.krum_clip(n)
        if X.device.type == "cuda" and n:
            wait = K.krum_async(X, n - clip, n - clip, on_accept=on_accept)
            with self.timer.phase("verify.krum_wait"):
                acc, _ = wait()
        else:
            acc, _ = K.krum(X, n - clip, n - clip, on_accept=on_accept)
        return [bool(a) for a in acc.cpu().tolist()]

    # ------------------------------------------------------------------ secure aggregation path
    def _secure_aggregation(self, plan, live, approved, delta, qdelta, local_workers, row_of, commit_of,
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
            routes = fsm.route_shares(approved)
            lv = fsm.leader_view(routes)
        if not (lv.leader_online and lv.quorum):
            return None
        node_list, contributing = list(lv.node_list), list(lv.contributing_miners)
        part_of = {m: dict(routes[m])[node_list[0]] for m in contributing}
        if sa is not None and sa.get("accepted") is not None and contributing == sa["contributing"] \
                and part_of == sa["part"] and set(node_list) == sa["accepted"]:
            # the device already aggregated exactly these workers' shares (queued behind the
            # committee's selection, before the host knew the approvals): recovery and audit are in flight
            self.stats["device_aggregations"] = self.stats.get("device_aggregations", 0) + 1
            with tm.phase("recover"):
                return self._finish_secagg(plan, node_list, commit_of, sa)
        # host-decided path (no device selection, RONI, or a prediction mismatch): the leader's block
        # carries lv.node_list only (its first NUM_SAMPLES/2 arrivals), so only those workers' shares
        # are computed; every rank takes this branch together (replicated decisions)
        with tm.phase("shares"):
            local_used = [w for w in node_list if w in self.local]
            pts = ys = None
            rowsel: list = []
            if local_used:
                spec_row = {w: i for i, w in enumerate(spec[0])} if spec is not None else {}
                if spec is not None and all(w in spec_row for w in local_used):
                    sp = spec[1]
                    if sp.ev is None:   # deferred and not launched by a device-side selection
                        used = set(local_used)
                        sp.alive.copy_(h2d([1 if w in used else 0 for w in spec[0]], torch.int32, self.dev))
                    sp.launch()
                    pts, ys = sp.pts, sp.ys
                    S.current().wait_event(sp.ev)
                    rowsel = [spec_row[w] for w in local_used]   # rows of the speculative tensors
                else:
                    sel = h2d([row_of[w] for w in local_used], torch.long, self.dev)
                    pts, ys = self.crypto.shares(qdelta.index_select(0, sel).contiguous())
                    rowsel = list(range(len(local_used)))
        with tm.phase("recover"):
            agg = self._aggregate(pts, ys, rowsel, contributing, part_of, self._now(plan.iteration))
            return self._finish_secagg(plan, node_list, commit_of, agg)

    def _finish_secagg(self, plan, node_list, commit_of, h):
        """Read back the recovered model (and the ranks' clocks), fall back to least squares for
        inconsistent chunks, build the block, then check the aggregate audit (running on the side
        stream meanwhile)."""
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
            block = fsm.make_secagg_block(W_np, node_list, [commit_of[w] for w in node_list], now)
            self._early_vrf_submit(block.hash)
        self._W_next = W_new if st.all() and self.gpu else None
        if self._W_next is not None:
            self._spec_head_launch(block)
        if audit_ok is not None:
            if self._idle_work is not None:   # host-only work (no collective): overlap it with the audit
                self._idle_work()
                self._idle_work = None
            if self.gpu and (self._pre_vrf_work or self._evals):
                # the next round's VRF batch has just started (_early_vrf_submit): this round's deferred
                # signature prep (its batch starts behind those outputs) and the earlier rounds'
                # evaluation read-backs fill the audit wait instead of the next round's VRF wait
                with tm.phase("recover.idle"):
                    ej = self._early_vrf["job"] if self._early_vrf is not None else None
                    work, self._pre_vrf_work = self._pre_vrf_work, []
                    for f in work:
                        f(ej)
                    self._resolve_evals()
            with tm.phase("recover.audit"):
                ok = audit_ok()
            if not ok.all():
                # a miner's sums do not commit to the recovered update: refuse it (the round
                # ends like the reference's missing-quorum path, with an empty block)
                self.stats["audit_failures"] += 1
                self.log.info("aggregate audit failed for %d (miner, chunk) pairs in iteration %d: empty block",
                              int((ok == 0).sum()), plan.iteration)
                return None
        self._last_nodes = node_list
        if self._kzg_pending:
            self._kzg_poll()
        return block

    # ------------------------------------------------------------------ plain aggregation path
    def _plain_aggregation(self, plan, live, approved, delta, noised, local_workers, commit_of, signatures,
                           gathered=(None, None, None)):
        """RegisterUpdate path (-sa=false): the leader miner's block carries every routed update in
        full.  With several ranks the deltas, noised deltas and clocks already travelled in the
        verification all_gather, so every rank builds the leader's block itself (no broadcast)."""
        cfg, R, fsm, comm, tm = self.cfg, self.R, self.fsm, self.comm, self.timer
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
                dsrc, nsrc = delta, noised
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

    # ------------------------------------------------------------------ logging
    def _log_round(self, r: RoundResult) -> None:
        peers = list(self.local) if self.cfg.log_every_peer else [self.lo]
        for p in peers:
            self.log.info("%d:Train Error is %.5f in Iteration %d", p, r.test_error, r.iteration)
            if self.cfg.dataset != "creditcard":
                self.log.info("%d:Attack Rate is %.5f in Iteration %d", p, r.attack_rate, r.iteration)
        self.trace.write({"iteration": r.iteration, "wall_s": r.wall, "empty": r.empty, "nodes": len(r.node_list),
                          "approved": len(r.approved), "test_error": r.test_error, "attack_rate": r.attack_rate,
                          "hash": r.block_hash.hex(), **{f"t_{k}": v for k, v in r.phases.items()}})

    def print_chain(self) -> str:
        return self.fsm.chain.print_chain()
