"""The Biscotti round engine (SPMD over ranks, virtual peers per rank).

One call of :meth:`BiscottiEngine.run_round` performs everything one reference iteration does
across all N peer processes (DistSys/main.go prepareForNextIteration -> messageSender ->
VerifyUpdateKRUM -> RegisterSecret -> startShareDeadlineTimer -> createBlockSecAgg -> sendBlock):

  1. roles        native FSM: stake lottery on the latest block hash; noisers by each worker's
                  own ECVRF output (batched over host threads)
  2. local step   fused gfx950 kernel for all local workers (softmax / logistic regression)
  3. commitments  fixed-base MSM (commit-only pass) for every online worker
  4. noising      counter-based DP noise averaged over each worker's noisers
  5. verification one packed all_gather of commitments + noised deltas; Multi-Krum (f64 MFMA
                  Gram) replicated on every rank; Schnorr signatures of the local verifiers
  6. secure agg.  speculative share/witness MSM (rows Krum rejects are cancelled on the device);
                  one all_to_all of per-miner share bytes; miner-side sums; one packed all_gather
                  of the miners' sums; exact recovery + W update replicated on every rank;
                  device audit of the aggregate against the summed chunk commitments
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
from ..utils import JsonlWriter, PhaseTimer, flush_logs, get_logger, h2d
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


class _SpecShares:
    """Speculative share/witness MSM of some workers' rows on a side stream.  `alive` (int32, one
    flag per row) is cleared for rows the verifiers reject; the MSM skips flagged rows, whether the
    flags were cleared before it started or while it runs.  Consumers wait on `ev`."""

    def __init__(self, eng, qdelta: torch.Tensor, rows: list, stream):
        self.eng, self.qdelta, self.rows, self.stream = eng, qdelta, rows, stream
        self.alive = torch.ones((len(rows),), dtype=torch.int32, device=qdelta.device)
        self.pts = self.ys = self.ev = None

    def launch(self) -> None:
        if self.ev is not None:
            return
        main = S.current()
        S.wait(self.stream, main)              # qdelta (and any flag updates) come from main
        with S.use(self.stream):
            rows_t = h2d(self.rows, torch.int32, self.qdelta.device)
            self.pts, self.ys = self.eng.shares(self.qdelta, rows_t, check_rows=False, alive=self.alive)
            self.ev = torch.cuda.Event()
            self.ev.record(self.stream)
        for t in (self.qdelta, self.alive):
            t.record_stream(self.stream)
        for t in (self.pts, self.ys):              # allocated on the side stream, used on main
            t.record_stream(main)


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
            rows = torch.arange(n, dtype=torch.int32, device=qdelta.device)
            jac = self.eng.commit_rows(qdelta.contiguous(), rows, check_rows=False)
            host = torch.empty(jac.shape, dtype=jac.dtype, pin_memory=True)
            host.copy_(jac, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        qdelta.record_stream(stream)
        if stream is not main:
            jac.record_stream(main)
        return _PendingCommitments(host, ev, jac)

    def commitments(self, qdelta: torch.Tensor) -> np.ndarray:
        return self.commitments_async(qdelta).result()

    def shares(self, qdelta: torch.Tensor):
        rows = torch.arange(qdelta.shape[0], dtype=torch.int32, device=qdelta.device)
        return self.eng.shares(qdelta, rows)

    def shares_async(self, qdelta: torch.Tensor, rows: list, stream, launch: bool = True) -> "_SpecShares":
        """Shares + witnesses of qdelta[rows] on `stream` (the caller's work keeps flowing on its own
        stream).  launch=False prepares the per-row flags only; launch() then starts the MSM after
        everything queued so far on the caller's stream (e.g. Krum's selection), so rows already
        rejected cost nothing."""
        sp = _SpecShares(self.eng, qdelta, rows, stream)
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
            self.bg_cus = 0
            if cfg.bg_stream_complement and cfg.side_stream_skip_every > 0:
                self.bg_stream, self.bg_cus = B.cu_masked_stream(self.dev, -cfg.side_stream_skip_every)
            else:
                self.bg_stream = torch.cuda.Stream(device=self.dev, priority=lo)
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
        self.vrf_noise_seed = {i: _seed_bytes(cfg.seed, "vrf-noise", i) for i in self.local}
        self.vrf_roles_seed = {i: _seed_bytes(cfg.seed, "vrf-roles", i) for i in self.local}
        self.sigma = self.task.noise_sigma(cfg.epsilon)
        # every noiser's 100 pre-sampled noise vectors resident in HBM (314 MB for MNIST x 100 peers)
        self.noise_tbl = None
        if self.gpu and cfg.noising and cfg.noise_table and self.sigma > 0 and self.N * 100 * self.d * 4 <= (8 << 30):
            self.noise_tbl = K.noise_table(self.N, self.d, cfg.seed, self.dev)
        self._side_work: list = []   # (event, tensors) of off-critical-path device work of this round
        self._agg_idx: dict = {}      # (contributing, parts) -> resident aggregation index tensors
        self._W_next = None          # device copy of the model a block under construction carries
        self.stats = {"unmasked_updates": 0, "total_updates": 0, "audit_failures": 0}
        self.rounds_done = 0
        self._head = None
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
    def drain(self) -> None:
        """Join host work that belongs to rounds already returned (the last roles-VRF batch)."""
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
            if getattr(self, "bg_cus", 0):
                B.hip().bsc_stream_destroy(self.bg_stream.cuda_stream)
                self.bg_cus = 0
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
        if self.cfg.churn <= 0:
            return [1] * self.N
        seed = self.fsm.round_seed(7)
        perm = self.R.seeded_permutation(self.N, seed)
        k = int(round(self.cfg.churn * self.N))
        live = [1] * self.N
        for p in perm[:k]:
            live[p] = 0
        return live

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
        live = self._live_mask()
        plan = fsm.begin_round(live)
        head = {"live": live, "plan": plan}
        if plan.done:
            return head
        latest_hash = fsm.chain.latest().hash
        workers = [w for w in plan.workers if live[w]]
        local_workers = [w for w in workers if w in self.local]
        # noisers: each worker's own ECVRF over the latest block hash (vrf.go:54-100).  The host
        # proofs run on native threads while the GPU does the local step and the commitments; the
        # noise phase joins them.
        seeds = [self.vrf_noise_seed[w] for w in local_workers]
        fut_noise = R.vrf_prove_batch_async(seeds, latest_hash, cfg.host_threads) if seeds else None
        fut_roles = None
        if cfg.roles_vrf_proof:  # getVRFRoles proves with the roles key too (result unused, Q7)
            fut_roles = R.vrf_prove_batch_async([self.vrf_roles_seed[p] for p in self.local if live[p]],
                                                latest_hash, cfg.roles_vrf_threads, fut_noise)
        head.update(workers=workers, local_workers=local_workers, stake=dict(fsm.stake), fut_noise=fut_noise,
                    fut_roles=fut_roles)
        # the local step, the commitments and the speculative shares depend only on the new global
        # model too: queue them now, behind nothing but the block that produced it
        tm, it = self.timer, plan.iteration
        with tm.phase("local_step"):
            delta, qdelta = self.task.step(self.W, it, local_workers)
        with tm.phase("commit"):
            # only the first krum_thresh arrivals reach the verifiers (verifier_inbox), so only they
            # can be approved: they secret-share while verification runs (kyber.go:533-646), the MSM
            # on the CU-masked side stream; shares of workers the verifiers reject are never routed.
            # The MSM is the round's longest kernel, so it is launched first.
            inbox = fsm.verifier_inbox(workers) if cfg.verification else []
            row_of = {w: i for i, w in enumerate(local_workers)}
            spec = None
            if self.gpu and cfg.secure_agg and local_workers:
                cand = set(inbox) if cfg.verification else set(workers)
                spec_workers = [w for w in local_workers if w in cand]
                if spec_workers:
                    # with Krum the MSM can also wait for the selection (spec_msm=False): only the kept
                    # rows are then computed, after the verification instead of alongside it
                    defer = not cfg.spec_msm and cfg.verification and cfg.defense == "KRUM"
                    spec = (spec_workers, self.crypto.shares_async(qdelta, [row_of[w] for w in spec_workers],
                                                                   self.side_stream, launch=not defer))
            # full-vector commitments on the background stream: their first consumer is the signing
            # after Krum, so noise + Krum on the main stream do not queue behind them
            pending_commits = self.crypto.commitments_async(qdelta, self.bg_stream if self.gpu else None)
        head.update(delta=delta, qdelta=qdelta, pending_commits=pending_commits, inbox=inbox, row_of=row_of,
                    spec=spec)
        # one rank, Multi-Krum: the noise and Krum kernels (and, behind Krum's selection, the whole
        # device-side aggregation) depend only on this head, so they are queued now as well -- the
        # GPU then runs the round's dependency chain without waiting for the host in between
        if (cfg.early_krum and self.gpu and self.comm.world == 1 and cfg.secure_agg and cfg.verification
                and cfg.defense == "KRUM"
                and inbox and spec is not None and self.noise_tbl is not None and cfg.noising and self.sigma > 0
                and fut_noise is not None and any(live[v] for v in plan.verifiers)):
            with tm.phase("vrf_join"):
                noisers = self._select_noisers(fut_noise, head["stake"], local_workers)
            with tm.phase("noise"):
                _, X = self._noise(delta, noisers, local_workers, inbox, row_of, it)
            with tm.phase("verify.launch"):
                box: dict = {}
                n = len(inbox)
                clip = fsm.krum_clip(n)
                wait = K.krum_async(X, n - clip, n - clip, on_accept=self._on_accept(spec, inbox, plan, live, box))
            head["early"] = {"noisers": noisers, "krum": wait, "box": box}
        return head

    def _select_noisers(self, fut_noise, stake, local_workers) -> dict:
        """Each worker's noisers from its own VRF output (getVRFNoisers, vrf.go:54-100).  Waits for
        the outputs only; the proofs finish on the native threads and are joined at round end."""
        betas = fut_noise.betas() if fut_noise is not None else []
        sel = self.R.select_noisers_batch(stake, betas, local_workers, self.cfg.num_noisers, self.N) if betas else []
        return dict(zip(local_workers, sel))

    def _noise(self, delta, noisers, local_workers, inbox, row_of, it):
        """Noised deltas (requestNoise + NoisedDelta, main.go:1513-1660) -> (noised [n, d] or None,
        X_inbox or None).  On one rank with the secure path the noised deltas only feed Krum, so the
        noise kernel writes the verifiers' inbox directly, in arrival order."""
        cfg = self.cfg
        if not (cfg.noising and self.sigma > 0 and local_workers):
            return delta, None
        ids = [noisers[w] for w in local_workers]
        assert all(0 <= j < self.N for row in ids for j in row), "noiser id out of range"
        nz = h2d(ids, torch.int32, self.dev)
        sc = h2d([[0.0 if j in self.colluders else self.task.noise_scale(self.sigma) for j in noisers[w]]
                  for w in local_workers], torch.float32, self.dev)
        if self.comm.world == 1 and cfg.secure_agg and cfg.verification and inbox and self.noise_tbl is not None:
            rr = [row_of[w] for w in inbox]
            assert max(rr) < delta.shape[0]
            X = K.dp_noise(delta, nz, sc, cfg.seed, it, table=self.noise_tbl, rows=h2d(rr, torch.int32, self.dev))
            return None, X
        return K.dp_noise(delta, nz, sc, cfg.seed, it, table=self.noise_tbl), None

    def _on_accept(self, spec, inbox, plan, live, box):
        """Device-side follow-up of Krum's selection kernel: cancel the rejected speculative rows and
        (one rank) queue the aggregation of the kept rows; its handle lands in box['sa']."""
        srow = {w: i for i, w in enumerate(spec[0])}
        amap = h2d([srow.get(w, -1) for w in inbox], torch.int32, self.dev)
        sp = spec[1]
        pred = self._predict_miners(plan, live) if self.comm.world == 1 and self.cfg.secure_agg else None

        def on_accept(acc):
            with self.timer.phase("verify.queue_agg"):
                B.set_alive(acc, amap, sp.alive)
                sp.launch()   # no-op when the MSM already runs speculatively
                if pred is not None:
                    box["sa"] = self._spec_aggregate(spec, pred)
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
            inbox, row_of, spec = head["inbox"], head["row_of"], head["spec"]
        early = head.get("early")
        with tm.phase("vrf_join"):
            noisers = early["noisers"] if early else self._select_noisers(fut_noise, stake, local_workers)
        with tm.phase("noise"):
            noised, X_fused = (None, None) if early else \
                self._noise(delta, noisers, local_workers, inbox, row_of, it)
        # ---------------------------------------------------------------- verification
        with tm.phase("verify"):
            single = comm.world == 1
            commit_of: dict = {}
            g_commit = g_noised = g_delta = g_ts = None
            need_X = cfg.verification and bool(inbox)

            def _materialize_commits():  # first use comes after the Krum kernels are queued
                if commit_of:
                    return
                if single:
                    if local_workers:
                        cl = pending_commits.result()
                        commit_of.update({w: cl[row_of[w]].tobytes() for w in local_workers})
                elif workers:   # every worker's commitment: one batched marshal of the gathered rows
                    sel = h2d([self.flat[w] for w in workers], torch.long, self.dev)
                    cl = self.crypto.marshal_rows(g_commit.index_select(0, sel))
                    commit_of.update({w: cl[i].tobytes() for i, w in enumerate(workers)})
            if not single:
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
                    parts[0].index_copy_(0, lidx, cr.commit_rows_tensor(pending_commits).to(self.dev))
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
            local_verifiers = [v for v in plan.verifiers if live[v] and v in self.local]
            # Multi-Krum is a pure function of the gathered inbox, so on several ranks EVERY rank
            # evaluates it (identical inputs, deterministic kernel) instead of all_gathering the
            # verifiers' accept masks; RONI depends on each verifier's own data and still gathers
            replicated = not single and cfg.defense == "KRUM"
            judges = [v for v in plan.verifiers if live[v]] if replicated else local_verifiers
            # speculative shares of updates Krum rejects are cancelled on the device as soon as the
            # selection kernel has run (Krum approvals are a superset of the approved set); on one
            # rank the whole aggregation of the kept rows is queued right behind it
            on_accept = None
            box = early["box"] if early else {}
            if not early and need_X and spec is not None and cfg.defense == "KRUM":
                on_accept = self._on_accept(spec, inbox, plan, live, box)
            if need_X:
                nv, ni = len(plan.verifiers), len(inbox)
                if single:
                    X = None if (not judges or early) else X_fused if X_fused is not None else \
                        noised.index_select(0, h2d([row_of[w] for w in inbox], torch.long, self.dev))
                else:
                    X = g_noised.index_select(0, h2d([self.flat[w] for w in inbox], torch.long, self.dev)) \
                        if judges else None
                acc_np = np.zeros((nv, ni), np.uint8)
                sig_np = np.zeros((nv, ni, 64), np.uint8)
                krum_cache = None
                pos = {w: j for j, w in enumerate(inbox)}
                # every verifier's accept list first, then ONE native call signs the local ones' lists
                msgs, key_of, ids, slots, sks, bases = [], [], [], [], [], []
                for v in judges:
                    with tm.phase("verify.defense"):
                        if cfg.defense == "KRUM" and early:   # queued with the round head
                            krum_cache = krum_cache or [bool(a) for a in early["krum"]()[0].tolist()]
                            accept = krum_cache
                        elif cfg.defense == "KRUM":  # identical inputs -> identical Krum result
                            krum_cache = krum_cache or self._verify(X, inbox, it, v, on_accept)
                            accept = krum_cache
                        else:
                            accept = self._verify(X, inbox, it, v)
                    vi = plan.verifiers.index(v)
                    for j, a_ in enumerate(accept):
                        if a_:
                            acc_np[vi, j] = 1
                    if v not in self.local:
                        continue   # the verifier's own rank signs its approvals
                    _materialize_commits()
                    sks.append(self.sk[v])
                    bases.append(_seed_bytes(cfg.seed, f"nonce-{it}", v))
                    for w, a_ in zip(inbox, accept):
                        if a_:
                            msgs.append(commit_of[w])
                            key_of.append(len(sks) - 1)
                            ids.append(w)
                            slots.append((vi, pos[w]))
                if box.get("sa") is not None:   # the rows the device aggregation kept
                    keep = set(spec[0])
                    box["sa"]["accepted"] = {w for w, a_ in zip(inbox, krum_cache or []) if a_ and w in keep}
                # verifier signatures (main.go:1120-1140) sign on native threads while the GPU
                # computes shares; they are joined where first needed (plain blocks carry them,
                # --verify-signatures checks them) or at the end of the round
                sign_job = R.schnorr_sign_multi_async(msgs, sks, key_of, bases, ids, cfg.host_threads) \
                    if msgs else None
                acc_all = acc_np[None] if (single or replicated) else \
                    comm.all_gather(torch.from_numpy(acc_np).to(self.dev)).cpu().numpy()
                acc_row = {v: 0 if (single or replicated) else comm.owner(v, self.N) for v in plan.verifiers}
                for vi, v in enumerate(plan.verifiers):
                    if not live[v]:
                        continue
                    accepted_map[v] = [inbox[j] for j in np.nonzero(acc_all[acc_row[v], vi])[0]]

                def _join_signatures(sign_job=sign_job, slots=slots, sig_np=sig_np, acc_all=acc_all,
                                     acc_row=acc_row, inbox=inbox, live=live, plan=plan):
                    with tm.phase("verify.sign_join"):
                        sigs = sign_job.result() if sign_job is not None else []
                        for (vi, j), sg in zip(slots, sigs):
                            sig_np[vi, j] = np.frombuffer(sg, np.uint8)
                        sig_all = sig_np[None] if single else \
                            comm.all_gather(torch.from_numpy(sig_np).to(self.dev)).cpu().numpy()
                        for vi, v in enumerate(plan.verifiers):
                            if not live[v]:
                                continue
                            o = 0 if single else comm.owner(v, self.N)
                            for j in np.nonzero(acc_all[acc_row[v], vi])[0]:
                                signatures.setdefault(inbox[j], []).append(sig_all[o, vi, j].tobytes())
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
        if cfg.secure_agg:
            block = self._secure_aggregation(plan, live, approved, delta, qdelta, local_workers, row_of,
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
        with tm.phase("eval"):
            ev = eval_pending()
        with tm.phase("vrf_drain"):
            # the noiser proofs (nothing in the round consumes them once the lottery has joined on
            # the VRF outputs) and the discarded roles proofs (Q7) finish on the native threads;
            # they are joined one round later (drain() joins the last ones), so the round does not
            # wait for them
            self.drain()
            self._pending_roles = (fut_noise, fut_roles)
        with tm.phase("side_join"):
            self._join_side_work()
        self.stats["total_updates"] += n_up
        res = RoundResult(iteration=it, block_hash=bytes(block.hash), empty=n_up == 0,
                          node_list=self._last_nodes, approved=list(approved), verifiers=list(plan.verifiers),
                          miners=list(plan.miners), test_error=ev["test_error"], attack_rate=ev["attack_rate"],
                          phases=tm.reset(), wall=time.perf_counter() - t_round)
        self._log_round(res)
        self.rounds_done += 1
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
            ev = torch.cuda.Event()
            ev.record(bg)
        for t in inputs:
            if isinstance(t, torch.Tensor):
                t.record_stream(bg)
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
        return contributing, part

    def _spec_aggregate(self, spec, pred) -> dict:
        """Queue the secure aggregation of every speculative row Krum keeps -- masked share-value
        sums, exact recovery (main stream), the audit's commitment sums + check (side stream), the
        witness sums (background stream) -- right behind the selection kernel, before the host has
        read Krum's result.  The host later adopts it if the approvals, miners and parts match
        (_secure_aggregation), so the GPU never idles while the host approves, routes and signs."""
        contributing, part = pred
        spm, T, nch, nc = self.pc.shares_per_miner, self.T, self.nchunks, len(pred[0])
        sp = spec[1]
        sp.launch()
        pts, ys, ev, alive = sp.pts, sp.ys, sp.ev, sp.alive
        main = S.current()
        main.wait_event(ev)                      # the speculative MSM's shares
        key = (tuple(contributing), tuple(part[m] for m in contributing))
        hit = self._agg_idx.get(key)
        if hit is None:
            # a handful of miner layouts recur (the miners' parts are a permutation of 0..M-1): the
            # index tensors are built and uploaded once per layout and stay resident
            base = np.arange(nch) * (T + 1)
            ycols = np.concatenate([spm * part[m] + np.arange(spm) for m in contributing])
            wc = np.concatenate([(base[:, None] + spm * part[m] + np.arange(spm)[None, :]).reshape(-1)
                                 for m in contributing])
            parts = [np.tile(base + T, nc), wc, ycols, ycols - 10]
            idx = h2d(np.concatenate(parts).astype(np.int32), torch.int32, self.dev)
            offs = np.cumsum([0] + [len(a) for a in parts])
            hit = (idx, [idx[offs[i]:offs[i + 1]] for i in range(4)], (ycols - 10).tolist())
            if len(self._agg_idx) < 256:
                self._agg_idx[key] = hit
        idx, (ccols, wcols, ycols_t, xs_t), xs_list = hit
        flat = pts.view(pts.shape[0], nch * (T + 1), 24)
        csum = None
        if self.cfg.audit_aggregate:
            # the miners' chunk-commitment sums need only the MSM + the flags: they run on the side
            # stream alongside the share sums and the recovery below, not after them
            st = self.side_stream
            S.wait(st, main)
            with S.use(st):
                csum = B.sum_rows(flat, None, ccols, check=False, row_mask=alive).view(nc, nch, 24)
            for t in (pts, idx, alive):
                t.record_stream(st)
        agg = (ys * alive.view(-1, 1, 1)).sum(0).index_select(1, ycols_t)     # [nchunks, npts]
        W_new, coeffs, status = K.recover(agg, xs_t, self.cfg.poly_size, self.d, self.W, 10.0 ** self.cfg.precision)
        audit_ok = self._audit(coeffs, csum) if csum is not None else None
        self._background(lambda: B.sum_rows(flat, None, wcols, check=False, row_mask=alive), flat, idx, alive)
        return {"contributing": list(contributing), "part": dict(part), "accepted": None, "W_new": W_new,
                "status": status, "agg": agg, "xs": list(xs_list), "audit_ok": audit_ok}

    def _d2h(self, *ts: torch.Tensor) -> list:
        """Several device tensors to host numpy arrays with ONE wait (pinned, stream-ordered copies)."""
        if not self.gpu:
            return [t.numpy() for t in ts]
        hs = []
        for t in ts:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            hs.append(h)
        ev = S.record()
        ev.synchronize()
        return [h.numpy() for h in hs]

    def _audit(self, coeffs: torch.Tensor, csum: torch.Tensor):
        """Queue the aggregate audit (recovered chunks vs the miners' summed chunk commitments);
        returns a callable giving ok int32 [n_miners, nchunks].  On the GPU the check runs on the
        side stream while the host builds the block (gob + SHA-256)."""
        if not self.gpu:
            ok = self.crypto.check_aggregate(coeffs.cpu(), csum.cpu())
            return lambda: ok
        main = S.current()
        st = self.side_stream
        S.wait(st, main)
        with S.use(st):
            ok = self.crypto.check_aggregate(coeffs, csum)
            host = torch.empty(ok.shape, dtype=ok.dtype, pin_memory=True)
            host.copy_(ok, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        coeffs.record_stream(st)
        csum.record_stream(st)

        def result():
            ev.synchronize()
            return host.numpy()
        return result

    def _join_side_work(self) -> None:
        if self._side_work:
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
        cfg, R, fsm, comm, tm = self.cfg, self.R, self.fsm, self.comm, self.timer
        self._last_nodes = []
        spm, T, nch = self.pc.shares_per_miner, self.T, self.nchunks
        single = comm.world == 1
        if cfg.verify_signatures and cfg.verification:
            # miners reject shares without >= nv/2 valid verifier signatures (main.go:269-277, Q5)
            need = len(plan.verifiers) // 2
            approved = [w for w in approved
                        if sum(any(R.schnorr_verify(commit_of[w], self.pk[v], sg) for v in plan.verifiers)
                               for sg in signatures.get(w, [])) >= need]
        with tm.phase("shares"):
            routes = fsm.route_shares(approved)
            lv = fsm.leader_view(routes)
            local_approved = [w for w in approved if w in self.local]
            pts = ys = None
            ap_row = {w: i for i, w in enumerate(local_approved)}
            if local_approved and routes:  # workers share as soon as any miner is reachable
                spec_row = {w: i for i, w in enumerate(spec[0])} if spec is not None else {}
                if spec is not None and all(w in spec_row for w in local_approved):
                    spec[1].launch()
                    pts, ys, ev = spec[1].pts, spec[1].ys, spec[1].ev
                    S.current().wait_event(ev)
                    ap_row = {w: spec_row[w] for w in local_approved}   # rows of the speculative tensors
                else:
                    sel = h2d([row_of[w] for w in local_approved], torch.long, self.dev)
                    pts, ys = self.crypto.shares(qdelta.index_select(0, sel).contiguous())
        if not (lv.leader_online and lv.quorum):
            return None
        node_list, contributing = list(lv.node_list), list(lv.contributing_miners)
        part_of = {m: dict(routes[m])[node_list[0]] for m in contributing}
        if sa is not None and sa.get("accepted") is not None and contributing == sa["contributing"] and part_of == sa["part"] \
                and set(node_list) == sa["accepted"]:
            # the device already aggregated exactly these workers' shares (queued behind Krum's
            # selection kernel, before the host knew the approvals): recovery and audit are in flight
            self.stats["device_aggregations"] = self.stats.get("device_aggregations", 0) + 1
            with tm.phase("recover"):
                return self._finish_secagg(plan, node_list, commit_of, sa["W_new"], sa["status"], sa["agg"],
                                           sa["xs"], sa["audit_ok"], self._now(plan.iteration))
        pw, pdt = self.crypto.point_width, self.crypto.point_dtype
        esz = torch.empty((), dtype=pdt).element_size()
        ar = torch.arange(nch, dtype=torch.long, device=self.dev)
        nc = len(contributing)
        audit = cfg.audit_aggregate

        def cols_of(part):  # the miner's witness slots + the chunk-commitment slot
            return list(range(spm * part, spm * part + spm)) + [T]

        with tm.phase("share_exchange"):
            recv: dict = {}  # miner -> (pts [E, nch, spm+1, pw] or None, ys [E, nch, spm], rows or None)
            if single:
                rows = h2d([ap_row[w] for w in node_list], torch.long, self.dev)
                for m in contributing:
                    recv[m] = (None, None, rows)
            else:
                # ONE all_to_all: per (miner, worker) entry the miner's witness + chunk-commitment
                # points, then its share values, as raw bytes.  Every rank derives what it receives
                # from the replicated routing, so no size exchange precedes it.
                per_p, per_y = nch * (spm + 1) * pw, nch * spm
                pbytes = per_p * esz
                ent_bytes = pbytes + per_y * 8
                send = []
                for dst in range(comm.world):
                    ents = [(m, w) for m in contributing if comm.owner(m, self.N) == dst
                            for w in node_list if w in ap_row]
                    if ents:
                        ir = h2d([ap_row[w] for _, w in ents], torch.long, self.dev)
                        ic = h2d([cols_of(part_of[m]) for m, _ in ents], torch.long, self.dev)
                        g = pts[ir[:, None, None], ar[None, :, None], ic[:, None, :]]       # [E, nch, spm+1, pw]
                        gy = ys[ir[:, None, None], ar[None, :, None], ic[:, None, :spm]]  # [E, nch, spm]
                        send.append(torch.cat([g.reshape(len(ents), -1).view(torch.uint8),
                                               gy.reshape(len(ents), -1).view(torch.uint8)], dim=1).reshape(-1))
                    else:
                        send.append(torch.empty((0,), dtype=torch.uint8, device=self.dev))
                src_ents = {src: [(mm, w) for mm in contributing if comm.owner(mm, self.N) == comm.rank
                                  for w in node_list if comm.owner(w, self.N) == src] for src in range(comm.world)}
                rb = comm.all_to_all(send, [len(src_ents[s]) * ent_bytes for s in range(comm.world)])
                for m in contributing:
                    if m not in self.local:
                        continue
                    ps_, ys_ = [], []
                    for src in range(comm.world):
                        for k, (mm, w) in enumerate(src_ents[src]):
                            if mm == m:
                                e = rb[src][k * ent_bytes:(k + 1) * ent_bytes]
                                ps_.append(_bytes_as(e[:pbytes], pdt).view(nch, spm + 1, pw))
                                ys_.append(_bytes_as(e[pbytes:], torch.int64).view(nch, spm))
                    recv[m] = (torch.stack(ps_), torch.stack(ys_), None)
        with tm.phase("miner_aggregate"):
            agg_y = torch.zeros((nc, nch, spm), dtype=torch.int64, device=self.dev)
            # every miner's summed chunk commitments (aggregateSecret, kyber.go:251-253): the audit
            # checks the recovered aggregate against them
            csum = torch.zeros((nc, nch, pw), dtype=pdt, device=self.dev)
            agg_direct = xs_direct = None
            if single and self.gpu and contributing:
                # aggregateSecret for every miner: the rows (contributing workers) are shared.  The
                # chunk-commitment sums feed only the audit (side stream); the 7 witness sums per
                # chunk and miner -- which nothing in a round reads: the reference's leader never
                # checks aggregated witnesses -- run on the background stream, off the critical path.
                # Every index list goes up in ONE upload; the share values go straight into the
                # recovery's [nchunks, points] layout.
                row_list = [ap_row[w] for w in node_list]
                base = np.arange(nch) * (T + 1)
                ycols = np.concatenate([spm * part_of[m] + np.arange(spm) for m in contributing])
                wc = np.concatenate([(base[:, None] + spm * part_of[m] + np.arange(spm)[None, :]).reshape(-1)
                                     for m in contributing])
                assert max(row_list) < pts.shape[0] and wc.max() < nch * (T + 1) and ycols.max() < T
                parts = [np.asarray(row_list), np.tile(base + T, nc), wc, ycols, ycols - 10]
                idx = h2d(np.concatenate(parts).astype(np.int32), torch.int32, self.dev)
                offs = np.cumsum([0] + [len(a) for a in parts])
                rows_i, ccols, wcols, ycols_t, xs_t_ = (idx[offs[i]:offs[i + 1]] for i in range(5))
                flat = pts.view(pts.shape[0], nch * (T + 1), pw)
                if audit:
                    st = self.side_stream
                    S.wait(st, S.current())
                    with S.use(st):
                        csum = B.sum_rows(flat, rows_i, ccols, check=False).view(nc, nch, pw)
                    for t in (pts, idx):   # main-stream tensors read on the side stream
                        t.record_stream(st)
                self._background(lambda: B.sum_rows(flat, rows_i, wcols, check=False), flat, idx)
                agg_direct = ys.index_select(0, rows_i).sum(0).index_select(1, ycols_t)   # [nch, npts]
                xs_direct = ((ycols - 10).tolist(), xs_t_)
            else:
                for ci, m in enumerate(contributing):
                    if m not in self.local:
                        continue
                    p_, y_, rows = recv[m]
                    part = part_of[m]
                    if rows is not None:  # single rank (CPU): aggregate straight out of the share tensors
                        cols = h2d([k * (T + 1) + c for k in range(nch) for c in cols_of(part)], torch.long,
                                   self.dev)
                        flat = pts.view(pts.shape[0], nch * (T + 1), pw)
                        s = self.crypto.sum_rows(flat.index_select(0, rows).index_select(1, cols))
                        csum[ci] = s.view(nch, spm + 1, pw)[:, spm]
                        agg_y[ci] = ys.index_select(0, rows)[:, :, spm * part: spm * part + spm].sum(0)
                    elif self.gpu:
                        flatm = p_.reshape(p_.shape[0], nch * (spm + 1), pw)
                        cc = h2d(np.arange(nch, dtype=np.int32) * (spm + 1) + spm, torch.int32, self.dev)
                        csum[ci] = B.sum_rows(flatm, None, cc, check=False)
                        wc = h2d((np.arange(nch)[:, None] * (spm + 1) + np.arange(spm)[None, :]).reshape(-1)
                                 .astype(np.int32), torch.int32, self.dev)
                        self._background(lambda f=flatm, c=wc: B.sum_rows(f, None, c, check=False), flatm, wc)
                        agg_y[ci] = y_.sum(0)
                    else:
                        s = self.crypto.sum_rows(p_.reshape(p_.shape[0], -1, pw))
                        csum[ci] = s.view(nch, spm + 1, pw)[:, spm]
                        agg_y[ci] = y_.sum(0)
        with tm.phase("recover"):
            now = self._now(plan.iteration)
            if single:
                agg_all, cs_all, ts_all = agg_y[None], csum[None], None
            else:
                # ONE all_gather: every miner's share sums (+ its chunk-commitment sums for the audit)
                # and every rank's clock.  Each rank then recovers the aggregate itself -- exact
                # integer recovery on identical inputs, so every rank builds the leader's block bit
                # for bit -- instead of waiting for a block broadcast.
                parts = [agg_y.reshape(1, -1), torch.full((1, 1), now, dtype=torch.int64, device=self.dev)]
                if audit:
                    parts.append(csum.reshape(1, -1))
                got = comm.all_gather_packed(parts)
                agg_all = got[0].view(comm.world, nc, nch, spm)
                ts_all = got[1]
                cs_all = got[2].view(comm.world, nc, nch, pw) if audit else None
            leader_rank = comm.owner(plan.leader, self.N)
            own = [0 if single else comm.owner(m, self.N) for m in contributing]
            if agg_direct is not None:
                agg, (xs, xs_t) = agg_direct, xs_direct
            else:
                xs = [spm * part_of[m] + s_ - 10 for m in contributing for s_ in range(spm)]
                agg = torch.cat([agg_all[own[ci], ci] for ci in range(nc)], dim=1).contiguous()   # [nchunks, npts]
                xs_t = h2d(xs, torch.int32, self.dev)
            with tm.phase("recover.kernel"):
                W_new, coeffs, status = K.recover(agg, xs_t, cfg.poly_size, self.d, self.W, 10.0 ** cfg.precision)
                audit_ok = None
                if audit:
                    audit_ok = self._audit(coeffs, cs_all[0] if single else
                                           torch.stack([cs_all[own[ci], ci] for ci in range(nc)]))
                if ts_all is not None:
                    now = int(ts_all[leader_rank].reshape(-1)[0])   # the leader's clock stamps the block
            return self._finish_secagg(plan, node_list, commit_of, W_new, status, agg, xs, audit_ok, now)

    def _finish_secagg(self, plan, node_list, commit_of, W_new, status, agg, xs, audit_ok, now):
        """Read back the recovered model, fall back to least squares for inconsistent chunks, build
        the block, then check the aggregate audit (running on the side stream meanwhile)."""
        cfg, R, fsm, tm = self.cfg, self.R, self.fsm, self.timer
        with tm.phase("recover.readback"):
            st, W_np = self._d2h(status, W_new)
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
        self._W_next = W_new if st.all() and self.gpu else None
        if audit_ok is not None:
            if self.comm.world == 1 and self._idle_work is not None:
                self._idle_work()
                self._idle_work = None
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
