"""The Biscotti round engine (SPMD over ranks, virtual peers per rank).

One call of :meth:`BiscottiEngine.run_round` performs everything one reference iteration does
across all N peer processes (DistSys/main.go prepareForNextIteration -> messageSender ->
VerifyUpdateKRUM -> RegisterSecret -> startShareDeadlineTimer -> createBlockSecAgg -> sendBlock):

  1. head         (head.py) roles from the stake lottery on the latest block hash; each rank's
                  workers' noiser VRF outputs (its own peers only); the fused local step; the
                  commitment MSM; the speculative share MSM; the noise-aware Krum Gram
  2. noising      (verify.py) the noiser lottery on the VRF outputs; DP noise from the noisers'
                  pre-sampled vectors (or, noise-aware, their ids and weights only)
  3. verification (verify.py) the committee's Multi-Krum replicated on every rank (one f64-MFMA
                  Gram, every verifier's selection on its own inbox, the >= floor(nv/2) vote and the
                  leader's NUM_SAMPLES/2 arrival cap); the local verifiers' Schnorr signatures
  4. secure agg.  (secagg.py) per-rank partial share sums of the kept rows; ONE all_gather; exact
                  recovery + W update replicated on every rank; device audit of the aggregate
  5. block        every rank builds the leader's block (gob + SHA-256) from identical inputs and
                  the leader's clock; empty blocks on the reference's timeout paths
  6. evaluation   test error / attack rate (logged in the reference's line format)

Collectives per secure round on several ranks (parallel/comm.py): the deltas' all_gather for the
noise-aware Gram (queued with the previous round's recovery), one all_gather of commitments + noiser
ids after the VRF outputs, one all_gather of the share / commitment sums.  Every decision (roles,
inbox, approvals, share routing, leader quorum, block contents) comes from the native
:class:`RoundFSM`, replicated identically on every rank.  Failure injection is in faults.py, the
batched verifySecret audit in kzg_audit.py, the crypto backends in crypto_backends.py.
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
from ..utils import JsonlWriter, PhaseTimer, StampedPhaseTimer, fast_info, flush_logs, get_logger
from ..utils import streams as S
from .config import RunConfig
from .crypto_backends import DeviceCrypto, HostCrypto
from .faults import FaultsMixin
from .head import PlanView, RoundHeadMixin
from .kzg_audit import KzgAuditMixin
from .secagg import SecAggMixin
from .verify import VerifyMixin

SIDE_STREAM_SKIP_EVERY = 4   # the speculative-MSM stream leaves every 4th CU to the critical path
VRF_BATCH_ROUNDS = 16        # device VRF proofs: rounds per prover launch
_LOG_WHERE = "engine.py:428"   # file:line the per-round Train Error / Attack Rate lines name


def _seed_bytes(seed: int, tag: str, i: int) -> bytes:
    return hashlib.sha256(f"{seed}:{tag}:{i}".encode()).digest()


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


class BiscottiEngine(RoundHeadMixin, VerifyMixin, SecAggMixin, KzgAuditMixin, FaultsMixin):
    def __init__(self, cfg: RunConfig, comm: Comm | None = None):
        cfg.validate()
        self.cfg = cfg
        self.comm = comm or Comm()
        self.R = rt()
        self.dev = self.comm.device if cfg.device != "cpu" else torch.device("cpu")
        self.gpu = self.dev.type == "cuda"
        from ..parallel.comm import ranks_per_device

        # several ranks share this GPU (rehearsals on a 1-GPU box; Comm.init counts them)
        self._shared_device = self.gpu and ranks_per_device() > 1
        self.N = cfg.num_nodes
        if self.comm.world > self.N:
            raise ValueError(f"{self.comm.world} ranks for {self.N} peers: every rank must host at least one peer")
        self.pc = cfg.protocol(self.R)
        self.local = self.comm.peer_range(self.N)
        self.lo = self.local.start
        self.maxlocal = self.comm.max_local(self.N)
        # peer -> row in a [world * maxlocal] gathered buffer (the flat layout)
        self.flat = {p: r * self.maxlocal + (p - self.comm.peer_range(self.N, r).start)
                     for r in range(self.comm.world) for p in self.comm.peer_range(self.N, r)}
        tag = f"{cfg.log_dir}/log_{self.comm.rank}_{self.N}.log" if cfg.log_dir else None
        self.log = get_logger("peer", tag)
        self.trace = JsonlWriter(cfg.trace_file if self.comm.rank == 0 else None)
        # phase_sync: synchronise the device at every phase boundary so GPU time lands in its phase
        # (diagnostics); off, phase times are host-side and the device pipeline runs undisturbed
        self.timer = (StampedPhaseTimer if cfg.phase_log else PhaseTimer)(
            sync=(lambda: torch.cuda.synchronize(self.dev)) if self.gpu and cfg.phase_sync else None)
        self.golog = None
        if cfg.phase_log:
            from .golog import GoPhaseLog

            self.golog = GoPhaseLog(self.log, self.lo, self.N, log_dir=cfg.log_dir, world=self.comm.world)
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
            # every rank has read the file before rank 0 rewrites it: genesis, or the verified prefix of a
            # resumed chain (a torn final record left by a crash is dropped here)
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
            self._make_streams()
        self.crypto = DeviceCrypto(key, cfg.poly_size, self.T, self.dev) if self.gpu else \
            HostCrypto(key, cfg.poly_size, self.T, cfg.host_threads)
        self.nchunks = self.crypto.nchunks
        # the aggregation behind the committee's selection and the pre-step are enqueued natively (round.hip),
        # on any number of ranks
        self._native = None
        if self.gpu:
            # wave priority classes (kernels/wave_prio.h): one rank drives its GPU alone; with several ranks the
            # collectives' kernels must not queue behind prio-2 share MSMs
            B.set_wave_priorities(self.comm.world == 1 or cfg.has("wave_prio_multi"))
            B.hip().bsc_set_side_prio(1 if cfg.has("side_prio_low") else 0)
            B.hip().bsc_set_witness_tree(1 if cfg.has("witness_sums_tree") else 0)
            # host waits spin up to 5 ms before sleeping when this rank has its GPU (and a core of the quota) to
            # itself -- one rank, or one rank per GPU; ranks sharing a GPU (rehearsals) spin 200 us
            S.set_spin(5e-3 if not self._shared_device and not cfg.has("short_spin") else 2e-4)
            self._native = B.NativeSecAgg(self.crypto.eng, self.main_stream, self.side_stream, self.bg_stream,
                                          10.0 ** cfg.precision, witness=self.witness_stream)
            if self.comm.world > 1:
                self._native.gather_buffers(self.comm.world)
        if cfg.pkey_file:
            ks = self.R.read_client_keys(cfg.pkey_file)
            self.sk = {i: ks[i][0] for i in range(self.N)}
            self.pk = {i: ks[i][1] for i in range(self.N)}
        else:
            self.sk, self.pk = {}, {}
            for i in range(self.N):
                s, p = self.R.client_key_from_entropy(_seed_bytes(cfg.seed, "client", i))
                self.sk[i], self.pk[i] = s, p
        # every peer's VRF seeds (churn restarts draw new ones; each rank proves its own peers only)
        self.vrf_noise_seed = {i: _seed_bytes(cfg.seed, "vrf-noise", i) for i in range(self.N)}
        self.vrf_roles_seed = {i: _seed_bytes(cfg.seed, "vrf-roles", i) for i in range(self.N)}
        self.sigma = self.task.noise_sigma(cfg.epsilon)
        # every noiser's 100 pre-sampled noise vectors (resident in HBM on the GPU: 314 MB for MNIST x 100)
        self.noise_rows = None
        if cfg.noising and self.sigma > 0 and self.N * 100 * self.d * 4 <= (8 << 30):
            self.noise_rows = K.NoiseRows(self.N, self.d, cfg.seed, self.dev)
        # several ranks with RCCL (or emulating rank 0): the round's collectives run inside the fused native calls on
        # the round's own communicator (NativeSecAgg.comm_init); the next noise-aware Gram's deltas gather and tile
        # pairs go with the aggregation's call when the packed verification row holds the layout (_multi_gram)
        self._multi_gram = False
        native_comm = False
        if self._native is not None and self.comm.world > 1:
            try:
                native_comm = self._native.comm_init(self.comm, cfg.comm_timeout_s)
            except RuntimeError as e:   # (every rank fails alike: the unique id or the library is the problem)
                import warnings

                warnings.warn(f"native round collectives unavailable ({e}): torch's collectives instead",
                              RuntimeWarning)
        self._native_comm = native_comm
        if native_comm:
            vg = self._vgather()
            if vg is not None:
                vg.native = self._native
            self._native.bind_multi(self.maxlocal, self.N, vg)
            self._multi_gram = vg is not None and self._noise_krum()
        self.vrf_dev = None
        if self.gpu and cfg.vrf_device:
            from ..ops.vrf import DeviceVrfProver
            # VRF_BATCH_ROUNDS rounds per launch: a launch (~2.2 ms) occupies its SIMDs' register files (352
            # registers per wave) and slows the MSM waves that share them; per-round launches round-robin over
            # several streams cut the end-of-run drain but cost ~0.07 ms in every round (docs/PERF.md round 3)
            self.vrf_dev = DeviceVrfProver(self.dev, VRF_BATCH_ROUNDS)
        self._agg_idx: dict = {}      # (contributing, parts) -> resident aggregation index tensors
        self._W_next = None          # device copy of the model a block under construction carries
        self._pre = None             # next round's local step + commitments, queued behind the recovery
        self._early_vrf = None       # next round's VRF outputs, started as soon as the block hash exists
        self._pinned: dict = {}      # persistent pinned read-back buffers (_d2h_async)
        self._evals: list = []       # (result, evaluation read-back) of rounds not resolved yet (lazy_eval)
        self._pre_vrf_work: list = []  # host work for the next round's VRF wait (deferred signature prep)
        self._sign_joins: list = []    # deferred signature joins of the last rounds (secure path)
        self._stale_vrf: list = []     # early VRF batches the next head did not adopt (joined by drain)
        self._spec_next = None        # next round's share MSM launched at block build (_spec_head_launch)
        self._idle_work = None
        self._last_nodes: list = []
        self.stats = {"unmasked_updates": 0, "total_updates": 0, "audit_failures": 0, "vrf_outputs": 0,
                      "native_collectives": int(self._native_comm)}
        self._kzg_init(cfg)
        self._churn = {"down": {}, "view": {}, "epoch": {}, "acc": 0.0, "kills": 0, "rejoins": 0,
                       "synced_blocks": 0}
        self.stats["churn"] = self._churn
        self.rounds_done = 0
        self._partitions = cfg.partitions()
        self._head = None
        self._front = None            # the next round's front, started at the end of the previous round
        self._host_proofs: list = []  # the run's last round's VRF proofs, proved on the host (joined by drain)
        self._front_planned = False
        self._spec_front = None       # the next round's front launched before the block's commit (_spec_front_launch)
        self._front_remaining = None
        self._warm_up()
        import atexit
        import weakref
        ref = weakref.ref(self)
        atexit.register(lambda: ref() is not None and ref().close())
        # everything allocated so far (torch, datasets, keys, tables) lives for the whole run: move it out of
        # the cyclic collector's generations, so an occasional full collection scans only the rounds'
        # garbage instead of pausing a round for ~0.1 s
        import gc
        gc.collect()
        gc.freeze()

    def _make_streams(self) -> None:
        """The round's HIP streams: the protocol critical path on a high-priority stream; speculative share
        MSMs on a low-priority one masked to 3/4 of the CUs (they fill the GPU while the host waits for
        VRF outputs / Krum, and the critical path keeps the rest)."""
        lo, hi = torch.cuda.Stream.priority_range()
        self.main_stream = torch.cuda.Stream(device=self.dev, priority=hi)
        # (side_all_cus: on every CU -- emulated rank 0 of 2 measured 0.959 vs 0.991 ms on one box and no different on
        # another, docs/PERF.md round 6: the quarter stays with the critical path)
        full = self.cfg.has("side_all_cus")
        self.side_stream, self.side_cus = B.cu_masked_stream(self.dev, 0 if full else SIDE_STREAM_SKIP_EVERY)
        # work the round's end waits for at most (the pre-step's commitments: the block carries them)
        self.bg_stream = torch.cuda.Stream(device=self.dev, priority=lo)
        # work no consumer in the round waits for (the miners' witness sums): on bg they queued the
        # commitments behind them
        self.witness_stream = torch.cuda.Stream(device=self.dev, priority=lo)
        # long device work nothing in a round waits for -- the VRF proofs (kernels/vrf.hip) and the KZG
        # audit sums (kernels/kzg.hip) -- gets a stream of its own
        self.vrf_stream = torch.cuda.Stream(device=self.dev, priority=lo)
        # the pre-step and its Krum Gram (NativeSecAgg pre-step): beside the main stream, so the evaluation and
        # the audit queued there do not wait for it.  High priority: the Gram is on the next round's critical
        # path (Krum waits for it) and is released together with the speculative MSM; at low priority the MSM
        # took the CUs first and the Gram ran 5x slower (200 -> 1000 us; verify.krum_wait 0.32 -> 0.02 ms,
        # driver-style round 1.75 -> 1.55 ms, profiles/r3/gram_priority_ab.txt)
        self.gram_stream = torch.cuda.Stream(device=self.dev, priority=hi)
        # small uploads that must not queue behind any round work (_spec_head_launch)
        self.upload_stream = torch.cuda.Stream(device=self.dev, priority=hi)
        torch.cuda.synchronize(self.dev)   # everything set up so far is visible to the new streams
        torch.cuda.set_stream(self.main_stream)

    def _warm_up(self) -> None:
        """One-off costs that would otherwise land in the first rounds that meet them."""
        cfg = self.cfg
        if self.gpu and cfg.secure_agg and 0 < cfg.num_miners <= 4:
            # every full-quorum miner layout's aggregation indices and exact recovery weights (~8 ms of host
            # work each; the parts are a permutation of 0..M-1); layouts with offline miners are built on use
            import itertools

            M = cfg.num_miners
            for perm in itertools.permutations(range(M)):
                self._agg_index(list(range(M)), {i: perm[i] for i in range(M)})
        if self.gpu and self._noise_krum():
            self._noise_gram_table()   # the 100 periodic noise Grams (~8 MB), built now rather than in round 1
        if self.gpu and cfg.secure_agg:
            # the host-decided path's share MSM (a speculative miss): its torch kernels (row gather, arange)
            # are loaded at their first launch -- tens of ms in the first round that misses otherwise
            q = torch.zeros((2, self.d), dtype=torch.int64, device=self.dev)
            self.crypto.shares(q.index_select(0, torch.arange(2, dtype=torch.long, device=self.dev)).contiguous())
            torch.cuda.synchronize(self.dev)
        if self.vrf_dev is not None:
            # the key material of every peer this rank proves for (secret scalar, nonce prefix, public key:
            # a fixed-base multiplication each) -- the host batches and the device prover share the cache
            self.vrf_dev._rows([self.vrf_noise_seed[p] for p in self.local] +
                               [self.vrf_roles_seed[p] for p in self.local])
            # one proof now: the prover kernel's code object is loaded at its first launch (several ms)
            with S.use(self.vrf_stream):
                self.vrf_dev.prove([self.vrf_noise_seed[self.lo]], [bytes(self.vrf_dev.ALPHA_LEN)])
            # the batched launches' buffers: noiser + roles proofs of every local peer per round
            self.vrf_dev.reserve(self.vrf_stream, self.vrf_dev.batch_rounds * 2 * len(self.local))
            torch.cuda.synchronize(self.dev)
            self.vrf_dev.proofs = 0

    # ------------------------------------------------------------------ lifecycle
    def _resolve_evals(self, wait: bool = True) -> None:
        """Read the queued evaluations of earlier rounds (lazy_eval) into their results and log them, in round
        order.  wait=False: only those whose read-back has landed (the last round's evaluation is queued just
        before the next round starts; waiting for it there held the round's host thread ~0.13 ms)."""
        evs = self._evals
        k = 0
        while k < len(evs) and (wait or getattr(evs[k][1], "ready", lambda: True)()):
            res, f = evs[k]
            ev = f()
            res.test_error, res.attack_rate = ev["test_error"], ev["attack_rate"]
            self._log_round(res)
            k += 1
        del evs[:k]

    def drain(self, final: bool = True) -> None:
        """Join work that belongs to rounds already returned: the last host VRF batch and, when final,
        the outstanding KZG audits, the device VRF proofs still in flight, the deferred signatures
        and the lazy evaluations."""
        if final:
            t0 = time.perf_counter()
            if self._kzg_pending or self._kzg_stage:
                self._kzg_poll(final=True)
            work, self._pre_vrf_work = self._pre_vrf_work, []
            for f in work:   # the run's last signature batch: nothing else needs the host threads now
                f(None, threads=max(1, self.cfg.host_threads))
            t1 = time.perf_counter()
            if self.vrf_dev is not None:
                self.vrf_dev.drain(self.vrf_stream)
                self.stats["vrf_device_proofs"] = self.vrf_dev.proofs
            hp, self._host_proofs = self._host_proofs, []
            for j in hp:
                j.wait()
            t2 = time.perf_counter()
            joins, self._sign_joins = self._sign_joins, []
            for join in joins:
                join()
            t3 = time.perf_counter()
            self._resolve_evals()
            # where a final drain's time goes (bench reports it next to drain_ms)
            self.drain_parts_ms = {"kzg_and_sign_start": 1e3 * (t1 - t0), "device_vrf": 1e3 * (t2 - t1),
                                   "signature_joins": 1e3 * (t3 - t2), "evals": 1e3 * (time.perf_counter() - t3)}
        futs, self._pending_roles = getattr(self, "_pending_roles", None), None
        if final:
            self._stale_vrf = []
            for fut in futs or ():
                if fut is not None:
                    fut.wait()   # the proofs themselves are discarded: no Python objects built
        else:
            # the previous round's batches are joined once they are done (a job dropped while it runs would be
            # waited for by its destructor): waiting here held the round's thread ~25 us
            self._stale_vrf = [j for j in self._stale_vrf if not j.done()]
            self._stale_vrf.extend(f for f in futs or () if f is not None and not f.done())

    def close(self) -> None:
        """Join the pre-opened round's native VRF jobs and drain the device.  Idempotent; also registered
        with atexit so interpreter teardown never races native threads."""
        flush_logs(self.log)
        if self.golog is not None:
            self.golog.flush()
        self.drain()
        heads = []
        sf, self._spec_front = self._spec_front, None
        if sf is not None:
            self._drop_spec_front(sf)
        fr, self._front = self._front, None
        if fr is not None:
            # the next round's front was started (its Krum, the aggregation behind it, the pre-step) but its round
            # never ran: stop the suspended verification generator, join the head's VRF jobs, drop its tensors
            ver = fr.get("verify")
            if hasattr(ver, "close"):
                ver.close()
            heads.append(fr["head"])
        head, self._head = self._head, None
        heads.append(head)
        for head in heads:
            if head:
                for k in ("fut_noise", "fut_roles"):
                    if head.get(k) is not None:
                        head[k].result()
        fr = head = heads = None  # drop the round's tensors while their streams are all still alive
        self._pre = self._spec_next = None
        if self.gpu:
            torch.cuda.synchronize(self.dev)
            S.clear_holds()
        self._agg_idx.clear()   # resident index tensors were used on the side stream destroyed below
        import gc
        gc.unfreeze()   # the engine's own reference cycles become collectable again (see __init__)
        if self.gpu and getattr(self, "side_stream", None) is not None:
            torch.cuda.synchronize(self.dev)
            torch.cuda.set_stream(torch.cuda.default_stream(self.dev))
            # the HBM-resident tables (up to ~90 GB) go now, not whenever the engine is collected
            if isinstance(self.crypto, DeviceCrypto):
                self.crypto.eng.release()
            if self._native is not None:
                self._native.close()
                self._native = None
            self.noise_rows = None
            if getattr(self, "side_cus", 0):
                # every tensor used on the CU-masked stream is gone (round locals, the head above): flush the
                # allocator's stream-use events, then release the stream before interpreter teardown (the
                # HIP runtime must not be left to destroy it at exit)
                gc.collect()
                torch.cuda.synchronize(self.dev)
                torch.cuda.empty_cache()
                B.hip().bsc_stream_destroy(self.side_stream.cuda_stream)
            self.side_stream = None

    EVAL_RING = 6   # evaluation inputs in flight (lazy_eval keeps at most 4 unread: _round_front)

    def _eval_input(self, W: torch.Tensor) -> torch.Tensor:
        """The model an evaluation reads, copied (current stream) into a slot of a ring of its own: the copy is
        ordered after the recovery that wrote W and before any later round's recovery can rewrite W's ring
        slot.  A slot is reused only after its previous evaluation has passed (an event wait that is
        normally long satisfied: the evaluations lag by at most ~4 rounds)."""
        ring = self.__dict__.get("_eval_ring")
        if ring is None or ring[0].shape != W.shape:
            ring = self._eval_ring = [torch.empty_like(W) for _ in range(self.EVAL_RING)]
            self._eval_done = [None] * self.EVAL_RING
            self._eval_k = -1
        self._eval_k = k = (self._eval_k + 1) % self.EVAL_RING
        if self._eval_done[k] is not None:
            S.current().wait_event(self._eval_done[k])
        ring[k].copy_(W)
        return ring[k]

    def _now(self, iteration: int) -> int:
        return iteration + 1 if self.cfg.deterministic_time else int(time.time())

    # ------------------------------------------------------------------ the round
    def run_round(self, last: bool = False, front: bool = True, remaining: int | None = None) -> RoundResult | None:
        """One protocol round.  last: the caller ends its run after this round (its final iteration), so the
        device VRF proofs still batched are launched with this round's instead of at drain() -- the same
        proofs, one prover latency earlier.  The protocol's own last iteration (max_iterations) counts too.
        front=False: the next round's front (_round_front) is not started at the end of this one (bench.py's
        last warm-up round, so a timed window holds exactly its own rounds' fronts).  remaining: the caller's rounds
        left, this one included -- the penultimate round's front sends the queued VRF proofs to the device and
        the last round's front proves its own on the host (_round_front), so the run's end waits for neither."""
        cfg, R, fsm, comm = self.cfg, self.R, self.fsm, self.comm
        t_round = time.perf_counter()
        tm = self.timer
        # the next round's front starts right after this round's block (engine._round_front): the host work of
        # the audit wait that nothing before it needs (signature prep, evaluation read-backs) moves behind it
        self._front_planned = front and not last and self._early_front_ok()
        self._front_remaining = remaining - 1 if remaining else None
        fr, self._front = self._front, None
        if fr is None:
            with tm.phase("roles"):
                head, self._head = self._head or self._open_round(), None
                if head["plan"].done:
                    return None
            fr = self._round_front(head, 1 if last else remaining)
        else:
            self.stats["early_fronts"] = self.stats.get("early_fronts", 0) + 1
            if last and fr["head"].get("vrf_proofs") is not None and fr.get("remaining") != 1:
                self.vrf_dev.flush(self.vrf_stream, urgent=True)   # started before the caller said it is the last
        head, noisers, noised = fr["head"], fr["noisers"], fr["noised"]
        live, plan = head["live"], head["plan"]
        it = plan.iteration
        local_workers, inboxes = head["local_workers"], head["inboxes"]
        with tm.phase("verify"):
            v = self._finish_verification(fr["verify"])
        approved, commit_of, signatures = v["approved"], v["commit_of"], v["signatures"]
        # ---------------------------------------------------------------- aggregation + block
        # host work nothing before the block needs: one rank runs it while it waits for the aggregate audit
        # (_finish_secagg); several ranks run it after the block (its signature all_gather must come at
        # the same point on every rank)
        pending_signatures = v["pending_signatures"]
        self._idle_work = pending_signatures
        if pending_signatures is not None and v["defer_sign"]:
            # joined at the next round's drain point instead of under this round's audit (two rounds later:
            # the batch starts behind the next round's VRF outputs)
            self._idle_work = None
            self._sign_joins.append(pending_signatures)
            if not self._front_planned:   # else after the next round's front (the block build comes first)
                while len(self._sign_joins) > 2:
                    self._sign_joins.pop(0)()
        if cfg.secure_agg:
            block = self._secure_aggregation(plan, live, approved, head["qdelta"], local_workers, head["row_of"],
                                             commit_of, signatures, head["spec"],
                                             v["box"].get("sa") if cfg.verification else None)
        else:
            delta_w = self._worker_rows(head["delta"], head["row_of"], local_workers) if local_workers else None
            block = self._plain_aggregation(plan, live, approved, delta_w, noised, local_workers, commit_of,
                                            signatures, v["gathered"])
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
            if self.gpu:
                # on the witness stream (low priority; nothing in the round waits for either): on the main
                # stream the evaluation sat between the audit and the next round's Krum kernels.  Launched
                # after the next round's front when that runs (ordered on main's position here).  self.W is a
                # slot of the native W ring, which a later round's recovery rewrites while a lagging evaluation
                # may still read it: the evaluation reads a copy of its own (_eval_input), taken where the evaluation is
                # launched -- after the next round's front (the copy is not on the way to its Krum launch; no
                # recovery queued in between can pick this model's ring slot, bsc_ring_pick)
                W_eval_src = self.W
            else:
                eval_pending = self.task.evaluate_async(self.W)
        with tm.phase("next_head"):
            sf, self._spec_front = self._spec_front, None
            if sf is not None:   # the next round's front, launched before this block's commit: adopted or dropped
                self._adopt_spec_front(sf)
            else:
                self._head = self._open_round()   # next round's committee + VRF outputs start now
        if self._front_planned:
            if self._head is not None and not self._head["plan"].done:
                # the next round's front -- noiser lottery, Krum launch and the aggregation queued behind its
                # selection -- before this round's remaining host work: the selection lands earlier and
                # cancels the speculative MSM's rejected rows sooner; the work below fills the next round's waits
                work, self._pre_vrf_work = self._pre_vrf_work, []   # this round's: after the launch
                self._front = self._round_front(self._head, remaining - 1 if remaining else None)
                self._head = None
                self._pre_vrf_work = work + self._pre_vrf_work
            with tm.phase("recover.idle"):
                work, self._pre_vrf_work = self._pre_vrf_work, []
                for f in work:
                    f(None)
                self._resolve_evals(wait=False)   # this round's evaluation was just queued: not waited for
            with tm.phase("verify.sign_join"):
                while len(self._sign_joins) > 2:   # the signature batch of two rounds ago
                    self._sign_joins.pop(0)()
        if self.gpu:
            W_eval = self._eval_input(W_eval_src)
            W_ev = S.record()
            ws = self.witness_stream
            ws.wait_event(W_ev)
            with S.use(ws):
                eval_pending = self.task.evaluate_async(W_eval)
                self._eval_done[self._eval_k] = S.record(ws)   # the copy's slot is free again after this
        if self._idle_work is not None:  # every rank, same point: the collective stays aligned
            self._idle_work()
            self._idle_work = None
        lazy = cfg.lazy_eval and self.gpu
        with tm.phase("eval"):
            # lazy_eval: the evaluation kernels are queued (above) but their two numbers are read in the next
            # round's VRF wait (or by drain()); the round's result and log lines get them then
            ev = {"test_error": float("nan"), "attack_rate": float("nan")} if lazy else eval_pending()
        with tm.phase("vrf_drain"):
            # the discarded roles proofs (Q7) of the host path finish on the native threads; they are
            # joined one round later (drain() joins the last ones), so the round does not wait for them
            self.drain(final=False)
            self._pending_roles = (head["fut_noise"], head["fut_roles"])
        self.stats["total_updates"] += n_up
        if n_up:
            self._note_block_depth(head, self._last_nodes)
        accepted_map = v["accepted_map"]
        if self.golog is not None:
            self.golog.round(it, plan, tm.take_stamps(), noisers, approved, cfg.secure_agg, cfg.noising)
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
        if self.gpu:
            S.rotate_holds()   # cross-stream tensors of two rounds ago are free to go
        self._maybe_fail(it)
        return res

    def _round_front(self, head: dict, remaining: int | None) -> dict:
        """A round up to its verification's device launch: the host work that does not need the VRF outputs,
        the noiser lottery (waits for them), the noise and the verification up to the committee's launch
        (_verification_steps; the Multi-Krum path stops there, the rest runs through).  run_round finishes it
        (_finish_verification) -- in the same call, or one round later when the previous round started it."""
        cfg, tm = self.cfg, self.timer
        live, plan = head["live"], head["plan"]
        it = plan.iteration
        local_workers, inboxes = head["local_workers"], head["inboxes"]
        krum_pre = head.get("krum_pre")
        kst = None
        with tm.phase("pre_vrf"):
            # host work that does not need the VRF outputs, done while they are computed: the previous round's
            # signature batch (starts once these outputs are known) and Krum's static tables
            work, self._pre_vrf_work = self._pre_vrf_work, []
            for f in work:
                f(head["fut_noise"])
            if krum_pre is not None and cfg.verification and inboxes and cfg.defense == "KRUM":
                kst = head.get("kst") or self._krum_static(krum_pre["xrow"], krum_pre["U1"], plan, live, inboxes, head["spec"],
                                        head.get("arrivals"))
        with tm.phase("vrf_join"):
            noisers = self._select_noisers(head["fut_noise"], head["stake"], local_workers, head.get("vrf_index"),
                                           after=head.get("after_block"))
        with tm.phase("noise"):
            # with the phase-1 Gram the noised deltas are never materialised (only Krum reads them)
            noised = None if krum_pre is not None else \
                self._noise(head["delta"], head["row_of"], noisers, local_workers, it)
        with tm.phase("verify"):
            steps = self._verification_steps(head, noisers, noised, kst)
            try:
                next(steps)
                ver = steps
            except StopIteration as done:
                ver = done
        with tm.phase("pre_vrf"):
            # behind the committee's launch (nothing before it needs them): the unread VRF proofs go to the
            # device prover, and the landed evaluation read-backs are taken
            if head.get("vrf_proofs") is not None:
                lw, lv, h = head["vrf_proofs"]
                last = remaining == 1 or it == cfg.max_iterations - 1
                if last:
                    # the run's last round: the rounds queued so far go to the device now, this round's proofs
                    # run on the host threads (AVX-512 IFMA, 8 keys a batch: ~0.3 ms for a round's ~200) -- one
                    # device launch takes ~2.2 ms (a variable-base multiplication per proof), which the run's
                    # end would otherwise wait out
                    self.vrf_dev.flush(self.vrf_stream, urgent=True)
                    seeds = [self.vrf_noise_seed[w] for w in lw]
                    if cfg.roles_vrf_proof:
                        seeds += [self.vrf_roles_seed[p] for p in self.local if lv[p]]
                    if seeds:
                        # (8 threads: the round's own host thread and the runtime keep cores of the quota)
                        self._host_proofs.append(self.R.vrf_proofs_async(seeds, h,
                                                                         max(1, min(8, cfg.host_threads - 2))))
                        self.stats["vrf_host_proofs"] = self.stats.get("vrf_host_proofs", 0) + len(seeds)
                else:
                    self.vrf_dev.submit(self._vrf_key_rows(lw, lv), h, self.vrf_stream)
                    if remaining == 2:   # the penultimate round: its launch (~2.2 ms) ends with the last round
                        self.vrf_dev.flush(self.vrf_stream)
            self._resolve_evals(wait=len(self._evals) > 3)   # a bounded backlog: the host rings hold 4
        return {"head": head, "noisers": noisers, "noised": noised, "verify": ver, "remaining": remaining}

    def _spec_front_launch(self, block) -> None:
        """The speculative front: the next round's front launched from the block just built, before its audit is
        read and it is committed.  Everything the next head would hold is ready then -- the successor plan,
        inboxes, candidates and share MSM (_spec_head_launch), the pre-step's deltas, commitments and Gram, the VRF
        outputs started at the block build (_early_vrf_submit) and the stake the block leaves -- so a head is built
        from them here and _round_front runs on it: the noiser lottery, the Krum launch and the aggregation behind
        the selection are queued before the audit wait, the read-back and the commit instead of after them (the
        selection cancels the speculative MSM's rejected rows sooner).  run_round adopts it when the committed
        block and the FSM's plan match (_adopt_spec_front), else drops it (an audit failure empties the block)."""
        sn, pre, ej = self._spec_next, self._pre, self._early_vrf
        h = bytes(block.hash)
        if not (self._front_planned and self._spec_front_ok() and sn is not None and ej is not None and pre is not None
                and sn["hash"] == h and sn["pre"] is pre and ej["hash"] == h
                and ej["ver"] == getattr(self, "_seed_version", 0) and pre.get("gram") is not None
                and pre["W"] is self._W_next and not sn["plan"].done and sn["inboxes"]):
            return
        plan, lo = sn["plan"], self.lo
        workers = sn["workers"]
        local_workers = [w for w in workers if w in self.local]
        if not local_workers and self.comm.world == 1:
            return   # (several ranks: every rank runs the front, with or without workers -- its collectives line up)
        self._spec_next = self._early_vrf = self._pre = None   # consumed (the pre-step's rows are the head's)
        live = [1] * self.N
        S.current().wait_event(pre["ev"])   # the step ran on the Gram stream
        head = {"live": live, "plan": plan, "workers": workers, "local_workers": local_workers, "stake": None,
                "after_block": block, "fut_noise": ej["job"], "fut_roles": None,
                "vrf_index": [w - lo for w in local_workers], "delta": pre["delta"], "qdelta": pre["qdelta"],
                "pending_commits": pre["commits"], "inboxes": sn["inboxes"], "row_of": {w: w - lo for w in local_workers},
                "row_is_slot": True, "spec": sn["spec"], "spec_cand": sn["cand"], "arrivals": sn["arrivals"],
                "cand_order": sn.get("cand_order"), "krum_pre": pre["gram"], "W": self._W_next,
                "vrf_proofs": (local_workers, live, h)}
        if sn.get("kst") is not None:
            head["kst"] = sn["kst"]
        with self.timer.phase("spec_front"):
            work, self._pre_vrf_work = self._pre_vrf_work, []   # this round's: run in the audit wait, after the launch
            fr = self._round_front(head, self._front_remaining)
            self._pre_vrf_work = work + self._pre_vrf_work
        self._spec_front = {"front": fr, "hash": h}

    def _adopt_spec_front(self, sf: dict) -> None:
        """Begin the round the speculative front was launched for; adopt the front when the committed block is the
        one it was launched from and the plan is the one it used, else drop it and open the round afresh."""
        live = self._live_mask()
        plan = PlanView(self.fsm.begin_round(live))
        sp = sf["front"]["head"]["plan"]
        if (not plan.done and all(live) and bytes(self.fsm.chain.latest_hash()) == sf["hash"]
                and plan.iteration == sp.iteration and plan.leader == sp.leader
                and list(plan.verifiers) == list(sp.verifiers) and list(plan.miners) == list(sp.miners)
                and list(plan.workers) == list(sp.workers)):
            self._front = sf["front"]
            st = self.stats
            for k in ("spec_fronts", "early_vrf", "pre_steps", "spec_head"):
                st[k] = st.get(k, 0) + 1
            return
        self._drop_spec_front(sf)
        self._head = self._open_round(begun=(live, plan))

    def _drop_spec_front(self, sf: dict) -> None:
        """A speculative front whose round will not run from it: its verification generator is stopped and its VRF
        job joined later; its device work (Krum, the aggregation, the pre-step behind it) is left to finish unread
        -- the round that runs instead re-launches its own behind it on the same streams."""
        fr = sf["front"]
        ver = fr.get("verify")
        if hasattr(ver, "close"):
            ver.close()
        job = fr["head"].get("fut_noise")
        if job is not None:
            self._stale_vrf.append(job)
        self._pre = None   # the dropped aggregation's pre-step (from a model that is not the chain's)
        self.stats["spec_front_drops"] = self.stats.get("spec_front_drops", 0) + 1

    def _spec_front_ok(self) -> bool:
        """The speculative front (_spec_front_launch) applies: the native round (several ranks: the multi_spec_front
        ablation, the round's own collectives and the next Gram in its call, and the speculative MSM launched -- on a
        shared GPU only under spec_head_shared), the device VRF prover (no host roles proofs to start with the head), no KZG audit (its
        capture of the aggregate follows the commit), the noise-aware Krum input, and not the no_spec_front
        ablation.  Every input is the same on every rank."""
        cfg = self.cfg
        # several ranks: under multi_spec_front only -- emulated rank 0, same box (docs/PERF.md, round 6): N = 2
        # 1.174 / 1.002 vs 0.954 / 0.979 ms, N = 8 0.895 vs 0.841 without it (the host, not the MSM, is the limit there)
        multi_ok = (self._multi_gram and cfg.has("multi_spec_front")
                    and (not self._shared_device or cfg.has("spec_head_shared")))
        return ((self.comm.world == 1 or multi_ok) and self._native is not None and self.vrf_dev is not None
                and cfg.kzg_audit == "off" and self._noise_krum() and not cfg.has("no_spec_front"))

    def _early_front_ok(self) -> bool:
        """The next round's front runs at the end of this one: one rank per process on a GPU, the pipelined
        noise-aware Multi-Krum path, no churn / partitions / fault injection (whose next round may differ from
        the head built here) and no per-round phase records (trace, phase log, phase sync: their phases would
        move to the previous round).  The no_early_front ablation turns it off; the chain is the same.  With
        several ranks it runs with the native collectives, as the speculative front (_spec_front_ok) or under the
        multi_early_front ablation (at the commit): same-box A/B of the latter
        of emulated rank 0, 3 runs each (docs/PERF.md, round 6), 1.214 / 1.107 / 0.994 ms with it against 1.123 /
        1.024 / 0.877 without at N = 2 / 4 / 8 -- the front's collectives and Krum wait on the device behind the
        previous round's tail instead of the host work they used to overlap."""
        cfg = self.cfg
        # (several ranks: the speculative front launches it before the commit; the front at the commit runs only
        # where that front could not be launched)
        multi = self._multi_gram and (cfg.has("multi_early_front") or self._spec_front_ok())
        return (self.gpu and (self.comm.world == 1 or multi)
                and self._pipelined() and cfg.secure_agg and cfg.verification
                and cfg.defense == "KRUM" and self._noise_krum() and not cfg.has("no_early_front")
                and cfg.churn == 0 and cfg.churn_kill_per_min == 0 and not self._partitions
                and cfg.fail_point()[0] < 0 and not cfg.phase_log and not cfg.phase_sync and not cfg.trace_file)

    # ------------------------------------------------------------------ logging
    def _log_round(self, r: RoundResult) -> None:
        peers = list(self.local) if self.cfg.log_every_peer else [self.lo]
        for p in peers:
            fast_info(self.log, _LOG_WHERE, f"{p}:Train Error is {r.test_error:.5f} in Iteration {r.iteration}")
            if self.cfg.dataset != "creditcard":
                fast_info(self.log, _LOG_WHERE, f"{p}:Attack Rate is {r.attack_rate:.5f} in Iteration {r.iteration}")
        if self.trace.f is None:
            return
        self.trace.write({"iteration": r.iteration, "wall_s": r.wall, "empty": r.empty, "nodes": len(r.node_list),
                          "approved": len(r.approved), "test_error": r.test_error, "attack_rate": r.attack_rate,
                          "hash": r.block_hash.hex(), **{f"t_{k}": v for k, v in r.phases.items()}})

    def print_chain(self) -> str:
        return self.fsm.chain.print_chain()
