"""The Biscotti round engine (SPMD over ranks, virtual peers per rank).

One call of :meth:`BiscottiEngine.run_round` performs everything one reference iteration does
across all N peer processes (DistSys/main.go prepareForNextIteration -> messageSender ->
VerifyUpdateKRUM -> RegisterSecret -> startShareDeadlineTimer -> createBlockSecAgg -> sendBlock):

  1. roles        native FSM: stake lottery on the latest block hash; noisers by each worker's
                  own ECVRF output (batched over host threads)
  2. local step   fused gfx950 kernel for all local workers (softmax / logistic regression)
  3. commitments  fixed-base MSM (commit-only pass) for every online worker
  4. noising      counter-based DP noise averaged over each worker's noisers
  5. verification all_gather of noised deltas + commitments; Multi-Krum (f64 MFMA Gram) on each
                  rank that hosts a verifier; Schnorr signatures; all_gather of accept masks
  6. secure agg.  fused share/witness MSM for approved workers; all_to_all of per-miner share
                  slices; miner-side sums; all_gather of miner aggregates to the leader; exact
                  recovery + W update
  7. block        leader builds the block (gob + SHA-256), broadcast, every rank appends and
                  re-verifies the hash; empty blocks on the reference's timeout paths
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
from ..utils import JsonlWriter, PhaseTimer, get_logger, h2d
from .config import RunConfig


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


class _Ready:
    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


class _PendingCommitments:
    def __init__(self, host: torch.Tensor, event):
        self.host, self.event, self.value = host, event, None

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
        main = torch.cuda.current_stream()
        stream = stream or main
        stream.wait_stream(main)
        with torch.cuda.stream(stream):
            rows = torch.arange(n, dtype=torch.int32, device=qdelta.device)
            jac = self.eng.commit_rows(qdelta.contiguous(), rows, check_rows=False)
            host = torch.empty(jac.shape, dtype=jac.dtype, pin_memory=True)
            host.copy_(jac, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        qdelta.record_stream(stream)
        return _PendingCommitments(host, ev)

    def commitments(self, qdelta: torch.Tensor) -> np.ndarray:
        return self.commitments_async(qdelta).result()

    def shares(self, qdelta: torch.Tensor):
        rows = torch.arange(qdelta.shape[0], dtype=torch.int32, device=qdelta.device)
        return self.eng.shares(qdelta, rows)

    def shares_async(self, qdelta: torch.Tensor, rows: list, stream):
        """Shares + witnesses of qdelta[rows] on `stream` (the caller's work keeps flowing on its own
        stream); returns (pts, ys, event).  Consumers wait on the event before touching them."""
        main = torch.cuda.current_stream()
        stream.wait_stream(main)                       # qdelta is produced on the main stream
        with torch.cuda.stream(stream):
            rows_t = h2d(rows, torch.int32, qdelta.device)
            pts, ys = self.eng.shares(qdelta, rows_t, check_rows=False)
            ev = torch.cuda.Event()
            ev.record(stream)
        qdelta.record_stream(stream)
        for t in (pts, ys):                            # allocated on `stream`, consumed on main
            t.record_stream(main)
        return pts, ys, ev

    def sum_rows(self, pts: torch.Tensor) -> torch.Tensor:
        """[R, C, 24] -> [C, 24]"""
        return B.sum_rows(pts.contiguous(), None, None)


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
        if cfg.chain_file and self.comm.rank == 0:
            import os

            if not (cfg.resume and os.path.exists(cfg.chain_file)):
                self.fsm.chain.save(cfg.chain_file)  # genesis (or the resumed prefix) first
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
            self.main_stream = torch.cuda.Stream(device=self.dev, priority=hi)
            # speculative MSMs: a stream masked to 3/4 of the CUs (critical path keeps the rest)
            self.side_stream, self.side_cus = B.cu_masked_stream(self.dev, cfg.side_stream_skip_every) \
                if cfg.side_stream_skip_every > 0 else (torch.cuda.Stream(device=self.dev, priority=lo), 0)
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
        self.stats = {"unmasked_updates": 0, "total_updates": 0}
        self.rounds_done = 0
        self._head = None
        import atexit
        import weakref
        ref = weakref.ref(self)
        atexit.register(lambda: ref() is not None and ref().close())

    # ------------------------------------------------------------------ lifecycle
    def close(self) -> None:
        """Join the pre-opened round's native VRF jobs and drain the device.  Idempotent; also
        registered with atexit so interpreter teardown never races native threads."""
        head, self._head = self._head, None
        if head:
            for k in ("fut_noise", "fut_roles"):
                if head.get(k) is not None:
                    head[k].result()
        head = None  # drop the round's tensors while their streams are all still alive
        if self.gpu and getattr(self, "side_stream", None) is not None:
            torch.cuda.synchronize(self.dev)
            torch.cuda.set_stream(torch.cuda.default_stream(self.dev))
            if getattr(self, "side_cus", 0):
                # every tensor used on the CU-masked stream is gone (round locals, the head above):
                # flush the allocator's stream-use events, then release the stream before
                # interpreter teardown (the HIP runtime must not be left to destroy it at exit)
                import gc
                gc.collect()
                torch.cuda.synchronize(self.dev)
                torch.cuda.empty_cache()
                B.hip().bsc_stream_destroy(self.side_stream.cuda_stream)
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
            pending_commits = self.crypto.commitments_async(qdelta)
            # only the first krum_thresh arrivals reach the verifiers (verifier_inbox), so only they
            # can be approved: they secret-share while verification runs (kyber.go:533-646), the MSM
            # on the CU-masked side stream; shares of workers the verifiers reject are never routed
            inbox = fsm.verifier_inbox(workers) if cfg.verification else []
            row_of = {w: i for i, w in enumerate(local_workers)}
            spec = None
            if self.gpu and cfg.secure_agg and local_workers:
                cand = set(inbox) if cfg.verification else set(workers)
                spec_workers = [w for w in local_workers if w in cand]
                if spec_workers:
                    spec = (spec_workers, self.crypto.shares_async(qdelta, [row_of[w] for w in spec_workers],
                                                                   self.side_stream))
        head.update(delta=delta, qdelta=qdelta, pending_commits=pending_commits, inbox=inbox, row_of=row_of,
                    spec=spec)
        return head

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
        with tm.phase("vrf_join"):
            outs = fut_noise.result() if fut_noise is not None else []
            sel = R.select_noisers_batch(stake, [beta for beta, _ in outs], local_workers, cfg.num_noisers,
                                         self.N) if outs else []
            noisers = dict(zip(local_workers, sel))
        with tm.phase("noise"):
            if cfg.noising and self.sigma > 0 and local_workers:
                nz = h2d([noisers[w] for w in local_workers], torch.int32, self.dev)
                sc = h2d([[0.0 if j in self.colluders else self.task.noise_scale(self.sigma)
                           for j in noisers[w]] for w in local_workers], torch.float32, self.dev)
                noised = K.dp_noise(delta, nz, sc, cfg.seed, it)
            else:
                noised = delta
        # ---------------------------------------------------------------- verification
        with tm.phase("verify"):
            single = comm.world == 1
            commit_of: dict = {}

            def _materialize_commits():  # single rank: first use, after the Krum kernels are queued
                if not commit_of and local_workers:
                    cl = pending_commits.result()
                    commit_of.update({w: cl[row_of[w]].tobytes() for w in local_workers})
            if not single:
                commits_local = pending_commits.result()
                cbuf = torch.zeros((self.maxlocal, 64), dtype=torch.uint8, device=self.dev)
                if local_workers:
                    lidx = h2d([w - self.lo for w in local_workers], torch.long, self.dev)
                    cbuf.index_copy_(0, lidx, torch.from_numpy(commits_local).to(self.dev))
                commits_all = comm.all_gather(cbuf).reshape(-1, 64).cpu().numpy()
                commit_of = {w: commits_all[self.flat[w]].tobytes() for w in workers}
            if cfg.colluders > 0:  # privacy experiment bookkeeping (isCollusionAttack, main.go:1026-1057)
                thr = self.pc.collusion_thresh
                if any(v >= thr for v in plan.verifiers):
                    self.stats["unmasked_updates"] += sum(
                        1 for w in local_workers if all(j >= thr for j in noisers[w]))
            accepted_map: dict = {}
            signatures: dict = {}
            pending_signatures = None
            local_verifiers = [v for v in plan.verifiers if live[v] and v in self.local]
            if cfg.verification and inbox:
                nv, ni = len(plan.verifiers), len(inbox)
                if single:
                    X = noised.index_select(0, h2d([row_of[w] for w in inbox], torch.long, self.dev)) \
                        if local_verifiers else None
                else:
                    nbuf = torch.zeros((self.maxlocal, self.d), dtype=torch.float32, device=self.dev)
                    if local_workers:
                        nbuf.index_copy_(0, lidx, noised)
                    gathered = comm.all_gather(nbuf).reshape(-1, self.d)
                    X = gathered.index_select(0, h2d([self.flat[w] for w in inbox], torch.long, self.dev)) \
                        if local_verifiers else None
                acc_np = np.zeros((nv, ni), np.uint8)
                sig_np = np.zeros((nv, ni, 64), np.uint8)
                krum_cache = None
                pos = {w: j for j, w in enumerate(inbox)}
                # every local verifier's accept list first, then ONE native call signs them all
                msgs, key_of, ids, slots, sks, bases = [], [], [], [], [], []
                for v in local_verifiers:
                    with tm.phase("verify.defense"):
                        if cfg.defense == "KRUM":  # identical inputs -> identical Krum result per rank
                            krum_cache = krum_cache or self._verify(X, inbox, it, v)
                            accept = krum_cache
                        else:
                            accept = self._verify(X, inbox, it, v)
                    vi = plan.verifiers.index(v)
                    _materialize_commits()
                    sks.append(self.sk[v])
                    bases.append(_seed_bytes(cfg.seed, f"nonce-{it}", v))
                    for w, a_ in zip(inbox, accept):
                        if a_:
                            msgs.append(commit_of[w])
                            key_of.append(len(sks) - 1)
                            ids.append(w)
                            slots.append((vi, pos[w]))
                # verifier signatures (main.go:1120-1140) sign on native threads while the GPU
                # computes shares; they are joined where first needed (plain blocks carry them,
                # --verify-signatures checks them) or at the end of the round
                sign_job = R.schnorr_sign_multi_async(msgs, sks, key_of, bases, ids, cfg.host_threads) \
                    if msgs else None
                for vi, j in slots:
                    acc_np[vi, j] = 1
                acc_all = acc_np[None] if single else \
                    comm.all_gather(torch.from_numpy(acc_np).to(self.dev)).cpu().numpy()
                for vi, v in enumerate(plan.verifiers):
                    if not live[v]:
                        continue
                    o = 0 if single else comm.owner(v, self.N)
                    accepted_map[v] = [inbox[j] for j in np.nonzero(acc_all[o, vi])[0]]

                def _join_signatures(sign_job=sign_job, slots=slots, sig_np=sig_np, acc_all=acc_all,
                                     inbox=inbox, live=live, plan=plan):
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
                            for j in np.nonzero(acc_all[o, vi])[0]:
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
        if cfg.secure_agg:
            block = self._secure_aggregation(plan, live, approved, delta, qdelta, local_workers, row_of,
                                             commit_of, signatures, spec)
        else:
            block = self._plain_aggregation(plan, live, approved, delta, noised, local_workers, commit_of,
                                            signatures)
        with tm.phase("block"):
            if block is None:
                block = fsm.make_empty_block()
            r = fsm.commit_block(block)
            if r < 0:
                raise RuntimeError("block refused by the ledger")
            if cfg.chain_file and comm.rank == 0:
                R.Blockchain.append_to_file(cfg.chain_file, block)
            self.W = torch.from_numpy(np.asarray(block.data.global_w, dtype=np.float64)).to(self.dev)
            eval_pending = self.task.evaluate_async(self.W)   # queued ahead of the next round's MSMs
        with tm.phase("next_head"):
            self._head = self._open_round()   # next round's committee + VRF proofs start now
        if pending_signatures is not None:  # every rank, same point: the collective stays aligned
            pending_signatures()
        with tm.phase("eval"):
            ev = eval_pending()
            if fut_roles is not None:
                fut_roles.result()
        self.stats["total_updates"] += len(block.data.deltas)
        res = RoundResult(iteration=it, block_hash=bytes(block.hash), empty=len(block.data.deltas) == 0,
                          node_list=self._last_nodes, approved=list(approved), verifiers=list(plan.verifiers),
                          miners=list(plan.miners), test_error=ev["test_error"], attack_rate=ev["attack_rate"],
                          phases=tm.reset(), wall=time.perf_counter() - t_round)
        self._log_round(res)
        self.rounds_done += 1
        return res

    # ------------------------------------------------------------------ verification defences
    def _verify(self, X: torch.Tensor, inbox: list, it: int, verifier: int) -> list[bool]:
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
        acc, _ = K.krum(X, n - clip, n - clip)
        return [bool(a) for a in acc.cpu().tolist()]

    # ------------------------------------------------------------------ secure aggregation path
    def _secure_aggregation(self, plan, live, approved, delta, qdelta, local_workers, row_of, commit_of,
                            signatures, spec=None):
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
                    pts, ys, ev = spec[1]
                    torch.cuda.current_stream().wait_event(ev)
                    ap_row = {w: spec_row[w] for w in local_approved}   # rows of the speculative tensors
                else:
                    sel = h2d([row_of[w] for w in local_approved], torch.long, self.dev)
                    pts, ys = self.crypto.shares(qdelta.index_select(0, sel).contiguous())
        if not (lv.leader_online and lv.quorum):
            return None
        node_list, contributing = list(lv.node_list), list(lv.contributing_miners)
        part_of = {m: dict(routes[m])[node_list[0]] for m in contributing}
        pw = 24 if self.gpu else 64
        pdt = torch.int32 if self.gpu else torch.uint8
        ar = torch.arange(nch, dtype=torch.long, device=self.dev)

        def cols_of(part):  # the miner's witness slots + the chunk-commitment slot
            return list(range(spm * part, spm * part + spm)) + [T]

        with tm.phase("share_exchange"):
            recv: dict = {}  # miner -> (pts [E, nch, spm+1, pw] or None, ys [E, nch, spm], rows or None)
            if single:
                rows = h2d([ap_row[w] for w in node_list], torch.long, self.dev)
                for m in contributing:
                    recv[m] = (None, None, rows)
            else:
                send_p, send_y = [], []
                for dst in range(comm.world):
                    ents = [(m, w) for m in contributing if comm.owner(m, self.N) == dst
                            for w in node_list if w in ap_row]
                    if ents:
                        ir = h2d([ap_row[w] for _, w in ents], torch.long, self.dev)
                        ic = h2d([cols_of(part_of[m]) for m, _ in ents], torch.long, self.dev)
                        g = pts[ir[:, None, None], ar[None, :, None], ic[:, None, :]]
                        gy = ys[ir[:, None, None], ar[None, :, None], ic[:, None, :spm]]
                        send_p.append(g.reshape(-1))
                        send_y.append(gy.reshape(-1))
                    else:
                        send_p.append(torch.empty((0,), dtype=pdt, device=self.dev))
                        send_y.append(torch.empty((0,), dtype=torch.int64, device=self.dev))
                rp, ry = comm.all_to_all(send_p), comm.all_to_all(send_y)
                for m in contributing:
                    if m not in self.local:
                        continue
                    ps_, ys_ = [], []
                    for src in range(comm.world):
                        src_ents = [(mm, w) for mm in contributing if comm.owner(mm, self.N) == self.comm.rank
                                    for w in node_list if comm.owner(w, self.N) == src]
                        per_p, per_y = nch * (spm + 1) * pw, nch * spm
                        for k, (mm, w) in enumerate(src_ents):
                            if mm == m:
                                ps_.append(rp[src][k * per_p:(k + 1) * per_p].view(nch, spm + 1, pw))
                                ys_.append(ry[src][k * per_y:(k + 1) * per_y].view(nch, spm))
                    recv[m] = (torch.stack(ps_), torch.stack(ys_), None)
        with tm.phase("miner_aggregate"):
            nc = len(contributing)
            agg_y = torch.zeros((nc, nch, spm), dtype=torch.int64, device=self.dev)
            if single and self.gpu and contributing:
                # aggregateSecret for every miner in ONE launch: the rows (contributing workers) are
                # shared, the column list concatenates each miner's witness + commitment slots
                rows = recv[contributing[0]][2]
                base = np.arange(nch)[:, None] * (T + 1)
                cols = np.concatenate([(base + np.asarray(cols_of(part_of[m]))[None, :]).reshape(-1)
                                       for m in contributing])
                flat = pts.view(pts.shape[0], nch * (T + 1), pw)
                _ = B.sum_rows(flat, rows.int(), h2d(cols.astype(np.int32), torch.int32, self.dev))
                ysum = ys.index_select(0, rows).sum(0)   # [nch, T]
                for ci, m in enumerate(contributing):
                    agg_y[ci] = ysum[:, spm * part_of[m]: spm * part_of[m] + spm]
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
                        _ = self.crypto.sum_rows(flat.index_select(0, rows).index_select(1, cols))
                        agg_y[ci] = ys.index_select(0, rows)[:, :, spm * part: spm * part + spm].sum(0)
                    else:
                        _ = self.crypto.sum_rows(p_.reshape(p_.shape[0], -1, pw))
                        agg_y[ci] = y_.sum(0)
        with tm.phase("recover"):
            agg_all = agg_y[None] if single else comm.all_gather(agg_y)   # [world, nc, nch, spm]
            leader_rank = comm.owner(plan.leader, self.N)
            block = block_bytes = None
            if comm.rank == leader_rank:
                cols, xs = [], []
                for ci, m in enumerate(contributing):
                    o = 0 if single else comm.owner(m, self.N)
                    cols.append(agg_all[o, ci])
                    xs += [spm * part_of[m] + s_ - 10 for s_ in range(spm)]
                agg = torch.cat(cols, dim=1).contiguous()      # [nchunks, npts]
                xs_t = h2d(xs, torch.int32, self.dev)
                with tm.phase("recover.kernel"):
                    W_new, coeffs, status = K.recover(agg, xs_t, cfg.poly_size, self.d, self.W, 10.0 ** cfg.precision)
                    st = status.cpu().numpy()
                    W_np = W_new.cpu().numpy()
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
                    block = fsm.make_secagg_block(W_np, node_list, [commit_of[w] for w in node_list],
                                                  self._now(plan.iteration))
                if not single:
                    block_bytes = block.serialize()
            if not single:
                data = comm.broadcast_bytes(block_bytes, leader_rank)
                if comm.rank != leader_rank:
                    block = R.Block.deserialize(data)
                    if block.compute_hash() != block.hash:
                        raise RuntimeError("received block with a bad hash")
            self._last_nodes = node_list
            return block

    # ------------------------------------------------------------------ plain aggregation path
    def _plain_aggregation(self, plan, live, approved, delta, noised, local_workers, commit_of, signatures):
        cfg, R, fsm, comm, tm = self.cfg, self.R, self.fsm, self.comm, self.timer
        self._last_nodes = []
        with tm.phase("aggregate"):
            routes = fsm.route_updates(approved)
            leader = plan.leader
            if not live[leader] or not routes.get(leader):
                return None
            ups = routes[leader]
            idx = {w: i for i, w in enumerate(local_workers)}
            dbuf = self._rows_buffer({w: delta[idx[w]] for w in local_workers}, self.d, torch.float32)
            nbuf = self._rows_buffer({w: noised[idx[w]] for w in local_workers}, self.d, torch.float32)
            dall, nall = comm.all_gather(dbuf), comm.all_gather(nbuf)
            leader_rank = comm.owner(leader, self.N)
            block_bytes = None
            if comm.rank == leader_rank:
                rows = h2d([comm.owner(w, self.N) * self.maxlocal + (w - comm.peer_range(self.N, comm.owner(w, self.N)).start)
                            for w in ups], torch.long, self.dev)
                dv = dall.reshape(-1, self.d).index_select(0, rows).double().cpu().numpy()
                nv = nall.reshape(-1, self.d).index_select(0, rows).double().cpu().numpy()
                blk = fsm.make_plain_block_arrays(self.W.cpu().numpy(), list(ups), dv, nv,
                                                  [commit_of[w] for w in ups],
                                                  [signatures.get(w, []) for w in ups], self._now(plan.iteration))
                if comm.world == 1:
                    self._last_nodes = list(ups)
                    return blk
                block_bytes = blk.serialize()
            data = comm.broadcast_bytes(block_bytes, leader_rank)
            self._last_nodes = list(ups)
            return R.Block.deserialize(data)

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
