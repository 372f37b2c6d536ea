"""Peer <-> rank mapping and the collectives of a Biscotti round.

The reference moves every protocol message as a point-to-point Go net/rpc call (DistSys/main.go,
SURVEY.md section 2.7).  Here peers are *virtual* and packed into contiguous blocks per rank (one
process per GPU); a secure-aggregation round issues two collectives, both one-shot all_gathers that
use every xGMI link at once:

  commitments + noised deltas -> verifiers       all_gather (every rank replicates the committee's
                                                 Multi-Krum on identical inputs: no accept-mask or
                                                 signature traffic on the secure path)
  share sums -> miners -> leader                 all_gather of each rank's per-miner partial share
                                                 sums + chunk-commitment sums + clock (the reduce-
                                                 scatter to the miners fused with the leader's
                                                 gather; every rank recovers the aggregate itself,
                                                 so no block broadcast follows)

The plain (-sa=false) path adds the deltas and clocks to the first gather; RONI verification and
--verify-signatures add one all_gather of accept masks / signatures.  With world size 1 all of these
are local no-ops.  Backend "nccl" is RCCL on ROCm (xGMI); "gloo" runs the same code on CPU for tests
and the plumbing configuration.
"""
from __future__ import annotations

import os
import time
from collections import deque
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

_RANKS_PER_DEVICE = 1   # ranks sharing this process's GPU (Comm.init); 1 with one rank per GPU


def ranks_per_device() -> int:
    """How many ranks share this process's GPU: the HBM table budget is split between them
    (ops/bn256.choose_b0) and the speculative head stays off by default (head.py)."""
    return _RANKS_PER_DEVICE


@dataclass
class Comm:
    world: int = 1
    rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    # (collective, host seconds inside the call) of every collective since the last take_calls(): with RCCL the
    # call returns once the kernel is queued, so a long one means the host thread itself was held (a CFS quota
    # throttle, the GIL, a full queue); with gloo it is the whole exchange
    calls: deque = field(default_factory=lambda: deque(maxlen=16384))

    # ------------------------------------------------------------------ setup
    @staticmethod
    def init(device: str | None = None, backend: str | None = None, timeout_s: float | None = None) -> "Comm":
        """Initialise from torchrun-style env vars (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT).

        `timeout_s` bounds every collective: a rank that dies (the reference's crashed peer) makes
        the survivors' next collective fail within that time instead of hanging, the job exits and
        an elastic launcher (torchrun --max-restarts) restarts it from the persisted chain."""
        from ..utils.threadcpu import mark_new_threads

        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        want_gpu = device != "cpu" and torch.cuda.is_available()
        mark_new_threads("pre-init")
        if want_gpu:
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
            dev = torch.device("cuda", torch.cuda.current_device())
            torch.empty(1, device=dev)   # the HIP runtime's helper threads start here
            mark_new_threads("hip-runtime")
        else:
            dev = torch.device("cpu")
        if world > 1 and not dist.is_initialized():
            if os.environ.get("BISCOTTI_RCCL_SHARED_DEVICE") == "1":
                # rehearsal of the RCCL path with several ranks on one GPU: a distinct host id per rank
                # makes RCCL connect them through its socket transport instead of refusing the
                # duplicate device (test_gpu_multirank.py, scripts/archive/gpu_rccl_bench.sh)
                os.environ.setdefault("NCCL_HOSTID", f"biscotti-rank{rank}")
                os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
                os.environ.setdefault("NCCL_IB_DISABLE", "1")
            be = backend or ("nccl" if dev.type == "cuda" else "gloo")
            local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            if be == "nccl" and torch.cuda.device_count() < local_world and not os.environ.get("NCCL_HOSTID"):
                # (with a distinct NCCL_HOSTID per rank RCCL treats the ranks as separate hosts and
                # connects them over its socket transport: the RCCL path rehearsed on one GPU)
                # several ranks share one device (rehearsals on a 1-GPU box): RCCL refuses
                # duplicate devices, gloo moves the same device tensors through host memory.  Said
                # out loud: a multi-GPU run must never end up on gloo by accident.
                import warnings

                warnings.warn(f"{local_world} local ranks on {torch.cuda.device_count()} visible GPU(s): "
                              "using gloo instead of RCCL", RuntimeWarning)
                be = "gloo"
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {"device_id": dev} if be == "nccl" else {}
            import datetime

            if timeout_s:
                kw["timeout"] = datetime.timedelta(seconds=float(timeout_s))
            attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT")
            if attempt is not None:
                # a restarted job (torchrun --max-restarts) must not read the previous attempt's
                # rendezvous keys: a dead rank's stale address makes the new mesh dial a closed port
                agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
                base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                                     is_master=(rank == 0 and not agent),
                                     timeout=datetime.timedelta(seconds=float(timeout_s or 300)))
                kw["store"] = dist.PrefixStore(f"biscotti/attempt{attempt}", base)
            try:
                dist.init_process_group(be, rank=rank, world_size=world, **kw)
            except TypeError:
                dist.init_process_group(be, rank=rank, world_size=world)
        be = dist.get_backend() if dist.is_initialized() else "none"
        c = Comm(world, rank, dev, be)
        if dev.type == "cuda":
            # how many ranks share this GPU (1 on a node with one rank per GPU; several in rehearsals on a
            # 1-GPU box): the HBM table budget is split between them (ops/bn256.choose_b0)
            global _RANKS_PER_DEVICE
            _RANKS_PER_DEVICE = c.ranks_sharing_device()
        if world > 1:
            c.barrier()   # the backend's communicators (and their proxy / progress threads) exist after this
            mark_new_threads(f"comm-{be}")
        return c

    @staticmethod
    def emulated(world: int, device: str | None = None) -> "Comm":
        """Rank 0 of a `world`-rank job, alone in this process (bench.py --emulate-world): the engine hosts
        rank 0's peers and does exactly rank 0's work -- its local step, commitments and VRF outputs, its
        slice of the Gram tiles, its partial sums, then the replicated recovery, audit and block -- while
        every collective fills the other ranks' slots with rank 0's own contribution (deterministic, the
        same bytes an all_gather would deliver in shape, not in value).  Measures what one rank of an
        N-GPU job costs per round on a one-GPU box; collective latency is not included."""
        from ..utils.threadcpu import mark_new_threads

        mark_new_threads("pre-init")
        if device != "cpu" and torch.cuda.is_available():
            dev = torch.device("cuda", torch.cuda.current_device())
            torch.empty(1, device=dev)
            mark_new_threads("hip-runtime")
        else:
            dev = torch.device("cpu")
        return Comm(int(world), 0, dev, "emulated")

    @property
    def emulating(self) -> bool:
        return self.backend == "emulated"

    def ranks_sharing_device(self) -> int:
        """Ranks whose GPU is this rank's GPU (same host, same device UUID), from one all_gather_object
        at start-up -- HIP_VISIBLE_DEVICES isolation, shared boxes and multi-node jobs all count right."""
        if self.world == 1 or self.device.type != "cuda":
            return 1
        import socket

        props = torch.cuda.get_device_properties(self.device)
        me = (socket.gethostname(), str(getattr(props, "uuid", "")) or f"{props.name}:{self.device.index}",
              os.environ.get("NCCL_HOSTID", ""))
        everyone = [None] * self.world
        dist.all_gather_object(everyone, me)
        # a distinct NCCL_HOSTID per rank (the RCCL-over-sockets rehearsal) still shares the physical GPU
        return sum(1 for o in everyone if o[:2] == me[:2])

    def shutdown(self) -> None:
        if self.world > 1 and not self.emulating and dist.is_initialized():
            dist.destroy_process_group()

    # ------------------------------------------------------------------ ownership
    def peer_range(self, num_peers: int, rank: int | None = None) -> range:
        r = self.rank if rank is None else rank
        return range(r * num_peers // self.world, (r + 1) * num_peers // self.world)

    def owner(self, peer: int, num_peers: int) -> int:
        for r in range(self.world):
            if peer in self.peer_range(num_peers, r):
                return r
        raise ValueError(peer)

    def max_local(self, num_peers: int) -> int:
        return max(len(self.peer_range(num_peers, r)) for r in range(self.world))

    # ------------------------------------------------------------------ collectives
    # ------------------------------------------------------------------ the collectives' stream
    def _comm_stream(self):
        """ONE stream for every RCCL collective of this communicator.  torch issues a synchronous collective on
        the caller's current stream, and the round issues them from two streams (the deltas' gather for the
        split Gram on the Gram stream, the verification and aggregation gathers on the main stream): two
        kernels of one communicator could then run concurrently, or in a different order on each rank --
        undefined for RCCL (ranks' channel FIFOs pair up op by op), seen as 50-330 ms stalls of the 2-rank
        rehearsal (docs/PERF.md).  Collectives run here in issue order, which every rank shares."""
        st = getattr(self, "_cstream", None)
        if st is None and self.backend == "nccl":
            st = self._cstream = torch.cuda.Stream(device=self.device,
                                                   priority=torch.cuda.Stream.priority_range()[1])
        return st

    def _ordered(self, fn):
        """Run fn() (one collective) on the comm stream, ordered after the caller's stream and before its
        later work."""
        cs = self._comm_stream()
        if cs is None:
            return fn()
        from ..utils import streams as S

        cur = S.current()
        S.wait(cs, cur)
        with S.use(cs):
            r = fn()
        S.wait(cur, cs)
        return r

    def take_calls(self) -> list:
        out = list(self.calls)
        self.calls.clear()
        return out

    def barrier(self) -> None:
        if self.world > 1 and not self.emulating:
            if self.backend == "nccl":
                self._ordered(lambda: dist.barrier(device_ids=[self.device.index]))
            else:
                dist.barrier()

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[...] per rank -> [world, ...] (same shape on every rank)."""
        t = t.contiguous()
        if self.world == 1:
            return t.unsqueeze(0)
        flat = t.reshape(-1)
        out = torch.empty((self.world * flat.numel(),), dtype=t.dtype, device=t.device)
        t0 = time.perf_counter()
        if self.emulating:
            out.view(self.world, -1).copy_(flat.unsqueeze(0).expand(self.world, -1))
        else:
            self._ordered(lambda: dist.all_gather_into_tensor(out, flat))
        self.calls.append(("all_gather", time.perf_counter() - t0))
        return out.view(self.world, *t.shape)

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """all_gather of `t` into the caller's (resident) buffer out [world, *t.shape], on the current
        stream: no allocation, and the receiving buffer's address is stable across rounds."""
        if self.world == 1:
            out[0].copy_(t)
            return out
        t0 = time.perf_counter()
        if self.emulating:
            flat = out.view(self.world, -1)
            if t.data_ptr() == flat[0].data_ptr():   # in place: rank 0's row is the source
                flat[1:].copy_(flat[0:1].expand(self.world - 1, -1))
            else:
                flat.copy_(t.reshape(1, -1).expand(self.world, -1))
        else:
            src = t.contiguous().view(-1)
            self._ordered(lambda: dist.all_gather_into_tensor(out.view(-1), src))
        self.calls.append(("all_gather_into", time.perf_counter() - t0))
        return out

    def all_gather_packed(self, parts: list[torch.Tensor]) -> list[torch.Tensor]:
        """ONE all_gather for several tensors of any shapes and dtypes (a round's small messages share a
        launch instead of paying one xGMI latency each): every part's bytes are concatenated into one
        row per rank.  Each rank passes the same shapes; returns [world, *shape] per part, bytes
        reinterpreted back to its dtype."""
        if self.world == 1:
            return [p.unsqueeze(0) for p in parts]
        raw = [p.contiguous().reshape(-1).view(torch.uint8) for p in parts]
        g = self.all_gather(torch.cat(raw))            # [world, total bytes]
        out, o = [], 0
        for p, r in zip(parts, raw):
            nb = r.numel()
            out.append(g[:, o:o + nb].contiguous().view(p.dtype).view(self.world, *p.shape))
            o += nb
        return out

    def broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if self.world > 1 and not self.emulating:
            t0 = time.perf_counter()
            self._ordered(lambda: dist.broadcast(t, src))
            self.calls.append(("broadcast", time.perf_counter() - t0))
        return t
