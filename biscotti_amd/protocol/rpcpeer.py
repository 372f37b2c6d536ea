"""One Biscotti peer taking part in rounds over Go net/rpc + gob -- the reference's deployment model (one process
per peer, every protocol message a point-to-point RPC, DistSys/main.go).

The SPMD engine (engine.py) replaces those messages by collectives between ranks that host many peers.  This
runtime keeps the reference's message flow for a peer among peers it does not share a job with (reference
peers included), with the same ledger, lottery, crypto and Krum as the engine:

  worker   computeUpdate (honest.go:165-200) -> requestNoiseFromNoisers (main.go:1592-1660, Peer.RequestNoise)
           -> sendUpdateToVerifiers (main.go:1666-1775, Peer.VerifyUpdateKRUM; approved with >= floor(nv/2)
           signatures, main.go:1686) -> sendUpdateSecretsToMiners (main.go:1847-1952, Peer.RegisterSecret: each
           miner its slice of every chunk's Shamir shares + witnesses, generateMinerSecretShares,
           kyber.go:456-512)
  leader   the highest-id miner (getLeaderAddress, main.go:2027-2045): waits for the share threshold
           (startShareDeadlineTimer, main.go:2046-2155), intersects the miners' node lists (getNodesList,
           Peer.GetUpdateList, main.go:2237-2324), gathers their summed parts (getSecretShares, Peer.GetMinerPart,
           main.go:2157-2235), recovers the aggregate exactly (recoverSecret, kyber.go:809-857), builds the block
           (createBlockSecAgg, honest.go:391-440) and floods it (sendBlock, Peer.RegisterBlock, main.go:1403-1444)
  others   verifier / noiser / miner roles are answered by netrpc.PeerService; every peer commits the round's
           block through its own RoundFSM when it arrives (processBlock, main.go:1238-1330)

Host crypto (the CPU backend's native BN256); the transport is netrpc (a fresh connection per call, like rpc.Dial
+ Call under a timeout, main.go:1453-1475).  Empty blocks on the reference's timeout paths (no quorum, no block).
"""
from __future__ import annotations

import threading
import time

import numpy as np
import torch

from ..native import rt
from ..parallel import gob as G
from ..parallel import netrpc as N
from .config import RunConfig
from .head import PlanView


class RpcPeer:
    def __init__(self, cfg: RunConfig, peer_id: int, addresses: list[str], host: str = "127.0.0.1",
                 port: int | None = None, timeout_s: float = 20.0):
        from ..data import dataset_dims
        from ..models import make_task
        from .engine import _seed_bytes

        R = self.R = rt()
        self.cfg, self.id, self.addrs, self.timeout = cfg, int(peer_id), list(addresses), timeout_s
        self.N = cfg.num_nodes
        self.d = dataset_dims(cfg.dataset)[0]
        self.pc = cfg.protocol(R)
        self.fsm = R.RoundFSM(self.pc, self.d)
        self.fsm.addresses = self.addrs
        poisoned = {self.id} if self.fsm.is_poisoner(self.id) else set()
        self.task = make_task(cfg.dataset, range(self.id, self.id + 1), self.N, torch.device("cpu"), cfg.seed,
                              poisoned=poisoned, batch_size=cfg.batch_size, epsilon=cfg.epsilon)
        self.key = R.CommitKey.generate(self.d, 2)   # publicKey.go: s = 2 (every peer derives the same key)
        self.sk, self.pk = R.client_key_from_entropy(_seed_bytes(cfg.seed, "client", self.id))
        self.vrf_seed = _seed_bytes(cfg.seed, "vrf-noise", self.id)
        self.sigma = self.task.noise_sigma(cfg.epsilon)
        scale = self.task.noise_scale(self.sigma)

        def noise(it: int):   # this peer's pre-sampled vector of iteration it, as RequestNoise returns it
            from ..ops import ml as K

            return scale * K.noise_vector(self.id, it, self.d, cfg.seed)
        self.svc = N.PeerService(R, self.fsm.chain, peer_id=self.id, sk=self.sk, noise=noise,
                                 krum_thresh=max(1, self.pc.krum_thresh), krum_timeout_s=timeout_s, live=True,
                                 dim=self.d)
        h, p = self.addrs[self.id].rsplit(":", 1) if port is None else (host, port)
        self.srv = N.RpcServer(self.svc.handlers(), h, int(p), max_conns=N.conns_for(self.N),
                               max_message=N.message_limit(self.d, self.N)).start()
        self.W = np.asarray(self.fsm.chain.latest().data.global_w, np.float64)
        self.log: list = []   # (iteration, event) -- what this peer did in each round

    def close(self) -> None:
        self.srv.close()

    # ------------------------------------------------------------------ one round
    def run_round(self) -> "rt.Block":
        """This peer's part of one round; returns the block it committed (the leader's, or an empty one)."""
        R, fsm = self.R, self.fsm
        plan = PlanView(fsm.begin_round([1] * self.N))
        it = plan.iteration
        roles = set()
        if self.id in plan.verifiers:
            roles.add("verifier")
        if self.id in plan.miners:
            roles.add("miner")
        block = None
        if not roles and self.id in plan.workers:
            self._work(plan)
        if self.id == plan.leader:
            block = self._lead(plan)
        if block is None:
            block = self._await_block(it)
        if fsm.commit_block(block) < 0:
            raise RuntimeError(f"peer {self.id}: block for iteration {it} refused by the ledger")
        if block.data.n_deltas:
            self.W = np.asarray(block.data.global_w, np.float64)
        self.log.append((it, "committed", bytes(block.hash).hex()[:16]))
        return block

    def _addr(self, peer: int) -> str:
        return self.addrs[peer]

    # ------------------------------------------------------------------ worker
    def _work(self, plan) -> None:
        cfg, R, fsm, it = self.cfg, self.R, self.fsm, plan.iteration
        delta, qdelta = self.task.step(torch.from_numpy(self.W), it, [self.id])
        delta = delta[0].double().numpy()
        q = qdelta[0].numpy()
        commitment = bytes(self.key.commit(q, 0))
        noised = delta
        noise = np.zeros_like(delta)
        if cfg.noising and self.sigma > 0 and cfg.num_noisers > 0:
            # this peer's noisers from its own VRF over the latest block hash (getVRFNoisers, vrf.go:54-100)
            beta, _ = R.vrf_prove(self.vrf_seed, bytes(fsm.chain.latest().hash))
            noisers = R.select_noisers(dict(fsm.stake), beta, self.id, cfg.num_noisers, self.N)
            noise = request_noise([self._addr(j) for j in noisers], it, self.d, self.timeout)
            noised = delta + noise
        update = {"SourceID": self.id, "Iteration": it, "Delta": delta.tolist(), "Commitment": commitment,
                  "Noise": noise.tolist(), "NoisedDelta": noised.tolist()}
        sigs, approved = send_update_to_verifiers([self._addr(v) for v in plan.verifiers], update, self.timeout) \
            if cfg.verification else ([], True)
        self.log.append((it, f"verified:{len(sigs)}"))
        if not approved:
            return
        parts = miner_parts(self.key, q, cfg.poly_size, self.pc.total_shares, len(plan.miners))
        send_update_secrets_to_miners([self._addr(m) for m in plan.miners], parts, it, self.id, commitment, sigs,
                                      self.timeout)

    # ------------------------------------------------------------------ leader
    def _lead(self, plan):
        """The leader's block: wait for the share threshold (or the deadline), intersect the miners' node lists,
        gather their summed parts, recover, build; flooded to every other peer."""
        cfg, R, fsm, it = self.cfg, self.R, self.fsm, plan.iteration
        thresh = max(1, fsm.leader_cap_size()) if cfg.verification else max(1, self.pc.krum_thresh // 2)
        deadline = time.monotonic() + self.timeout
        while time.monotonic() < deadline:
            have = len(self.svc.secrets_of(it))
            if have >= thresh:
                break
            time.sleep(0.01)
        miners = [self._addr(m) for m in plan.miners]
        lists = get_update_lists(miners, it, self.timeout)
        node_list = sorted(set.intersection(*map(set, lists))) if lists and all(lists) else []
        node_list = node_list[:thresh]
        block = None
        if node_list and len(lists) == len(miners):
            parts = get_secret_shares(miners, node_list, self.timeout)
            if len(parts) == len(miners):
                W_new = recover_from_parts(R, parts, cfg.poly_size, self.d, self.W, cfg.precision)
                mine = self.svc.secrets_of(it)
                comms = [bytes(mine[w].get("CommitmentUpdate") or bytes(64)) if w in mine else bytes(64)
                         for w in node_list]
                now = it + 1 if cfg.deterministic_time else int(time.time())
                block = fsm.make_secagg_block(W_new, node_list, comms, now)
        if block is None:   # no quorum before the deadline: the reference's empty block
            block = fsm.make_empty_block()
        self.log.append((it, f"lead:{len(node_list)}"))
        N.flood_block([a for i, a in enumerate(self.addrs) if i != self.id], block, self.timeout)
        return block

    def _await_block(self, it: int):
        """The first flooded block of iteration `it` that verified and extends this peer's chain (processBlock,
        main.go:1238-1330); the empty block after the deadline."""
        deadline = time.monotonic() + 3 * self.timeout
        tip = bytes(self.fsm.chain.latest().hash)
        while time.monotonic() < deadline:
            for it_b, kind, b in self.svc.take_blocks():
                if int(it_b) == it and kind == "ahead" and bytes(b.prev_hash) == tip:
                    return b
            time.sleep(0.005)
        return self.fsm.make_empty_block()


# ---------------------------------------------------------------------------- the reference's client calls
def request_noise(addrs: list[str], iteration: int, d: int, timeout: float) -> np.ndarray:
    """requestNoiseFromNoisers (main.go:1592-1660): every noiser's vector of this iteration, averaged over the
    noisers that answered."""
    acc, got = np.zeros(d, np.float64), 0
    for a in addrs:
        try:
            acc += np.asarray(N.call(a, "Peer.RequestNoise", G.INT, int(iteration), timeout), np.float64)
            got += 1
        except (OSError, N.RpcError):
            continue
    return acc / got if got else acc


def send_update_to_verifiers(addrs: list[str], update: dict, timeout: float) -> tuple[list, bool]:
    """sendUpdateToVerifiers (main.go:1666-1775): the update to every verifier at once; approved with at least
    floor(nv/2) signatures (main.go:1686).  A verifier that rejects answers with an error."""
    sigs: list = []
    lock = threading.Lock()

    def one(a):
        try:
            s = N.call(a, "Peer.VerifyUpdateKRUM", G.Update, update, timeout)
        except (OSError, N.RpcError):
            return
        with lock:
            sigs.append(bytes(s))
    ts = [threading.Thread(target=one, args=(a,)) for a in addrs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return sigs, len(sigs) >= len(addrs) // 2


def miner_parts(key, q: np.ndarray, poly: int, total: int, nminers: int) -> list[dict]:
    """generateMinerSecretShares (kyber.go:456-512): the update's chunks, each Shamir-shared at x = i - 10 with
    its witnesses; miner m gets shares [m * spm, (m + 1) * spm) of every chunk.  MinerPartRPC values without the
    envelope fields (send_update_secrets_to_miners adds them)."""
    commitment, chunk_commits, ys, wits = key.make_shares(np.ascontiguousarray(q, np.int64), poly, total)
    nch = len(chunk_commits)
    spm = total // nminers
    out = []
    for m in range(nminers):
        pm = {}
        for k in range(nch):
            sl = range(m * spm, (m + 1) * spm)
            pm[k] = {"Polynomial": [], "Commitment": bytes(chunk_commits[k]),
                     "Secrets": [{"X": s - 10, "Y": int(ys[k, s])} for s in sl],
                     "Witnesses": [bytes(wits[k * total + s]) for s in sl]}
        out.append({"CommitmentUpdate": bytes(commitment), "PolyMap": pm})
    return out


def send_update_secrets_to_miners(addrs: list[str], parts: list[dict], iteration: int, node_id: int,
                                  commitment: bytes, sigs: list, timeout: float) -> int:
    """sendUpdateSecretsToMiners (main.go:1847-1952): the miners' addresses sorted as strings, part i to the
    i-th; returns how many miners took their part."""
    ok = 0
    for i, a in enumerate(sorted(addrs)):
        v = dict(parts[i], Iteration=int(iteration), NodeID=int(node_id), SignatureList=list(sigs),
                 CommitmentUpdate=commitment)
        try:
            N.call(a, "Peer.RegisterSecret", G.MinerPartRPC, v, timeout)
            ok += 1
        except (OSError, N.RpcError):
            continue
    return ok


def get_update_lists(addrs: list[str], iteration: int, timeout: float) -> list[list[int]]:
    """getNodesList (main.go:2237-2324): every miner's contributor list for the iteration (GetUpdateList)."""
    out = []
    for a in addrs:
        try:
            out.append([int(x) for x in N.call(a, "Peer.GetUpdateList", G.INT, int(iteration), timeout)])
        except (OSError, N.RpcError):
            continue
    return out


def get_secret_shares(addrs: list[str], node_list: list[int], timeout: float) -> list[dict]:
    """getSecretShares (main.go:2157-2235): every miner's part summed over node_list (GetMinerPart)."""
    out = []
    for a in addrs:
        try:
            out.append(N.call(a, "Peer.GetMinerPart", G.Slice(G.INT), list(node_list), timeout))
        except (OSError, N.RpcError):
            continue
    return out


def recover_from_parts(R, parts: list[dict], poly: int, d: int, W: np.ndarray, precision: int) -> np.ndarray:
    """recoverSecret (kyber.go:809-857) on the miners' summed parts, exactly (recover_exact; the float64 least
    squares of the reference where a chunk is inconsistent), then W + sum of the deltas (honest.go:405-411)."""
    out = np.array(W, np.float64, copy=True)
    nch = (d + poly - 1) // poly
    for k in range(nch):
        pts = {}
        for p in parts:
            for s in (p.get("PolyMap") or {}).get(k, {}).get("Secrets") or []:
                pts[int(s.get("X") or 0)] = int(s.get("Y") or 0)
        xs = sorted(pts)
        c = R.recover_exact(xs, [pts[x] for x in xs], poly - 1)
        if c is None:
            c = R.recover_lstsq(xs, [pts[x] for x in xs], poly - 1)
        for j, v in enumerate(c):
            i = k * poly + j
            if i < d:
                out[i] += float(v) / 10.0 ** precision
    return out
