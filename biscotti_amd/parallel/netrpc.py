"""Go net/rpc over TCP with gob bodies -- the reference's transport, wire-compatible, with the reference's
method names (DistSys/main.go:191-485, krum.go:227-365).

The SPMD engine moves a round through collectives (parallel/comm.py); this module is the thin TCP
layer for talking to peers outside the job -- reference peers included -- with the messages they
understand:

  Peer.RegisterPeer      net.TCPAddr -> Blockchain       a joiner adopts the longest chain (main.go:420-436)
  Peer.RegisterBlock     Block -> Block                  block flooding: the block is echoed, processed
                                                         asynchronously (main.go:398-409, processBlock)
  Peer.RequestNoise      int -> []float64                a noiser's pre-sampled vector (main.go:239-248)
  Peer.VerifyUpdateKRUM  Update -> []byte                a verifier collects its inbox, runs Multi-Krum,
                                                         signs accepted commitments (krum.go:227-365)
  Peer.RegisterSecret    MinerPartRPC -> bool            a miner stores shares (main.go:256-286)
  Peer.RegisterUpdate    Update -> bool                  the plain path's update (main.go:375-390)
  Peer.GetUpdateList     int -> []int                    the miner's contributor list (main.go:438-457)
  Peer.GetMinerPart      []int -> MinerPartRPC           the miner's summed part (main.go:459-485)

Wire protocol (Go's rpc.gobServerCodec / gobClientCodec): each direction of a connection is ONE gob
stream; a call is gob(Request{ServiceMethod, Seq}) + gob(args), a reply gob(Response{ServiceMethod,
Seq, Error}) + gob(reply) (an empty struct when Error is set).  `call` dials per call like the
reference (rpc.Dial + Call under a timeout, main.go:1453-1475).

    python -m biscotti_amd.parallel.netrpc serve --port 8000 --chain-file chain.bin
    python -m biscotti_amd.parallel.netrpc call 127.0.0.1:8000 Peer.RegisterPeer
"""
from __future__ import annotations

import socket
import threading

import numpy as np

from . import gob as G


# ---------------------------------------------------------------------------- transport
def _send(sock, data: bytes) -> None:
    sock.sendall(data)


class _ValueReader:
    """Reads values (skipping type definitions) off a gob stream; messages over `limit` bytes are refused."""

    def __init__(self, stream, limit: int = G.MAX_MESSAGE):
        self.stream, self.dec, self.limit = stream, G.Decoder(), limit

    def next(self):
        while True:
            payload = G.read_message(self.stream, self.limit)
            r = G._Reader(payload)
            if r.int() < 0:
                self.dec.feed_message(payload)
                continue
            return self.dec.feed_message(payload)


class RpcServer:
    """net/rpc server: handlers maps "Peer.Method" -> (arg schema, reply schema, fn(args) -> reply).  One
    thread per connection, calls on a connection served in order (Go serves them concurrently; the
    reference's clients issue one call per connection).  At most `max_conns` connections are served at
    once; further ones wait in the listen backlog until a slot frees (a verifier holds one connection per
    worker until its Krum threshold, so closing them would starve the threshold -- size max_conns from the
    peer count, `conns_for`).  A connection idle for `idle_s` is dropped, and gob messages over
    `max_message` bytes are refused before their body is read, so a peer cannot exhaust the server's
    threads or memory."""

    def __init__(self, handlers: dict, host: str = "127.0.0.1", port: int = 0, max_conns: int = 256,
                 idle_s: float = 120.0, max_message: int = G.MAX_MESSAGE):
        self.handlers = handlers
        self._slots = threading.BoundedSemaphore(max_conns)
        self.idle_s, self.max_message = idle_s, max_message
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(max(128, 2 * max_conns))
        self.addr = self.sock.getsockname()
        self._stop = False
        self._thr = threading.Thread(target=self._accept, daemon=True)

    def start(self) -> "RpcServer":
        self._thr.start()
        return self

    def close(self) -> None:
        self._stop = True
        try:
            self.sock.close()
        except OSError:
            pass

    def _accept(self) -> None:
        while not self._stop:
            # a free slot first: while every slot is busy, new connections queue in the kernel's backlog
            if not self._slots.acquire(timeout=0.25):
                continue
            try:
                conn, _ = self.sock.accept()
            except OSError:
                self._slots.release()
                return
            conn.settimeout(self.idle_s)
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn) -> None:
        f = conn.makefile("rb")
        rd, enc = _ValueReader(f, self.max_message), G.Encoder()
        try:
            while True:
                try:
                    hdr = rd.next()
                except (EOFError, OSError, ValueError, KeyError, IndexError):
                    return   # closed, idle, or a malformed stream: drop the connection
                args = rd.next()   # the body is always read (also for an unknown method)
                name, seq = hdr.get("ServiceMethod") or "", hdr.get("Seq") or 0
                h = self.handlers.get(name)
                err, reply, rs = "", None, None
                if h is None:
                    err = f"rpc: can't find method {name}"
                else:
                    _, rs, fn = h
                    try:
                        reply = fn(args)
                    except Exception as e:   # reported to the caller like a Go error return
                        err = str(e) or type(e).__name__
                out = enc.encode(G.Response, {"ServiceMethod": name, "Seq": seq, "Error": err})
                out += enc.encode(G.InvalidRequest, {}) if err else enc.encode(rs, reply)
                _send(conn, out)
        except (EOFError, OSError, ValueError, KeyError, IndexError):
            return
        finally:
            f.close()
            conn.close()
            self._slots.release()


class RpcError(RuntimeError):
    pass


def conns_for(num_nodes: int) -> int:
    """Connections a peer's server may hold at once: every other peer's VerifyUpdateKRUM (held until the Krum
    threshold) plus its concurrent RequestNoise / RegisterSecret / RegisterBlock calls."""
    return 2 * max(1, int(num_nodes)) + 16


def message_limit(dim: int, num_nodes: int) -> int:
    """Largest gob message a peer expects: a block of every peer's update (three float64 vectors of `dim`,
    <= 9 bytes per gob float, plus commitments and signatures) dominates; 1 MB of envelope slack."""
    return (1 << 20) + 32 * max(1, int(dim)) * (max(1, int(num_nodes)) + 1)


def call(addr: str, method: str, arg_schema, args, timeout: float = 30.0):
    """One net/rpc call on a fresh connection (rpc.Dial + Call); returns the decoded reply."""
    host, port = addr.rsplit(":", 1)
    with socket.create_connection((host, int(port)), timeout=timeout) as s:
        enc = G.Encoder()
        _send(s, enc.encode(G.Request, {"ServiceMethod": method, "Seq": 0}) + enc.encode(arg_schema, args))
        f = s.makefile("rb")
        rd = _ValueReader(f)
        hdr = rd.next()
        body = rd.next()
        if hdr.get("Error"):
            raise RpcError(hdr["Error"])
        return body


# ---------------------------------------------------------------------------- ledger conversions
def block_to_gob(b) -> dict:
    """Native Block -> the reference's Block value."""
    d = b.data
    return {"Timestamp": int(b.timestamp), "PrevBlockHash": bytes(b.prev_hash), "Hash": bytes(b.hash),
            "StakeMap": {int(k): int(v) for k, v in dict(b.stake).items()},
            "Data": {"Iteration": int(d.iteration), "GlobalW": list(d.global_w),
                     "Deltas": [{"SourceID": u.source_id, "Iteration": u.iteration, "Delta": list(u.delta),
                                 "Commitment": bytes(u.commitment), "Noise": list(u.noise),
                                 "NoisedDelta": list(u.noised_delta), "Accepted": bool(u.accepted),
                                 "SignatureList": [bytes(s) for s in u.signatures]} for u in d.deltas]}}


def gob_to_block(v: dict, rt):
    """The reference's Block value -> native Block (hash fields taken as sent; verify separately)."""
    b = rt.Block()
    b.timestamp = int(v.get("Timestamp") or 0)
    b.prev_hash = bytes(v.get("PrevBlockHash") or b"")
    b.hash = bytes(v.get("Hash") or b"")
    b.stake = {int(k): int(x) for k, x in (v.get("StakeMap") or {}).items()}
    dv = v.get("Data") or {}
    d = rt.BlockData()
    d.iteration = int(dv.get("Iteration") or 0)
    d.global_w = list(dv.get("GlobalW") or [])
    ups = []
    for uv in dv.get("Deltas") or []:
        u = rt.Update()
        u.source_id, u.iteration = int(uv.get("SourceID") or 0), int(uv.get("Iteration") or 0)
        u.delta = list(uv.get("Delta") or [])
        u.commitment = bytes(uv.get("Commitment") or b"")
        u.noise = list(uv.get("Noise") or [])
        u.noised_delta = list(uv.get("NoisedDelta") or [])
        u.accepted = bool(uv.get("Accepted"))
        u.signatures = [bytes(s) for s in (uv.get("SignatureList") or [])]
        ups.append(u)
    d.deltas = ups
    b.data = d
    return b


# ---------------------------------------------------------------------------- the peer service
class PeerService:
    """The reference's `Peer` RPC service for one peer: ledger (chain sync and block flooding), noiser,
    verifier (Multi-Krum over its inbox, Schnorr signatures) and miner (share store and sums) roles.

    chain: a native Blockchain (the engine's, or a follower's); peer_id, sk: this peer's id and Schnorr
    key; noise(it) -> its scaled noise vector; krum_thresh: KRUM_UPDATETHRESH; krum_timeout_s: the
    verifier's deadline (startKRUMDeadlineTimer); dim: the model size (updates of another length are
    refused before they reach an inbox).

    live=True: `chain` belongs to a running engine, whose FSM alone commits blocks.  RegisterBlock then
    never touches the chain from the RPC thread: verified blocks are queued and the engine's loop takes
    them between rounds (take_blocks) -- the reference's asynchronous processBlock, without a second
    writer racing the round's commit.  live=False (a follower / the `serve` CLI): the service owns the
    chain and appends extensions itself.  Per-iteration state (inboxes, decisions, shares, updates) is
    kept for the last KEEP_ITERATIONS iterations only, measured from this peer's OWN progress (its chain's next
    iteration, or `progress()`): a message more than AHEAD_ITERATIONS past it is refused, so no remote
    Iteration field can evict the current round's state (the reference's RegisterUpdate / processBlock
    likewise judge staleness against the peer's own iterationCount)."""

    KEEP_ITERATIONS = 4
    AHEAD_ITERATIONS = 4
    MAX_QUEUED_BLOCKS = 64

    def __init__(self, rt, chain, peer_id: int = 0, sk: bytes | None = None, noise=None, krum_thresh: int = 1,
                 krum_timeout_s: float = 10.0, lock: threading.Lock | None = None, live: bool = False,
                 dim: int | None = None, progress=None):
        self.rt, self.chain, self.id, self.sk, self.noise = rt, chain, peer_id, sk, noise
        self._progress = progress
        self.lock = lock or threading.Lock()
        self.live, self.dim = live, dim
        self.peers: list = []           # addresses announced through RegisterPeer
        self.krum_thresh, self.krum_timeout_s = krum_thresh, krum_timeout_s
        self._inbox: dict = {}          # iteration -> [Update values]
        self._decided: dict = {}        # iteration -> {SourceID: accepted}
        self._cv = threading.Condition(self.lock)
        self._secrets: dict = {}        # iteration -> {NodeID: MinerPartRPC value}
        self._updates: dict = {}        # iteration -> [Update values]
        self._blocks: list = []         # live: verified blocks waiting for the engine (take_blocks)
        self.block_log: list = []       # (iteration, outcome) of every RegisterBlock, newest last (bounded)

    def _note(self, it: int, what: str) -> None:
        self.block_log.append((it, what))
        del self.block_log[:-256]

    def current_iteration(self) -> int:
        """The iteration this peer is working on: progress(), else its chain's latest block + 1."""
        if self._progress is not None:
            return int(self._progress())
        li = getattr(self.chain, "latest_iteration", None)   # native: no copy of the latest block (GlobalW)
        return int(li() if li is not None else self.chain.latest().data.iteration) + 1

    def _admit(self, it: int) -> None:
        """Refuse a message whose iteration is outside [current - KEEP, current + AHEAD] and forget state
        older than current - KEEP (caller holds the lock).  The window moves with this peer's own progress
        only: the largest Iteration a remote peer sends decides nothing."""
        cur = self.current_iteration()
        lo = cur - self.KEEP_ITERATIONS
        for d in (self._inbox, self._decided, self._secrets, self._updates):
            for k in [k for k in d if k < lo]:
                del d[k]
        if it < lo:
            raise ValueError(f"stale message for iteration {it} (this peer is at {cur})")
        if it > cur + self.AHEAD_ITERATIONS:
            raise ValueError(f"message for iteration {it} too far ahead (this peer is at {cur})")

    def secrets_of(self, it: int) -> dict:
        """{NodeID: MinerPartRPC value} stored for iteration it (a copy)."""
        with self.lock:
            return dict(self._secrets.get(it, {}))

    def handlers(self) -> dict:
        return {
            "Peer.RegisterPeer": (G.TCPAddr, G.Blockchain, self.register_peer),
            "Peer.RegisterBlock": (G.Block, G.Block, self.register_block),
            "Peer.RequestNoise": (G.INT, G.Slice(G.FLOAT), self.request_noise),
            "Peer.VerifyUpdateKRUM": (G.Update, G.BYTES, self.verify_update_krum),
            "Peer.RegisterSecret": (G.MinerPartRPC, G.BOOL, self.register_secret),
            "Peer.RegisterUpdate": (G.Update, G.BOOL, self.register_update),
            "Peer.GetUpdateList": (G.INT, G.Slice(G.INT), self.get_update_list),
            "Peer.GetMinerPart": (G.Slice(G.INT), G.MinerPartRPC, self.get_miner_part),
        }

    # ---- ledger
    def register_peer(self, addr: dict) -> dict:
        with self.lock:
            ip = bytes(addr.get("IP") or b"")
            host = ".".join(str(x) for x in ip[-4:]) if len(ip) >= 4 else ""
            self.peers.append(f"{host}:{int(addr.get('Port') or 0)}")
            return {"Blocks": [block_to_gob(self.chain.block(i)) for i in range(len(self.chain))]}

    def register_block(self, v: dict) -> dict:
        """RegisterBlock(block, *returnBlock) (main.go:398-409): echo the block and process it
        asynchronously -- the caller never gets an error (stale, duplicate and conflicting blocks are
        logged, as processBlock does).  live: queued for the engine; otherwise appended here when its
        hash verifies and it extends the chain."""
        b = gob_to_block(v, self.rt)
        it = int(b.data.iteration)
        ok_hash = bytes(b.compute_hash()) == bytes(b.hash)
        with self.lock:
            if not ok_hash:
                self._note(it, "bad-hash")
            elif self.live:
                if len(self._blocks) < self.MAX_QUEUED_BLOCKS:
                    self._blocks.append(b)
                    self._note(it, "queued")
                else:
                    self._note(it, "queue-full")
            else:
                self._note(it, self._append(b))
        return v

    def _append(self, b) -> str:
        """Follower: append b if it extends the chain (caller holds the lock)."""
        have = self.chain.get(int(b.data.iteration))
        if have is not None:
            return "duplicate" if bytes(have.hash) == bytes(b.hash) else "conflict"
        if bytes(b.prev_hash) != bytes(self.chain.latest().hash):
            return "not-extending"
        self.chain.append(b)
        return "appended"

    def take_blocks(self) -> list:
        """live: the blocks received since the last call, each classified against the engine's chain as
        duplicate (the engine committed the same block), conflict (another block for an iteration the
        engine has), ahead (an iteration the engine has not reached) -- call between rounds."""
        with self.lock:
            got, self._blocks = self._blocks, []
        out = []
        for b in got:
            it = int(b.data.iteration)
            have = self.chain.get(it)
            kind = "ahead" if have is None else ("duplicate" if bytes(have.hash) == bytes(b.hash) else "conflict")
            out.append((it, kind, b))
        return out

    def get_update_list(self, it: int) -> list:
        with self.lock:
            if it in self._secrets:
                return sorted(self._secrets[it])
            b = self.chain.get(int(it))
            return [] if b is None else [u.source_id for u in b.data.deltas]

    # ---- noiser
    def request_noise(self, it: int) -> list:
        if self.noise is None:
            raise ValueError("this peer is not a noiser")
        return [float(x) for x in np.asarray(self.noise(int(it)), np.float64)]

    # ---- verifier
    def verify_update_krum(self, u: dict) -> bytes:
        """Collect updates of the iteration until KRUM_UPDATETHRESH or the deadline, run Multi-Krum once
        over the inbox (n - floor(n/2) accepted, client_obj.py:114-143) and sign the accepted
        commitments (kyber.go:873-896); a rejected update gets an error."""
        from ..ops import ml as K

        import time
        import torch

        it = int(u.get("Iteration") or 0)
        row = u.get("NoisedDelta") or u.get("Delta") or []
        if self.dim is not None and len(row) != self.dim:
            raise ValueError(f"update of length {len(row)}: the model has {self.dim} parameters")
        with self._cv:
            self._admit(it)
            box = self._inbox.setdefault(it, [])
            box.append(u)
            if len(box) >= self.krum_thresh:
                self._cv.notify_all()
            deadline = time.monotonic() + self.krum_timeout_s
            while it not in self._decided:
                if it not in self._inbox:   # this peer moved past the iteration while we waited
                    raise ValueError(f"stale update for iteration {it}")
                if len(self._inbox[it]) >= self.krum_thresh or time.monotonic() >= deadline:
                    self._decide(it, K, torch)
                    break
                self._cv.wait(timeout=max(0.0, deadline - time.monotonic()))
            dec = self._decided.get(it)
            if dec is None:
                raise ValueError(f"stale update for iteration {it}")
            ok = dec.get(int(u.get("SourceID") or 0), False)
        if not ok:
            raise ValueError("update rejected by Multi-Krum")
        if self.sk is None:
            raise ValueError("this peer has no signing key")
        nonce = self.rt.sha256(bytes(self.sk) + bytes(u.get("Commitment") or b"") + it.to_bytes(8, "little"))
        return bytes(self.rt.schnorr_sign(bytes(u.get("Commitment") or b""), self.sk, nonce))

    def _decide(self, it, K, torch) -> None:
        """Krum over the inbox of `it`; a failure is recorded as every update rejected (later callers for
        the iteration then get that decision instead of re-running a failing Krum)."""
        box = self._inbox[it]
        box.sort(key=lambda x: int(x.get("SourceID") or 0))
        try:
            X = torch.tensor([list(x.get("NoisedDelta") or x.get("Delta") or []) for x in box], dtype=torch.float32)
            n = len(box)
            clip = n // 2
            acc, _ = K.krum(X, n - clip, n - clip) if n > 1 else (torch.ones(n, dtype=torch.bool), None)
            self._decided[it] = {int(x.get("SourceID") or 0): bool(a) for x, a in zip(box, acc.tolist())}
        except Exception:
            self._decided[it] = {}
        self._cv.notify_all()

    # ---- miner
    def register_secret(self, part: dict) -> bool:
        with self.lock:
            it = int(part.get("Iteration") or 0)
            self._admit(it)
            self._secrets.setdefault(it, {})[int(part.get("NodeID") or 0)] = part
            return True

    def register_update(self, u: dict) -> bool:
        with self.lock:
            it = int(u.get("Iteration") or 0)
            self._admit(it)
            self._updates.setdefault(it, []).append(u)
            return True

    def get_miner_part(self, node_list: list) -> dict:
        """aggregateSecret (kyber.go:244-287) over the listed nodes' parts of the latest iteration that has
        them: share values summed per chunk and x, witnesses and commitments added on G1."""
        with self.lock:
            its = [i for i, p in self._secrets.items() if all(n in p for n in node_list)]
            if not its or not node_list:
                raise ValueError("no stored parts for that node list")
            parts = [self._secrets[max(its)][n] for n in node_list]
        out_map = {}
        for chunk in parts[0].get("PolyMap") or {}:
            pp = [p["PolyMap"][chunk] for p in parts]
            ys: dict = {}
            for p in pp:
                for sh in p.get("Secrets") or []:
                    ys[int(sh.get("X") or 0)] = ys.get(int(sh.get("X") or 0), 0) + int(sh.get("Y") or 0)
            wit = np.stack([np.frombuffer(b"".join(p.get("Witnesses") or []), np.uint8).reshape(-1, 64) for p in pp])
            com = np.stack([np.frombuffer(bytes(p.get("Commitment") or bytes(64)), np.uint8).reshape(1, 64) for p in pp])
            ws = self.rt.g1_sum_marshaled(wit) if wit.shape[1] else wit[0]
            cs = self.rt.g1_sum_marshaled(com)
            out_map[int(chunk)] = {"Polynomial": [], "Commitment": bytes(np.asarray(cs)[0]),
                                   "Secrets": [{"X": x, "Y": y} for x, y in sorted(ys.items())],
                                   "Witnesses": [bytes(r) for r in np.asarray(ws)]}
        cu = np.stack([np.frombuffer(bytes(p.get("CommitmentUpdate") or bytes(64)), np.uint8).reshape(1, 64)
                       for p in parts])
        return {"CommitmentUpdate": bytes(np.asarray(self.rt.g1_sum_marshaled(cu))[0]),
                "Iteration": int(parts[0].get("Iteration") or 0), "NodeID": self.id, "SignatureList": [],
                "PolyMap": out_map}


def announce(addr: str, my_ip: str, my_port: int, timeout: float = 30.0) -> dict:
    """callRegisterPeerRPC (main.go:950-1024): announce to a peer, get its chain back."""
    ip = bytes(10) + b"\xff\xff" + bytes(int(x) for x in my_ip.split("."))   # net.IP: 16-byte form
    return call(addr, "Peer.RegisterPeer", G.TCPAddr, {"IP": ip, "Port": my_port, "Zone": ""}, timeout)


def flood_block(peers: list, block, timeout: float = 10.0) -> int:
    """sendBlock (main.go:1403-1444): RegisterBlock on every peer; returns how many acknowledged."""
    v = block_to_gob(block)
    ok = 0
    for p in peers:
        try:
            call(p, "Peer.RegisterBlock", G.Block, v, timeout)   # the reply echoes the block
            ok += 1
        except (OSError, RpcError):
            pass
    return ok


def main(argv=None) -> int:
    import argparse
    import time

    from ..native import rt

    ap = argparse.ArgumentParser(prog="python -m biscotti_amd.parallel.netrpc")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("serve", help="serve a chain file as a reference-compatible peer")
    s.add_argument("--host", default="127.0.0.1")
    s.add_argument("--port", type=int, default=8000)
    s.add_argument("--chain-file", default=None)
    s.add_argument("--seconds", type=float, default=0.0, help="serve this long (0: forever)")
    c = sub.add_parser("call", help="call RegisterPeer on a peer and print its chain")
    c.add_argument("addr")
    c.add_argument("method", choices=["Peer.RegisterPeer"])
    a = ap.parse_args(argv)
    R = rt()
    if a.cmd == "serve":
        chain = R.Blockchain.load(a.chain_file) if a.chain_file else R.Blockchain.with_genesis(0)
        srv = RpcServer(PeerService(R, chain).handlers(), a.host, a.port,
                        max_message=message_limit(len(chain.latest().data.global_w), 256)).start()
        print(f"serving {len(chain)} blocks on {srv.addr[0]}:{srv.addr[1]}", flush=True)
        t0 = time.time()
        while not a.seconds or time.time() - t0 < a.seconds:
            time.sleep(0.2)
        srv.close()
    else:
        got = announce(a.addr, "127.0.0.1", 0)
        for b in got.get("Blocks") or []:
            print(b["Data"]["Iteration"], bytes(b["Hash"]).hex())
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
