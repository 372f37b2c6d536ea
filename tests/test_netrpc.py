"""Go net/rpc + gob transport with the reference's method names (parallel/netrpc.py, parallel/gob.py):
byte-exact gob against the C++ ledger encoder, a loopback server answering RegisterPeer /
RegisterBlock / RequestNoise / VerifyUpdateKRUM / RegisterSecret + GetMinerPart, and a chain a
Biscotti engine produced synced to a follower over the wire."""
import numpy as np
import pytest

from biscotti_amd.parallel import gob as G
from biscotti_amd.parallel import netrpc as N


def test_gob_blockdata_matches_cpp_and_round_trips(rt):
    d = rt.BlockData()
    d.iteration, d.global_w = 7, [0.5, -1.25, 3.0]
    u = rt.Update()
    u.source_id, u.iteration, u.commitment, u.accepted = 4, 7, bytes(range(64)), True
    u.signatures = [b"\x01" * 64, b"\x02" * 64]
    d.deltas = [u]
    py = G.Encoder().encode(G.BlockData, {"Iteration": 7, "GlobalW": [0.5, -1.25, 3.0],
                                          "Deltas": [{"SourceID": 4, "Iteration": 7, "Commitment": bytes(range(64)),
                                                      "Accepted": True, "SignatureList": [b"\x01" * 64, b"\x02" * 64]}]})
    assert py == bytes(d.gob())
    dec = G.Decoder()
    vals = [dec.feed_message(m) for m in G.split_messages(py)]
    assert vals[-1]["Deltas"][0]["SignatureList"] == [b"\x01" * 64, b"\x02" * 64]
    for v in (0, 1, 127, 128, 255, 256, 2**63 - 1, -1, -129, -(2**63)):
        out = bytearray()
        G.enc_int(out, v)
        assert G._Reader(bytes(out)).int() == v


def _chain(rt, n=3):
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    eng = BiscottiEngine(RunConfig(num_nodes=6, dataset="creditcard", num_verifiers=2, num_miners=2, num_noisers=1,
                                   device="cpu", seed=2, deterministic_time=True))
    for _ in range(n):
        eng.run_round()
    return eng


def test_register_peer_and_block_flooding_sync_a_follower(rt):
    eng = _chain(rt)
    leader = N.RpcServer(N.PeerService(rt, eng.fsm.chain).handlers()).start()
    follower_chain = rt.Blockchain.with_genesis(eng.d)
    follower = N.RpcServer(N.PeerService(rt, follower_chain).handlers()).start()
    try:
        addr = f"127.0.0.1:{leader.addr[1]}"
        got = N.announce(addr, "127.0.0.1", follower.addr[1])           # RegisterPeer -> Blockchain
        blocks = got["Blocks"]
        assert len(blocks) == len(eng.fsm.chain)
        assert [bytes(b["Hash"]) for b in blocks] == [bytes(eng.fsm.chain.block(i).hash) for i in range(len(blocks))]
        # flood the leader's blocks to the follower one by one (RegisterBlock), duplicates acknowledged
        fol = f"127.0.0.1:{follower.addr[1]}"
        for i in range(1, len(eng.fsm.chain)):
            assert N.flood_block([fol], eng.fsm.chain.block(i)) == 1
        assert N.flood_block([fol], eng.fsm.chain.latest()) == 1
        assert bytes(follower_chain.latest().hash) == bytes(eng.fsm.chain.latest().hash)
        assert follower_chain.verify()[0]
        # RegisterBlock(block, *returnBlock): the reply decodes as a Block echoing the one sent
        echo = N.call(fol, "Peer.RegisterBlock", G.Block, N.block_to_gob(eng.fsm.chain.latest()))
        assert bytes(echo["Hash"]) == bytes(eng.fsm.chain.latest().hash)
        # a tampered block is echoed too (processBlock runs asynchronously and only logs) but not appended
        bad = N.block_to_gob(eng.fsm.chain.latest())
        bad["Data"]["Iteration"] += 1
        n0 = len(follower_chain)
        N.call(fol, "Peer.RegisterBlock", G.Block, bad)
        assert len(follower_chain) == n0
        with pytest.raises(N.RpcError):
            N.call(fol, "Peer.NoSuchMethod", G.INT, 1)
    finally:
        leader.close()
        follower.close()
        eng.close()


def test_noiser_verifier_and_miner_services(rt):
    from biscotti_amd.ops import ml as K

    sk, pk = rt.client_key_from_entropy(b"\x07" * 32)
    noise = lambda it: -0.5 * K.noise_vector(3, it, 25, 11)
    svc = N.PeerService(rt, rt.Blockchain.with_genesis(25), peer_id=3, sk=sk, noise=noise, krum_thresh=4,
                        krum_timeout_s=5.0)
    srv = N.RpcServer(svc.handlers()).start()
    addr = f"127.0.0.1:{srv.addr[1]}"
    try:
        got = N.call(addr, "Peer.RequestNoise", G.INT, 5)
        np.testing.assert_allclose(got, noise(5))
        # four updates, one outlier: Multi-Krum accepts n - floor(n/2) = 2, never the outlier
        import threading

        rng = np.random.default_rng(0)
        rows = [rng.normal(0, 0.01, 25) for _ in range(3)] + [np.full(25, 5.0)]
        out = {}

        def send(i):
            u = {"SourceID": 10 + i, "Iteration": 1, "Commitment": bytes([i]) * 64, "NoisedDelta": list(rows[i])}
            try:
                out[i] = N.call(addr, "Peer.VerifyUpdateKRUM", G.Update, u)
            except N.RpcError:
                out[i] = None
        ts = [threading.Thread(target=send, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert out[3] is None and sum(v is not None for v in out.values()) == 2
        for i, s in out.items():
            if s is not None:
                assert rt.schnorr_verify(bytes([i]) * 64, pk, bytes(s))
        # miner: two parts stored, summed per x on GetMinerPart
        g = rt.g1_generator()
        two = rt.g1_add(g, g)
        for node, y in ((21, 5), (22, 7)):
            part = {"CommitmentUpdate": g, "Iteration": 2, "NodeID": node,
                    "PolyMap": {0: {"Commitment": g, "Secrets": [{"X": -10, "Y": y}, {"X": -9, "Y": 2 * y}],
                                    "Witnesses": [g, g]}}}
            assert N.call(addr, "Peer.RegisterSecret", G.MinerPartRPC, part) is True
        assert N.call(addr, "Peer.GetUpdateList", G.INT, 2) == [21, 22]
        mp = N.call(addr, "Peer.GetMinerPart", G.Slice(G.INT), [21, 22])
        assert mp["PolyMap"][0]["Secrets"] == [{"X": -10, "Y": 12}, {"X": -9, "Y": 24}]
        assert mp["PolyMap"][0]["Commitment"] == two and mp["CommitmentUpdate"] == two
        assert mp["PolyMap"][0]["Witnesses"] == [two, two]
    finally:
        srv.close()


def test_live_service_never_writes_the_engine_chain(rt):
    """--rpc-listen serves the running engine's chain: a block for the iteration the engine is about to
    commit arrives over net/rpc first (a reference peer flooding its own block) -- the RPC thread only
    queues it, the engine commits its own block, and the queued one is classified between rounds."""
    eng = _chain(rt, 3)
    other = _chain_seed(rt, 4, seed=3)     # a different chain: its iteration-3 block conflicts with ours
    svc = N.PeerService(rt, eng.fsm.chain, live=True, dim=eng.d)
    srv = N.RpcServer(svc.handlers()).start()
    try:
        addr = f"127.0.0.1:{srv.addr[1]}"
        theirs = other.fsm.chain.block(4)
        assert theirs.data.iteration == eng.fsm.iteration
        N.call(addr, "Peer.RegisterBlock", G.Block, N.block_to_gob(theirs))
        assert len(eng.fsm.chain) == 4                # not spliced in by the RPC thread
        assert eng.run_round() is not None           # the engine's own commit is not refused
        got = svc.take_blocks()
        assert [(it, kind) for it, kind, _ in got] == [(3, "conflict")]
        assert eng.fsm.chain.verify()[0] and len(eng.fsm.chain) == 5
        # an update of the wrong length never reaches a verifier inbox
        with pytest.raises(N.RpcError):
            N.call(addr, "Peer.VerifyUpdateKRUM", G.Update, {"SourceID": 1, "Iteration": 4, "NoisedDelta": [0.0] * 3})
    finally:
        srv.close()
        eng.close()
        other.close()


def _chain_seed(rt, n, seed):
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    eng = BiscottiEngine(RunConfig(num_nodes=6, dataset="creditcard", num_verifiers=2, num_miners=2, num_noisers=1,
                                   device="cpu", seed=seed, deterministic_time=True))
    for _ in range(n):
        eng.run_round()
    return eng


def test_gob_decoder_bounds():
    """Go's decoder limits: uints of at most 8 bytes, messages of at most 1 GB, and element counts no
    larger than the bytes left (a declared count is never trusted for an allocation or a loop)."""
    import io

    with pytest.raises(ValueError):
        G._Reader(bytes([256 - 9]) + bytes(9)).uint()
    with pytest.raises(ValueError):
        G.read_message(io.BytesIO(bytes([256 - 4]) + (1 << 31).to_bytes(4, "big")))
    with pytest.raises(ValueError):
        G.read_message(io.BytesIO(bytes([256 - 2]) + (1000).to_bytes(2, "big") + bytes(1000)), limit=999)
    # a []float64 claiming 2^40 elements in a 10-byte message
    enc = G.Encoder()
    msgs = G.split_messages(enc.encode(G.Slice(G.FLOAT), [1.0, 2.0]))
    dec = G.Decoder()
    for m in msgs[:-1]:
        dec.feed_message(m)
    tid = G._Reader(msgs[-1]).int()
    forged = bytearray()
    G.enc_int(forged, tid)
    G.enc_uint(forged, 0)            # singleton field
    G.enc_uint(forged, 1 << 40)      # the declared element count
    G.enc_float(forged, 1.0)
    with pytest.raises(ValueError):
        dec.feed_message(bytes(forged))


def test_peer_cli_serves_and_floods(tmp_path):
    """peer.py --rpc-listen / --rpc-flood: a single-rank run serves its chain over net/rpc while a
    follower service receives every committed block."""
    import os
    import socket
    import subprocess
    import sys
    import time

    from biscotti_amd.native import rt

    R = rt()
    follower_chain = R.Blockchain.with_genesis(25)
    follower = N.RpcServer(N.PeerService(R, follower_chain).handlers()).start()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        p = subprocess.run([sys.executable, "-m", "biscotti_amd.peer", "-t=6", "-d=creditcard", "-na=2", "-nv=2",
                            "-nn=1", "--device", "cpu", "--rounds", "3", "--deterministic-time", "--print-chain", "none",
                            "--rpc-listen", f"127.0.0.1:{port}", "--rpc-flood", f"127.0.0.1:{follower.addr[1]}"],
                           cwd=root, env=dict(os.environ, PYTHONPATH=root), capture_output=True, timeout=300)
        assert p.returncode == 0, p.stderr.decode()[-2000:]
        assert len(follower_chain) == 4 and follower_chain.verify()[0]
    finally:
        follower.close()


def test_far_future_iteration_cannot_evict_current_round(rt):
    """pruning follows this peer's own progress (its chain), not the largest Iteration a remote
    peer sends -- a forged far-future message is refused and the current round's shares survive."""
    g = rt.g1_generator()
    svc = N.PeerService(rt, rt.Blockchain.with_genesis(25), peer_id=3, krum_thresh=2, krum_timeout_s=2.0)
    srv = N.RpcServer(svc.handlers()).start()
    addr = f"127.0.0.1:{srv.addr[1]}"
    try:
        assert svc.current_iteration() == 0
        part = {"CommitmentUpdate": g, "Iteration": 0, "NodeID": 5,
                "PolyMap": {0: {"Commitment": g, "Secrets": [{"X": -10, "Y": 1}], "Witnesses": [g]}}}
        assert N.call(addr, "Peer.RegisterSecret", G.MinerPartRPC, part) is True
        with pytest.raises(N.RpcError, match="too far ahead"):
            N.call(addr, "Peer.RegisterSecret", G.MinerPartRPC, dict(part, Iteration=10**9, NodeID=6))
        with pytest.raises(N.RpcError, match="too far ahead"):
            N.call(addr, "Peer.VerifyUpdateKRUM", G.Update,
                   {"SourceID": 1, "Iteration": 10**9, "Commitment": bytes(64), "NoisedDelta": [0.0] * 25})
        assert N.call(addr, "Peer.GetUpdateList", G.INT, 0) == [5]
        assert set(svc.secrets_of(0)) == {5}
        # within the window ahead (a peer one round ahead of this one) is accepted
        assert N.call(addr, "Peer.RegisterSecret", G.MinerPartRPC, dict(part, Iteration=2, NodeID=7)) is True
        assert set(svc.secrets_of(0)) == {5}
    finally:
        srv.close()


def test_verifier_threshold_above_old_connection_cap(rt):
    """a verifier holds one connection per worker until its Krum threshold; 80 concurrent
    VerifyUpdateKRUM calls (more than the 64 connections the server used to allow) all reach the threshold and
    get a decision before the deadline, and extra connections wait in the backlog instead of being closed."""
    import threading
    import time

    sk, _ = rt.client_key_from_entropy(b"\x09" * 32)
    n = 80
    svc = N.PeerService(rt, rt.Blockchain.with_genesis(25), peer_id=0, sk=sk, krum_thresh=n, krum_timeout_s=60.0)
    srv = N.RpcServer(svc.handlers(), max_conns=N.conns_for(n)).start()
    addr = f"127.0.0.1:{srv.addr[1]}"
    rng = np.random.default_rng(1)
    out = {}

    def send(i):
        u = {"SourceID": i, "Iteration": 0, "Commitment": bytes([i % 256]) * 64,
             "NoisedDelta": list(rng.normal(0, 0.01, 25))}
        try:
            out[i] = N.call(addr, "Peer.VerifyUpdateKRUM", G.Update, u, timeout=60.0)
        except N.RpcError as e:
            out[i] = str(e)
        except OSError as e:
            out[i] = ("socket", str(e))
    t0 = time.monotonic()
    try:
        ts = [threading.Thread(target=send, args=(i,)) for i in range(n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        srv.close()
    assert time.monotonic() - t0 < 30.0, "the threshold was not reached: the deadline decided"
    assert not [v for v in out.values() if isinstance(v, tuple)], "a connection was dropped"
    acc = [v for v in out.values() if isinstance(v, bytes)]
    assert len(acc) == n - n // 2, len(acc)
    # a server with fewer slots than the threshold queues the rest: the late callers get a decision (the
    # deadline's), never a closed socket
    svc2 = N.PeerService(rt, rt.Blockchain.with_genesis(25), peer_id=0, sk=sk, krum_thresh=6, krum_timeout_s=1.0)
    srv2 = N.RpcServer(svc2.handlers(), max_conns=3).start()
    addr, out = f"127.0.0.1:{srv2.addr[1]}", {}
    try:
        ts = [threading.Thread(target=send, args=(i,)) for i in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        srv2.close()
    assert len(out) == 6 and not [v for v in out.values() if isinstance(v, tuple)], out
