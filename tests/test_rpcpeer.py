"""Peers that take part in rounds over Go net/rpc + gob (protocol/rpcpeer.py), the reference's deployment model:
every message a point-to-point RPC between peer processes -- noise requests, updates to the verifiers (Multi-Krum
+ Schnorr signatures), Shamir shares to the miners, the leader's node-list intersection and part gather, exact
recovery, block flooding.  Eight peers on loopback (threads of this process, each with its own RPC server,
RoundFSM and ledger) must all end with the same valid chain, and the blocks must carry aggregated updates."""
import socket
import threading

import numpy as np

from biscotti_amd.protocol.config import RunConfig
from biscotti_amd.protocol.rpcpeer import RpcPeer


def _ports(n):
    socks = [socket.socket() for _ in range(n)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def test_rpc_peers_agree_on_the_chain(rt):
    n = 8
    cfg = RunConfig(num_nodes=n, dataset="creditcard", num_verifiers=2, num_miners=2, num_noisers=1, epsilon=1.0,
                    device="cpu", seed=21, deterministic_time=True)
    addrs = [f"127.0.0.1:{p}" for p in _ports(n)]
    peers = [RpcPeer(cfg, i, addrs, timeout_s=20.0) for i in range(n)]
    try:
        for _ in range(3):
            errs = []

            def run(p):
                try:
                    p.run_round()
                except Exception as e:   # noqa: BLE001 (reported below)
                    errs.append((p.id, repr(e)))
            ts = [threading.Thread(target=run, args=(p,)) for p in peers]
            for t in ts:
                t.start()
            for t in ts:
                t.join(timeout=180)
            assert not errs, errs
        chains = [[bytes(p.fsm.chain.block(i).hash) for i in range(len(p.fsm.chain))] for p in peers]
        assert all(c == chains[0] for c in chains) and len(chains[0]) == 4
        assert peers[0].fsm.chain.verify()[0]
        blocks = [peers[0].fsm.chain.block(i) for i in range(1, 4)]
        assert sum(b.data.n_deltas for b in blocks) > 0, [p.log for p in peers]
        assert np.abs(np.asarray(blocks[-1].data.global_w)).sum() > 0
    finally:
        for p in peers:
            p.close()


def test_rpc_peer_processes_localtest_oracle():
    """localTest.sh over net/rpc: N processes `peer -i k -t N -d creditcard --rpc-peer -f peers`, every chain
    dump identical (no collective group: every message is a net/rpc call between the processes)."""
    import os
    import subprocess
    import sys
    import tempfile

    from test_distributed_cpu import ROOT

    n = 6
    with tempfile.TemporaryDirectory() as td:
        pf = os.path.join(td, "peersfile.txt")
        with open(pf, "w") as f:
            f.write("".join(f"127.0.0.1:{p}\n" for p in _ports(n)))
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        env["PYTHONPATH"] = ROOT
        procs = [subprocess.Popen([sys.executable, "-m", "biscotti_amd.peer", f"-i={k}", f"-t={n}", "-d=creditcard",
                                   "-na=2", "-nv=2", "-nn=1", "-f", pf, "--rpc-peer", "--rounds", "3",
                                   "--deterministic-time", "--comm-timeout", "20", "--print-chain", "all"],
                                  cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
                 for k in range(n)]
        outs = []
        for p in procs:
            o, e = p.communicate(timeout=300)
            assert p.returncode == 0, e.decode()[-2000:]
            outs.append(o)
    assert all(o == outs[0] for o in outs) and outs[0].count(b"Hash: ") == 4
