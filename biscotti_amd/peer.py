"""Peer entry point: ``python -m biscotti_amd.peer -i <k> -t <N> -d <dataset> [reference flags]``.

Two launch modes share one engine:

* per-peer processes, like DistSys/localTest.sh (``-i k -t N`` and no WORLD_SIZE in the env): the
  process becomes rank k of an N-rank group (rendezvous at 127.0.0.1:8000 = basePort, or the first
  line of the ``-f`` peers file), hosting exactly one peer;
* SPMD under torchrun (WORLD_SIZE set): the N peers are packed as virtual peers onto the ranks,
  one rank per GPU, collectives over RCCL/xGMI.

Rank failure (the reference's crashed peer, FAIL_PROB / failAndRestartLocal.sh): every collective
has a timeout (``--comm-timeout``), so the survivors of a dead rank fail instead of hanging; run
under ``torchrun --max-restarts K`` with ``--chain-file F --resume`` and the restarted job resumes
from the last block on disk (a torn final record is dropped).  ``--fail-at IT --fail-rank R``
injects such a crash deterministically.

At exit rank 0 prints the chain with PrintChain's format (blockchain.go:43-54) to stdout, which
is what localTest.sh compares between peers.

``--rpc-peer`` (with ``-i k -t N`` and a ``-f`` peers file, or local ports 8000+i) runs the reference's own
deployment instead: this process is ONE peer that exchanges every protocol message with the others over Go
net/rpc + gob (protocol/rpcpeer.py: noise requests, VerifyUpdateKRUM, RegisterSecret, the leader's GetUpdateList /
GetMinerPart and RegisterBlock flooding) -- no collective group, so it can run among reference peers.

Talking to peers outside the job (reference peers included) uses the reference's own transport, Go
net/rpc + gob (parallel/netrpc.py): ``--rpc-listen HOST:PORT`` serves the ``Peer`` RPC methods on
rank 0 over the job's chain (RegisterPeer hands it to joiners, RegisterBlock accepts extensions,
RequestNoise / VerifyUpdateKRUM / RegisterSecret / GetMinerPart answer with this peer's roles), and
``--rpc-flood ADDR[,ADDR...]`` sends every committed block to those peers (RegisterBlock, main.go:1403-1444).
"""
from __future__ import annotations

import argparse
import os
import sys

from .protocol.config import add_framework_flags, add_reference_flags, config_from_args


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="biscotti_amd.peer", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    add_reference_flags(ap)
    add_framework_flags(ap)
    ap.add_argument("--rounds", type=int, default=None, help="stop after this many rounds")
    ap.add_argument("--print-chain", default="rank0", choices=["rank0", "all", "none"])
    ap.add_argument("--rpc-listen", default=None, help="HOST:PORT: serve the Peer net/rpc methods (rank 0)")
    ap.add_argument("--rpc-flood", default="", help="comma list of HOST:PORT peers that receive every block")
    ap.add_argument("--rpc-peer", action="store_true",
                    help="run as one peer over net/rpc (the reference's deployment; needs -i and -t)")
    ns = ap.parse_args(argv)
    cfg = config_from_args(ns)
    if cfg.num_nodes <= 0 or not cfg.dataset:
        ap.print_usage()
        return 1
    if ns.rpc_peer:
        return _rpc_peer_main(cfg, ns)
    if "WORLD_SIZE" not in os.environ and cfg.node_index >= 0:
        # one process per peer (reference deployment)
        os.environ["WORLD_SIZE"] = str(cfg.num_nodes)
        os.environ["RANK"] = str(cfg.node_index)
        os.environ.setdefault("LOCAL_RANK", "0")
        host, port = "127.0.0.1", "8000"
        if cfg.peers_file:
            with open(cfg.peers_file) as f:
                first = f.readline().strip()
            host, port = first.rsplit(":", 1)
        os.environ.setdefault("MASTER_ADDR", host)
        os.environ.setdefault("MASTER_PORT", port)
    from .parallel.comm import Comm
    from .protocol.engine import BiscottiEngine

    comm = Comm.init(device=cfg.device, timeout_s=cfg.comm_timeout_s)
    eng = BiscottiEngine(cfg, comm)
    srv, flood = None, [a for a in ns.rpc_flood.split(",") if a.strip()] if comm.rank == 0 else []
    if ns.rpc_listen and comm.rank == 0:
        from .parallel import netrpc

        host, port = ns.rpc_listen.rsplit(":", 1)
        me = eng.lo
        # live: the RPC thread never writes the engine's chain; received blocks are taken between rounds
        svc = netrpc.PeerService(eng.R, eng.fsm.chain, peer_id=me, sk=eng.sk[me],
                                 noise=lambda it: eng.task.noise_scale(eng.sigma) * _noise_row(eng, me, it),
                                 krum_thresh=max(1, eng.pc.krum_thresh), live=True, dim=eng.d)
        srv = netrpc.RpcServer(svc.handlers(), host, int(port), max_conns=netrpc.conns_for(cfg.num_nodes),
                               max_message=netrpc.message_limit(eng.d, cfg.num_nodes)).start()
        eng.log.info("serving Peer net/rpc on %s:%d", *srv.addr)
    n = 0
    while ns.rounds is None or n < ns.rounds:
        r = eng.run_round(last=ns.rounds is not None and n == ns.rounds - 1) if hasattr(eng, "drain") \
            else eng.run_round()
        if r is None:
            eng.log.info("Reached the max iterations!")
            break
        if flood:
            from .parallel import netrpc

            netrpc.flood_block(flood, eng.fsm.chain.latest())
        if srv is not None:
            # blocks flooded to us by outside peers, handled between rounds (processBlock): this job's own
            # FSM is the only writer of its chain, so they are counted and logged, never spliced in
            for it_b, kind, _ in svc.take_blocks():
                eng.stats[f"rpc_blocks_{kind}"] = eng.stats.get(f"rpc_blocks_{kind}", 0) + 1
                if kind != "duplicate":
                    eng.log.info("net/rpc block for iteration %d: %s", it_b, kind)
        n += 1
    if srv is not None:
        srv.close()
    if cfg.colluders > 0:
        print(eng.stats["unmasked_updates"], eng.stats["total_updates"], cfg.colluders / 100.0, cfg.num_noisers)
    if ns.print_chain == "all" or (ns.print_chain == "rank0" and comm.rank == 0):
        sys.stdout.write(eng.print_chain())
        sys.stdout.flush()
    comm.barrier()
    eng.close()
    comm.shutdown()
    return 0


def _rpc_peer_main(cfg, ns) -> int:
    """One peer of a net/rpc deployment (DistSys/main.go: a process per peer, addresses from the peers file or
    127.0.0.1:8000+i): runs --rounds rounds, prints the chain (PrintChain) like localTest.sh compares."""
    import dataclasses

    from .protocol.rpcpeer import RpcPeer

    if cfg.node_index < 0:
        raise SystemExit("--rpc-peer needs -i <index>")
    if cfg.peers_file:
        with open(cfg.peers_file) as f:
            addrs = [ln.strip() for ln in f if ln.strip()][: cfg.num_nodes]
    else:
        addrs = [f"127.0.0.1:{8000 + i}" for i in range(cfg.num_nodes)]
    cfg = dataclasses.replace(cfg, device="cpu")
    peer = RpcPeer(cfg, cfg.node_index, addrs, timeout_s=cfg.comm_timeout_s if cfg.comm_timeout_s < 300 else 30.0)
    try:
        import time

        time.sleep(1.0)   # every peer's server is up before the first round's messages (announceToNetwork)
        for _ in range(ns.rounds or cfg.max_iterations):
            peer.run_round()
        if ns.print_chain != "none":
            sys.stdout.write(peer.fsm.chain.print_chain())
            sys.stdout.flush()
    finally:
        peer.close()
    return 0


def _noise_row(eng, peer: int, it: int):
    """Peer `peer`'s pre-sampled N(0,1) vector of iteration `it` (RequestNoise payload before scaling)."""
    from .ops import ml as K

    return K.noise_vector(peer, it, eng.d, eng.cfg.seed)


if __name__ == "__main__":
    sys.exit(main())
