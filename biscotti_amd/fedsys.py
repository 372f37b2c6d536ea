"""FedSys baseline entry point: ``python -m biscotti_amd.fedsys -i <k> -t <N> -d <dataset> [-ns 35 -rs -po]``.

Same launch modes as ``biscotti_amd.peer`` (one process per peer like FedSys/localTest.sh, or SPMD
under torchrun).  Flags and defaults follow FedSys/main.go:195-218: -ns 35, -rs, -po; EPSILON = 5
(main.go:42) for the creditcard at-source noise.  At exit rank 0 prints the final model digest and
iteration, the value FedSys/localTest.sh compares between peers.
"""
from __future__ import annotations

import argparse
import os
import sys

from .protocol.config import add_framework_flags, add_reference_flags, config_from_args


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="biscotti_amd.fedsys", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    add_reference_flags(ap)
    add_framework_flags(ap)
    ap.set_defaults(perc_samples=35, epsilon=5.0)
    ap.add_argument("--rounds", type=int, default=None)
    ns = ap.parse_args(argv)
    cfg = config_from_args(ns)
    if cfg.num_nodes <= 1 or not cfg.dataset:
        ap.print_usage()
        return 1
    if "WORLD_SIZE" not in os.environ and cfg.node_index >= 0:
        os.environ.update(WORLD_SIZE=str(cfg.num_nodes), RANK=str(cfg.node_index))
        os.environ.setdefault("LOCAL_RANK", "0")
        host, port = "127.0.0.1", "8000"
        if cfg.peers_file:
            with open(cfg.peers_file) as f:
                host, port = f.readline().strip().rsplit(":", 1)
        os.environ.setdefault("MASTER_ADDR", host)
        os.environ.setdefault("MASTER_PORT", port)
    from .parallel.comm import Comm
    from .protocol.fedsys import FedSysEngine

    comm = Comm.init(device=cfg.device)
    eng = FedSysEngine(cfg, comm)
    n = 0
    while ns.rounds is None or n < ns.rounds:
        if eng.run_round() is None:
            eng.log.info("Reached the max iterations!")
            break
        n += 1
    if comm.rank == 0:
        sys.stdout.write(f"iteration {eng.iteration - 1} model {eng.model_digest()}\n")
        sys.stdout.flush()
    comm.barrier()
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
