"""Per-round poisoning diagnostics: poisoners submitted / in the verifiers' inbox / approved."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd.parallel.comm import Comm  # noqa: E402
from biscotti_amd.protocol.config import RunConfig  # noqa: E402
from biscotti_amd.protocol.engine import BiscottiEngine  # noqa: E402


def main():
    po = float(sys.argv[1]) if len(sys.argv) > 1 else 0.3
    nv = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    cfg = RunConfig(num_nodes=50, dataset="mnist", poisoning=po, num_verifiers=nv, seed=1, max_iterations=10**9)
    eng = BiscottiEngine(cfg, Comm.init())
    pois = {p for p in range(cfg.num_nodes) if eng.fsm.is_poisoner(p)}
    rows = []
    for _ in range(rounds):
        r = eng.run_round()
        ap = set(r.approved)
        rows.append({"it": r.iteration, "approved": len(ap), "approved_poisoners": len(ap & pois),
                     "block_nodes": len(r.node_list), "block_poisoners": len(set(r.node_list) & pois),
                     "test_err": round(r.test_error, 4), "attack": round(r.attack_rate, 4)})
    print(json.dumps({"poisoners": sorted(pois), "rows": rows}))
    eng.close()


if __name__ == "__main__":
    main()
