"""Per-round poisoning diagnostics of the engine (GPU or CPU) over several configs and seeds.

For every round: poisoners among the workers, in the verifiers' inboxes, accepted by at least one
verifier's Krum, approved (>= floor(nv/2) signatures), and in the leader's block; test error and the
digit-1 error ("attack rate", client.py:163-172) plus the 1->7 rate (share of digit-1 test rows
predicted as 7, which isolates the attack from the class's base error).

    python scripts/poison_diag.py --config mnist100_po30_ep1 --seeds 3 --rounds 100 -o out.json
    python scripts/poison_diag.py --all --seeds 3 -o profiles/poison_r2.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics as st
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

CONFIGS = {
    # MNIST 1->7 label flip; the reference's eval: 100 peers, -po 0.30 -ns 70 -ep 1.0
    "mnist100_clean_ep1": dict(num_nodes=100, epsilon=1.0),
    "mnist100_po30_ep1": dict(num_nodes=100, poisoning=0.3, epsilon=1.0),
    "mnist100_po30_ep1_5v": dict(num_nodes=100, poisoning=0.3, epsilon=1.0, num_verifiers=5),
    "mnist100_po30_ep1_shared": dict(num_nodes=100, poisoning=0.3, epsilon=1.0, ablation="shared_inbox,no_miner_cap"),
    "mnist200_po30_ep1": dict(num_nodes=200, poisoning=0.3, epsilon=1.0),
    "mnist50_po30_ep1": dict(num_nodes=50, poisoning=0.3, epsilon=1.0),
    "mnist50_po30_ep1_5v": dict(num_nodes=50, poisoning=0.3, epsilon=1.0, num_verifiers=5),
    "mnist50_po50_ep1_5v": dict(num_nodes=50, poisoning=0.5, epsilon=1.0, num_verifiers=5),
    "mnist100_po30_nonoise": dict(num_nodes=100, poisoning=0.3, noising=False),
    "mnist100_po30_ep1_indepnoise": dict(num_nodes=100, poisoning=0.3, epsilon=1.0, ablation="noise_independent"),
    "mnist50_po30_ep1_indepnoise": dict(num_nodes=50, poisoning=0.3, epsilon=1.0, ablation="noise_independent"),
    # creditcard label flip, 50 peers (nsdi-eval/credit)
    "credit50_clean": dict(num_nodes=50, dataset="creditcard"),
    "credit50_po30_3v": dict(num_nodes=50, dataset="creditcard", poisoning=0.3),
    "credit50_po30_5v": dict(num_nodes=50, dataset="creditcard", poisoning=0.3, num_verifiers=5),
    "credit50_po50_3v": dict(num_nodes=50, dataset="creditcard", poisoning=0.5),
    "credit50_po50_5v": dict(num_nodes=50, dataset="creditcard", poisoning=0.5, num_verifiers=5),
}


def run(name: str, over: dict, seed: int, rounds: int, burn: int) -> dict:
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    kw = dict(num_nodes=100, dataset="mnist", seed=seed, max_iterations=10**9, phase_sync=False)
    kw.update(over)
    cfg = RunConfig(**kw)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    eng = BiscottiEngine(cfg, Comm(device=dev))
    pois = {p for p in range(cfg.num_nodes) if eng.fsm.is_poisoner(p)}
    task = eng.task
    to7 = None
    if cfg.dataset == "mnist":
        att_X = task.att_X

        def to7():
            Wf = eng.W.float()
            logits = ((att_X - 0.5) / 0.5) @ Wf[:7840].view(10, 784).T + Wf[7840:]
            return float((logits.argmax(1) == 7).float().mean())
    rows = []
    t0 = time.perf_counter()
    for _ in range(rounds):
        r = eng.run_round()
        judged = set().union(*r.inboxes.values()) if r.inboxes else set()
        workers = set(r.approved) | judged
        rows.append({"it": r.iteration, "judged": len(judged), "judged_pois": len(judged & pois),
                     "krum_pois": len(set(r.approved_by_krum) & pois), "krum_acc": len(r.approved_by_krum),
                     "approved": len(r.approved), "approved_pois": len(set(r.approved) & pois),
                     "block": len(r.node_list), "block_pois": len(set(r.node_list) & pois),
                     "err": round(r.test_error, 5), "attack": round(r.attack_rate, 5),
                     "to7": round(to7(), 5) if to7 else None, "workers": len(workers)})
    wall = time.perf_counter() - t0
    eng.close()
    post = rows[burn:]
    seen = sum(x["judged_pois"] for x in post)
    kept = sum(x["block_pois"] for x in post)
    last = rows[-10:]
    return {"config": name, "seed": seed, "poisoners": len(pois), "rounds": rounds, "wall_s": wall,
            "poisoner_updates_judged_after_burnin": seen, "poisoner_updates_in_blocks_after_burnin": kept,
            "rejection_rate_after_burnin": (1 - kept / seen) if seen else None,
            "final_err": rows[-1]["err"], "err_last10": st.mean(x["err"] for x in last),
            "attack_final": rows[-1]["attack"], "attack_last10": st.mean(x["attack"] for x in last),
            "to7_last10": st.mean(x["to7"] for x in last) if to7 else None, "rows": rows}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", default=[])
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--seeds", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--burn", type=int, default=10)
    ap.add_argument("--no-rows", action="store_true", help="summaries only")
    ap.add_argument("-o", "--out", default=None)
    a = ap.parse_args(argv)
    names = list(CONFIGS) if a.all else a.config
    out = {"runs": [], "summary": {}}
    for name in names:
        runs = []
        for s in range(a.seeds):
            r = run(name, CONFIGS[name], s, a.rounds, a.burn)
            if a.no_rows:
                r.pop("rows")
            runs.append(r)
            print(json.dumps({k: v for k, v in r.items() if k != "rows"}), flush=True)
        out["runs"] += runs

        def ms(key):
            v = [r[key] for r in runs if r[key] is not None]
            return [round(st.mean(v), 5), round(st.pstdev(v), 5)] if v else None
        out["summary"][name] = {k: ms(k) for k in ("rejection_rate_after_burnin", "final_err", "err_last10",
                                                   "attack_final", "attack_last10", "to7_last10")}
        out["summary"][name]["overrides"] = CONFIGS[name]
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out["summary"]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
