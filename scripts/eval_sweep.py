"""Evaluation drivers (eval/*/runEval.sh, nsdi-eval/*): parameter sweeps over bench.py runs.

    python scripts/eval_sweep.py SWEEP --out results.jsonl [--steps 100]

Sweeps (reference driver in brackets):
  scaleup     peers 40/60/80/100, Biscotti and FedSys          [nsdi-eval/scaleup, eval_FedSys_scale]
  increments  secure-agg / verification / noising switched off  [nsdi-eval/increments]
  committee   noisers, verifiers, aggregators in {3, 5, 10}     [eval_vrf_scale, nsdi-eval/nvm-scale]
  poison      poisoner fraction x verifiers (Krum)              [eval_poison, eval_poison_nsamples]
  epsilon     DP epsilon sweep                                   [eval_noise_krum, eval_privacy_utility_krum]
  churn       fraction of peers offline per round                [eval_FT, nsdi-eval/churn]
Each point is one child process; a signal/abort/timeout stops the sweep (GPU pool rules).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SWEEPS = {
    "scaleup": [([f"--peers={n}"], f"biscotti_{n}") for n in (40, 60, 80, 100)]
    + [(["--config=fedsys", f"--peers={n}"], f"fedsys_{n}") for n in (40, 60, 80, 100)],
    "increments": [(["--config=" + c], c) for c in ("headline", "secagg_off", "verification_off", "noising_off")],
    "committee": [([f"--set=num_{r}={k}"], f"{r}_{k}") for r in ("noisers", "verifiers", "miners")
                  for k in (3, 5, 10)],
    "poison": [(["--set=poisoning=%s" % po, f"--set=num_verifiers={nv}"], f"po{po}_nv{nv}")
               for po in (0.1, 0.3, 0.5) for nv in (3, 5)],
    "epsilon": [([f"--set=epsilon={e}"], f"eps{e}") for e in (0.5, 1.0, 2.0, 5.0)],
    "churn": [([f"--set=churn={c}"], f"churn{c}") for c in (0.0, 0.1, 0.2, 0.3)],
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("sweep", choices=sorted(SWEEPS))
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args()
    with open(a.out, "a") as f:
        for args, tag in SWEEPS[a.sweep]:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup",
                   str(a.warmup), *args]
            try:
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=ROOT)
            except subprocess.TimeoutExpired:
                f.write(json.dumps({"sweep": a.sweep, "point": tag, "error": "timeout"}) + "\n")
                return 124
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("{")), None)
            rec = json.loads(line) if (p.returncode == 0 and line) else {"rc": p.returncode,
                                                                       "stderr_tail": p.stderr[-1500:]}
            rec.update(sweep=a.sweep, point=tag)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(tag, p.returncode, rec.get("ms_per_step"), rec.get("final_test_acc"), flush=True)
            if p.returncode < 0 or p.returncode in (124, 134, 137, 139):
                return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
