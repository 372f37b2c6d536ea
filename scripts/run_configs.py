"""Run bench.py over several BASELINE presets, one child process each, and collect the JSON lines.

    python scripts/run_configs.py --out gpurun_out/configs.jsonl --steps 50 fedsys poison30 ...

Stops at the first child killed by a signal, aborted or timed out (nothing more is started on the
GPU after that); an ordinary Python error in one preset is recorded and the next preset runs."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rc_all = 0
    with open(a.out, "a") as f:
        for c in a.configs:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", c, "--steps", str(a.steps),
                   "--warmup", str(a.warmup)]
            try:
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=ROOT)
            except subprocess.TimeoutExpired:
                f.write(json.dumps({"config": c, "error": "timeout"}) + "\n")
                return 124
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("{")), None)
            if p.returncode == 0 and line:
                f.write(line + "\n")
            else:
                f.write(json.dumps({"config": c, "rc": p.returncode, "stderr_tail": p.stderr[-2000:]}) + "\n")
                rc_all = 1
            f.flush()
            print(c, p.returncode, flush=True)
            if p.returncode < 0 or p.returncode in (124, 134, 137, 139):
                return p.returncode if p.returncode > 0 else 128 - p.returncode
    return rc_all


if __name__ == "__main__":
    sys.exit(main())
