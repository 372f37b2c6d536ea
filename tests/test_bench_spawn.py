"""bench.py's own multi-rank launch (the driver's `python bench.py --gpus N` contract without torchrun):
the parent spawns N ranks under torch.distributed.run, rank 0 prints ONE JSON line with the whole job's
numbers (the MAX of the ranks' elapsed times) and every rank's host-cost breakdown.  CPU / gloo here."""
import json
import os
import subprocess
import sys

from test_distributed_cpu import ROOT


def test_bench_spawns_ranks_and_reports_them():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--config", "credit4", "--steps", "2",
                        "--warmup", "1", "--rounds", "3"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"].startswith("dp2")
    assert out["chain_valid"] is True
    ranks = out["per_rank"]
    assert [p["rank"] for p in ranks] == [0, 1]
    # value = the slowest rank's elapsed time / steps
    assert abs(out["value"] - max(p["elapsed_s"] for p in ranks) / 2) < 1e-9
    for p in ranks:
        assert p["host_cpu_ms_per_round"] > 0 and p["thread_cpu_ms_per_round"]
        assert p["phase_ms_per_round"] and "engine_stats" in p
