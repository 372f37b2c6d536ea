"""Peer-log parsers (eval/eval_performance/parseLogs.py:25-296, nsdi-eval/scaleup/baselines.py).

The reference turns timestamped log lines into ``iteration,err,timestamp`` CSVs and reconstructs
per-phase latencies offline.  The engine writes the same ``Train Error is %.5f in Iteration %d``
lines (stderr, Go log format), so these parsers work on both; the JSONL trace (``--trace-file``)
carries exact per-phase times and is summarised by :func:`phase_breakdown`.

    python -m biscotti_amd.utils.logparse LOGFILE [--csv out.csv]
"""
from __future__ import annotations

import json
import re
import sys

LINE = re.compile(r"(\d{2}):(\d{2}):(\d{2})\.(\d+) \S+: (\d+):Train Error is ([0-9.]+) in Iteration (-?\d+)")
ATTACK = re.compile(r"(\d+):Attack Rate is ([0-9.]+) in Iteration (-?\d+)")


def parse_train_errors(lines) -> list[tuple[int, float, str]]:
    """[(iteration, error, 'HH:MM:SS.micro')] -- the parseLogs.py CSV rows, first peer reporting."""
    seen, rows = set(), []
    for ln in lines:
        m = LINE.search(ln)
        if not m:
            continue
        it = int(m.group(7))
        if it in seen:
            continue
        seen.add(it)
        rows.append((it, float(m.group(6)), f"{m.group(1)}:{m.group(2)}:{m.group(3)}.{m.group(4)}"))
    return rows


def parse_attack_rates(lines) -> dict[int, float]:
    out = {}
    for ln in lines:
        m = ATTACK.search(ln)
        if m:
            out.setdefault(int(m.group(3)), float(m.group(2)))
    return out


def seconds(ts: str) -> float:
    h, m, s = ts.split(":")
    return int(h) * 3600 + int(m) * 60 + float(s)


def sec_per_round(rows) -> float:
    """BASELINE.md's definition: mean gap between consecutive Train Error rows (midnight-safe)."""
    if len(rows) < 2:
        return float("nan")
    gaps = []
    for a, b in zip(rows, rows[1:]):
        d = seconds(b[2]) - seconds(a[2])
        gaps.append(d + 86400 if d < 0 else d)
    return sum(gaps) / len(gaps)


def phase_breakdown(trace_path: str) -> dict:
    """Mean seconds per round of every phase recorded in a JSONL trace."""
    tot, n = {}, 0
    with open(trace_path) as f:
        for ln in f:
            rec = json.loads(ln)
            n += 1
            for k, v in rec.items():
                if k.startswith("t_"):
                    tot[k[2:]] = tot.get(k[2:], 0.0) + v
    return {k: v / max(n, 1) for k, v in sorted(tot.items())} | {"rounds": n}


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="biscotti_amd.utils.logparse")
    ap.add_argument("log")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args(argv)
    with open(a.log) as f:
        lines = f.readlines()
    rows = parse_train_errors(lines)
    att = parse_attack_rates(lines)
    if a.csv:
        with open(a.csv, "w") as f:
            for it, err, ts in rows:
                f.write(f"{it},{err:.5f},{att.get(it, float('nan')):.5f},{ts}\n")
    print(json.dumps({"rounds": len(rows), "sec_per_round": sec_per_round(rows),
                      "final_error": rows[-1][1] if rows else None}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
