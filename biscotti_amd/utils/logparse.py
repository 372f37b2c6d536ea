"""Peer-log parsers (eval/eval_performance/parseLogs.py:25-296, nsdi-eval/scaleup/baselines.py).

The reference turns timestamped log lines into ``iteration,err,timestamp`` CSVs and reconstructs
per-phase latencies offline.  The engine writes the same ``Train Error is %.5f in Iteration %d``
lines (stderr, Go log format) and, with ``--phase-log``, the role / phase lines the reference's
breakdown pairs (protocol/golog.py), so these parsers work on both: parse_noise / parse_verif /
parse_aggr are parseLogs.py's three pairings (fractional seconds; int_seconds=True truncates like
its get_completion_time).  The JSONL trace (``--trace-file``) carries the phase timer's own numbers
(:func:`phase_breakdown`).

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


# ---------------------------------------------------------------------------- parseLogs.py's phase pairings
_TS = re.compile(r"^\[\w+\] (\d{2}:\d{2}:\d{2}\.\d+) ")


def _ts(line: str) -> float | None:
    m = _TS.match(line)
    return seconds(m.group(1)) if m else None


def _gap(a: float, b: float, int_seconds: bool) -> float:
    d = b - a
    d = d + 86400 if d < 0 else d
    return float(int(d)) if int_seconds else d   # parseLogs.get_completion_time returns timedelta.seconds


def _pairs(lines, start: str, ends: tuple, int_seconds: bool) -> list[float]:
    """For every line containing `start`, the time to the first later line containing any of `ends`
    (parse_noise / parse_verif, eval/eval_performance/parseLogs.py:79-143)."""
    out = []
    for i, ln in enumerate(lines):
        if start not in ln:
            continue
        t0 = _ts(ln)
        for ln2 in lines[i:]:
            if any(e in ln2 for e in ends):
                t1 = _ts(ln2)
                if t0 is not None and t1 is not None:
                    out.append(_gap(t0, t1, int_seconds))
                break
    return out


def parse_noise(lines, int_seconds: bool = False) -> list[float]:
    """Noising time per round: "Getting noise from" -> "Sending update to verifiers" (parseLogs.py:79-107)."""
    return _pairs(lines, "Getting noise from", ("Sending update to verifiers",), int_seconds)


def parse_verif(lines, int_seconds: bool = False) -> list[float]:
    """Verification time per round: "Sending update to verifiers" -> "Sending update to miners" or "Couldn't get
    enough signatures" (parseLogs.py:115-143)."""
    return _pairs(lines, "Sending update to verifiers", ("Couldn't get enough signatures", "Sending update to miners"),
                  int_seconds)


_MINERS = re.compile(r"Miners are \[([0-9 ]*)\]")


def parse_aggr(lines, leader_lines=None, int_seconds: bool = False) -> list[tuple[int, float | None]]:
    """Secure-aggregation time per round (parseLogs.py:146-194): iteration k is the k-th "Miners are" line of
    the peer's log; its leader (the highest miner id) logs "Got share for k, I am at k" -> "Sending block of
    iteration: k".  leader_lines(leader) -> that peer's log lines (default: the same lines, as the engine
    writes the leader's lines into the rank's own log)."""
    out = []
    k = 0
    for ln in lines:
        m = _MINERS.search(ln)
        if not m:
            continue
        miners = [int(x) for x in m.group(1).split()]
        ll = leader_lines(max(miners)) if leader_lines is not None and miners else lines
        got = _pairs(ll, f"Got share for {k}, I am at {k}", (f"Sending block of iteration: {k}",), int_seconds)
        out.append((k, got[0] if got else None))
        k += 1
    return out


def phase_columns(lines, leader_lines=None, int_seconds: bool = False) -> dict:
    """The breakdown parseLogs.py's main computes per run: mean noising, verification and sec-agg seconds over
    the rounds that logged them, and the mean round time from the Train Error rows."""
    import statistics as st

    def mean(v):
        v = [x for x in v if x is not None]
        return st.mean(v) if v else float("nan")
    rows = parse_train_errors(lines)
    return {"noising": mean(parse_noise(lines, int_seconds)), "verification": mean(parse_verif(lines, int_seconds)),
            "sec_agg": mean([t for _, t in parse_aggr(lines, leader_lines, int_seconds)]),
            "total": sec_per_round(rows), "rounds": len(rows)}


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
    ap.add_argument("--phases", action="store_true",
                    help="parseLogs.py's noising / verification / sec-agg breakdown (needs --phase-log lines)")
    a = ap.parse_args(argv)
    with open(a.log) as f:
        lines = f.readlines()
    rows = parse_train_errors(lines)
    att = parse_attack_rates(lines)
    if a.csv:
        with open(a.csv, "w") as f:
            for it, err, ts in rows:
                f.write(f"{it},{err:.5f},{att.get(it, float('nan')):.5f},{ts}\n")
    out = {"rounds": len(rows), "sec_per_round": sec_per_round(rows), "final_error": rows[-1][1] if rows else None}
    if a.phases:
        out["phases_s"] = phase_columns(lines)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
