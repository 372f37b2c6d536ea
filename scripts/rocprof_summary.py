"""Summarise a rocprofv3 --kernel-trace database into a small JSON (per-kernel totals)."""
import json
import sqlite3
import sys


def summarize(db_path: str, top: int = 25, per_round: int | None = None) -> dict:
    db = sqlite3.connect(db_path)
    cols = [r[1] for r in db.execute("PRAGMA table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"SELECT {name}, COUNT(*), SUM(end - start), AVG(end - start), MAX(end - start) "
                      f"FROM kernels GROUP BY {name} ORDER BY SUM(end - start) DESC").fetchall()
    total = sum(r[2] for r in rows)
    out = {"total_kernel_ms": total / 1e6, "kernels": []}
    for n, c, s, a, m in rows[:top]:
        e = {"name": n[:120], "calls": c, "total_ms": s / 1e6, "avg_us": a / 1e3, "max_us": m / 1e3,
             "pct": 100.0 * s / total}
        if per_round:
            e["ms_per_round"] = s / 1e6 / per_round
        out["kernels"].append(e)
    return out


if __name__ == "__main__":
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else None
    print(json.dumps(summarize(sys.argv[1], per_round=rounds), indent=1))
