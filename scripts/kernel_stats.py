"""Per-kernel statistics from a rocprofv3 database (rocpd SQLite, the default output of --kernel-trace):

    python scripts/kernel_stats.py gpurun_out/X/prof/run_results.db [out.csv]

Kernel, calls, total ms, mean / median / min / max us -- rocprofv3 --stats' kernel table, from the trace itself."""
import csv
import sqlite3
import sys
from collections import defaultdict


def main(path: str, out: str | None = None) -> None:
    con = sqlite3.connect(path)
    by = defaultdict(list)
    for name, s, e in con.execute("select name, start, end from kernels"):
        by[name.split("(")[0].replace("void ", "")].append((e - s) / 1e3)
    rows = []
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        o = sorted(v)
        rows.append([n, len(v), round(sum(v) / 1e3, 3), round(sum(v) / len(v), 1), round(o[len(o) // 2], 1),
                     round(o[0], 1), round(o[-1], 1)])
    head = ["kernel", "calls", "total_ms", "mean_us", "median_us", "min_us", "max_us"]
    if out:
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(head)
            w.writerows(rows)
    print(f"{head[0]:34s} {head[1]:>6s} {head[2]:>9s} {head[3]:>8s} {head[4]:>9s} {head[5]:>7s} {head[6]:>8s}")
    for r in rows[:30]:
        print(f"{r[0][:34]:34s} {r[1]:6d} {r[2]:9.3f} {r[3]:8.1f} {r[4]:9.1f} {r[5]:7.1f} {r[6]:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
