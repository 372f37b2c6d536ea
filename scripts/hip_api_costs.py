"""Host cost of the HIP runtime calls of a run, from a rocprofv3 --hip-trace database (rocpd SQLite):

    python scripts/hip_api_costs.py gpurun_out/X/ht_TAG/run_results.db [rounds]

Per API name on the busiest thread (the round's Python thread), over the last 60 % of its calls (the steady
state): calls, mean / median / p90 and total host microseconds, and the per-round share when the number of rounds
in that window is given."""
import sqlite3
import sys
from collections import Counter, defaultdict


def main(path: str, rounds: int = 0) -> None:
    con = sqlite3.connect(path)
    rows = list(con.execute("select tid, name, start, end from regions where category like '%HIP%'"))
    if not rows:
        print("no HIP API regions (run rocprofv3 with --hip-trace)")
        return
    main_tid = Counter(r[0] for r in rows).most_common(1)[0][0]
    mine = sorted((s, e, name) for tid, name, s, e in rows if tid == main_tid)
    # the steady state: between the ends of the last rounds' recoveries when their kernels are in the trace
    # (rounds = the recoveries in the window), else the last 60 % of the thread's calls
    rec = sorted(e for (e,) in con.execute("select end from kernels where name like 'k_recover_w%'"))
    if len(rec) >= 12:
        lo, hi = rec[-11], rec[-1]
        mine = [m for m in mine if lo <= m[0] < hi]
        rounds = 10
        print(f"window: the last 10 rounds (recovery ends {lo} .. {hi})")
    else:
        mine = mine[int(0.4 * len(mine)):]
    by = defaultdict(list)
    for s, e, name in mine:
        by[name].append((e - s) / 1e3)
    tot = sum(sum(v) for v in by.values())
    print(f"thread {main_tid}: {sum(len(v) for v in by.values())} calls, {tot / 1e3:.1f} ms in HIP calls")
    print(f"{'api':40s} {'calls':>7s} {'mean us':>8s} {'p50 us':>7s} {'p90 us':>7s} {'total ms':>9s}"
          + (f" {'us/round':>9s}" if rounds else ""))
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:30]:
        o = sorted(v)
        line = (f"{name[:40]:40s} {len(v):7d} {sum(v) / len(v):8.2f} {o[len(o) // 2]:7.2f} {o[int(0.9 * (len(o) - 1))]:7.2f}"
                f" {sum(v) / 1e3:9.2f}")
        if rounds:
            line += f" {sum(v) / rounds:9.1f}"
        print(line)


def by_kernel(path: str) -> None:
    """hipLaunchKernel host cost per launched kernel over the same window (kernels matched through stack_id)."""
    con = sqlite3.connect(path)
    rec = sorted(e for (e,) in con.execute("select end from kernels where name like 'k_recover_w%'"))
    if len(rec) < 12:
        return
    lo, hi = rec[-11], rec[-1]
    kname = {sid: n.split("(")[0] for n, sid in con.execute("select name, stack_id from kernels where stack_id != 0")}
    by = defaultdict(list)
    for sid, s, e in con.execute("select stack_id, start, end from regions where name = 'hipLaunchKernel'"):
        if lo <= s < hi and sid in kname:
            by[kname[sid]].append((e - s) / 1e3)
    print(f"\n{'launched kernel':40s} {'calls':>7s} {'mean us':>8s} {'p50 us':>7s} {'us/round':>9s}")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        o = sorted(v)
        print(f"{n[:40]:40s} {len(v):7d} {sum(v) / len(v):8.2f} {o[len(o) // 2]:7.2f} {sum(v) / 10:9.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    by_kernel(sys.argv[1])
