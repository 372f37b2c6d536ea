"""Per-round device timeline from a rocprofv3 --kernel-trace CSV: every kernel of rounds [a, b) with its
queue, start/end relative to the round's first kernel (the round boundary is k_recover_w, the exact
recovery of W), and a per-kernel duration summary (first vs last quarter of the run).

    python scripts/kt_timeline.py gpurun_out/kt/run_kernel_trace.csv [a b]
    python scripts/kt_timeline.py gpurun_out/kt/run_results.db [a b]     (rocprofv3's SQLite output)"""
import collections
import csv
import sys


def load(path):
    if path.endswith(".db"):   # rocprofv3's default rocpd (SQLite) output: its kernels view
        import sqlite3

        con = sqlite3.connect(path)
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Queue_Id": str(q), "Stream_Id": str(st)}
                for n, s, e, q, st in con.execute("select name, start, end, queue_id, stream_id from kernels")]
        try:   # blits and copies (--memory-copy-trace) as pseudo-kernels
            rows += [{"Kernel_Name": f"copy_{k}", "Start_Timestamp": s, "End_Timestamp": e, "Queue_Id": "copy",
                      "Stream_Id": str(st)}
                     for k, s, e, st in con.execute("select name, start, end, stream_id from memory_copies")]
        except sqlite3.Error:
            pass
    else:
        rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["d"] = (r["e"] - r["s"]) / 1e3
        r["n"] = r["Kernel_Name"].split("(")[0].replace("void ", "")[:32]
    rows.sort(key=lambda r: r["s"])
    return rows


def main():
    rows = load(sys.argv[1])
    a, b = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (50, 52)
    rec = [r for r in rows if r["n"] == "k_recover_w"]
    by = collections.defaultdict(list)
    for r in rows:
        by[r["n"]].append(r["d"])
    print(f"{'kernel':32s} {'n':>5s} {'total ms':>9s} {'mean us':>8s} {'1st 25%':>8s} {'last 25%':>8s}")
    for n, ds in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:16]:
        q = max(1, len(ds) // 4)
        print(f"{n:32s} {len(ds):5d} {sum(ds) / 1e3:9.2f} {sum(ds) / len(ds):8.1f} {sum(ds[:q]) / q:8.1f} "
              f"{sum(ds[-q:]) / q:8.1f}")
    gaps = [(rec[i + 1]["e"] - rec[i]["e"]) / 1e3 for i in range(len(rec) - 1)]
    print("recovery-to-recovery us:", [round(g) for g in gaps])
    # per round: every share MSM launched inside it (queue, start after the previous recovery, duration)
    print("round  wall  share MSMs (queue:start+duration us)")
    for i in range(len(rec) - 1):
        t0, t1 = rec[i]["e"], rec[i + 1]["e"]
        ms = [r for r in rows if r["n"].startswith("k_shares_msm") and t0 <= r["s"] < t1]
        print(f"{i + 1:5d} {(t1 - t0) / 1e3:6.0f}  " + " ".join(f"q{r['Queue_Id']}:{(r['s'] - t0) / 1e3:.0f}+{r['d']:.0f}"
                                                       for r in ms))
    for i in range(a, min(b, len(rec) - 1)):
        t0 = rec[i]["e"]
        print(f"--- round {i + 1} (t=0: end of recovery {i}), next recovery ends at {(rec[i + 1]['e'] - t0) / 1e3:.0f} us")
        for r in rows:
            if t0 - 200_000 <= r["s"] < rec[i + 1]["e"] or (r["s"] < t0 < r["e"]):
                print(f"  q{r['Queue_Id']:>2s} {r['n']:32s} {(r['s'] - t0) / 1e3:8.0f} {(r['e'] - t0) / 1e3:8.0f} "
                      f"{r['d']:7.0f}")


if __name__ == "__main__":
    main()
