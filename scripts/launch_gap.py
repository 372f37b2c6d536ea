"""When each kernel of interest was launched by the host and when it started on the device, relative to the end
of the previous recovery (k_recover_w), from a rocprofv3 --hip-trace --kernel-trace database (rocpd SQLite):

    python scripts/launch_gap.py gpurun_out/X/ht_TAG/run_results.db [kernel substrings, comma-separated]

Kernels and HIP API calls are matched through their correlation id.  Prints the schema when that fails."""
import sqlite3
import sys


def cols(con, t):
    return [r[1] for r in con.execute(f"pragma table_info({t})")]


def main(path: str, names: str = "k_shares_msm_ka,k_krum_vote,k_recover_w") -> None:
    con = sqlite3.connect(path)
    kc, rc = cols(con, "kernels"), cols(con, "regions")
    print("kernels:", kc)
    print("regions:", rc)
    for t in ("kernels", "regions"):
        for row in con.execute(f"select * from {t} limit 2"):
            print(t, row)
    # rocprofv3 7.x: a kernel's stack_id is the id of the HIP API region that dispatched it
    key = next((k for k in ("stack_id", "correlation_id") if k in kc and k in rc), None)
    if key is None:
        return
    launch, lname = {}, {}
    for c, st, nm in con.execute(f"select {key}, start, name from regions where {key} != 0"):
        launch[c], lname[c] = st, nm
    print(len(launch), "API regions with an id; launching APIs:",
          sorted({lname.get(c) for _, _, _, c in con.execute(f"select name, start, end, {key} from kernels")
                  if c in lname})[:8])
    ks = sorted(con.execute(f"select name, start, end, {key} from kernels"), key=lambda r: r[1])
    want = names.split(",")
    last_rec = None
    rows = []
    for name, s, e, c in ks:
        n = name.split("(")[0]
        if "k_recover_w" in n:
            if last_rec is not None:
                rows.append(("--- recovery ends", 0, 0, 0))
            last_rec = e
        if last_rec is None or not any(w in n for w in want):
            continue
        h = launch.get(c) if c else None
        rows.append((n, (h - last_rec) / 1e3 if h is not None else float("nan"), (s - last_rec) / 1e3,
                     (e - last_rec) / 1e3))
    rows = rows[len(rows) // 2:][:60]   # steady state
    print(f"{'kernel':28s} {'host launch':>12s} {'start':>8s} {'end':>8s}   (us after the previous recovery's end)")
    for n, h, s, e in rows:
        print(f"{n[:28]:28s} {h:12.1f} {s:8.1f} {e:8.1f}" if h or s else n)


if __name__ == "__main__":
    main(*sys.argv[1:])
