"""Per-round GPU timeline from a rocprofv3 kernel trace (CSV: *_kernel_trace.csv).

    python scripts/rocprof_timeline.py TRACE.csv [--rounds 3] [--skip 20]

Rounds are delimited by the local-step kernel (one launch per round, queued at the previous
block's commit).  For `--rounds` consecutive rounds after `--skip` it prints every kernel's start
offset and duration (us) relative to the round's local step, its queue/stream, and per round the
union of busy time (how much of the round any kernel was running) -- the idle gaps are host-bound.
"""
import argparse
import csv
import json
import sys


def load(path):
    with open(path, newline="") as f:
        rows = list(csv.DictReader(f))
    if not rows:
        return []
    keys = rows[0].keys()
    kname = next(k for k in keys if k.lower() in ("kernel_name", "name"))
    ks = next(k for k in keys if "start" in k.lower())
    ke = next(k for k in keys if "end" in k.lower())
    kq = next((k for k in keys if k.lower() in ("stream_id", "queue_id")), None)
    out = [(int(r[ks]), int(r[ke]), r[kname].split("(")[0][:60], r.get(kq, "") if kq else "") for r in rows]
    out.sort()
    return out


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--skip", type=int, default=20)
    ap.add_argument("--marker", default="k_softmax_step")
    a = ap.parse_args()
    ks = load(a.trace)
    marks = [s for s, e, n, q in ks if n.startswith(a.marker)]
    res = {"rounds": []}
    walls, busys = [], []
    for i in range(a.skip, min(len(marks) - 1, a.skip + 50)):
        t0, t1 = marks[i], marks[i + 1]
        inside = [(max(s, t0), min(e, t1)) for s, e, n, q in ks if e > t0 and s < t1]
        walls.append(t1 - t0)
        busys.append(union(inside))
    for i in range(a.skip, min(len(marks) - 1, a.skip + a.rounds)):
        t0, t1 = marks[i], marks[i + 1]
        ev = [{"k": n, "q": q, "t_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1)}
              for s, e, n, q in ks if t0 - 2_000_000 < s < t1]
        res["rounds"].append({"wall_us": (t1 - t0) / 1e3, "busy_us": union(
            [(max(s, t0), min(e, t1)) for s, e, n, q in ks if e > t0 and s < t1]) / 1e3, "kernels": ev})
    if walls:
        res["mean_wall_us"] = sum(walls) / len(walls) / 1e3
        res["mean_busy_us"] = sum(busys) / len(busys) / 1e3
        res["n_rounds_averaged"] = len(walls)
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
