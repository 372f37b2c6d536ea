"""Per-kernel share of the round's VALU work: total SQ_INSTS_VALU (and wave-cycles) over every dispatch of a
rocprofv3 --pmc run of the bench, grouped by kernel name.

    python scripts/pmc_round_mix.py <dir with */*counter_collection.csv> [rounds]"""
import collections
import csv
import glob
import json
import sys


def main():
    root = sys.argv[1]
    rounds = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", row.get("kernel_name", "")).split("(")[0].replace("void ", "")[:40]
                c = row.get("Counter_Name", row.get("counter_name"))
                tot[kn][c] += float(row.get("Counter_Value", row.get("counter_value", "nan")))
                disp[kn].add(row.get("Dispatch_Id", row.get("dispatch_id")))
    allv = sum(v.get("SQ_INSTS_VALU", 0.0) for v in tot.values()) or 1.0
    out = []
    for kn, cs in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0.0)):
        out.append({"kernel": kn, "dispatches": len(disp[kn]),
                    "valu_share": round(cs.get("SQ_INSTS_VALU", 0.0) / allv, 4),
                    **{c: v / rounds for c, v in cs.items()}})
    json.dump({"per_round_divisor": rounds, "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
