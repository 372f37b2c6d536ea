"""Summarise rocprofv3 --pmc CSVs: per kernel name (substring match), the median over dispatches of
every counter, plus derived VALU issue share and HBM bytes.

    python scripts/pmc_summary.py <dir with */*counter_collection.csv> KERNEL [KERNEL ...]
"""
import csv
import glob
import json
import statistics as st
import sys


def main():
    root, names = sys.argv[1], sys.argv[2:]
    per = {n: {} for n in names}
    for path in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", row.get("kernel_name", ""))
                for n in names:
                    if n in kn:
                        cid = row.get("Dispatch_Id", row.get("dispatch_id"))
                        c = row.get("Counter_Name", row.get("counter_name"))
                        v = float(row.get("Counter_Value", row.get("counter_value", "nan")))
                        per[n].setdefault(c, {}).setdefault(cid, 0.0)
                        per[n][c][cid] += v   # summed over the per-XCD/SE instances of a dispatch
    out = {}
    for n, cs in per.items():
        med = {c: st.median(list(v.values())) for c, v in cs.items() if v}
        if not med:
            continue
        d = dict(med)
        if "SQ_ACTIVE_INST_VALU" in med and "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"]:
            d["valu_active_share_of_wave_cycles"] = med["SQ_ACTIVE_INST_VALU"] / med["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_ANY" in med and "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"]:
            d["wait_any_share"] = med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"]
            d["wait_inst_any_share"] = med.get("SQ_WAIT_INST_ANY", 0) / med["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in med:
            d["fetch_bytes"] = med["FETCH_SIZE"] * 1024
        out[n] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
