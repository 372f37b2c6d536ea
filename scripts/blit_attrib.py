"""Which runtime blits (__amd_rocclr_copyBuffer / fillBuffer kernels) a round pays, and which HIP API call queued
each: joins a rocprofv3 kernel trace with its HIP runtime trace on Correlation_Id.  Per (API call, stream, grid
size): launches per round and mean duration; the round boundary is k_recover_w.

    python scripts/blit_attrib.py KERNEL_TRACE.csv HIP_API_TRACE.csv"""
import collections
import csv
import json
import sys

kt = list(csv.DictReader(open(sys.argv[1])))
api = {r["Correlation_Id"]: r for r in csv.DictReader(open(sys.argv[2]))}
rounds = max(1, sum(1 for r in kt if r["Kernel_Name"].startswith("k_recover_w")))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in kt:
    n = r["Kernel_Name"]
    if not n.startswith("__amd_rocclr"):
        continue
    a = api.get(r["Correlation_Id"], {})
    key = (n.split("(")[0], a.get("Function", "?"), r.get("Stream_Id"), r.get("Grid_Size_X"))
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
out = [{"blit": k[0], "api": k[1], "stream": k[2], "grid_x": k[3], "per_round": round(v[0] / rounds, 2),
        "mean_us": round(v[1] / v[0], 1)} for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])]
print(json.dumps({"rounds": rounds, "blits": out}, indent=1))
