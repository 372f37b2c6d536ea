"""Which hardware queue / stream each kernel ran on, from a rocprofv3 kernel_trace.csv:
kernel name -> {queue id: launches}.  Shows whether two streams shared a hardware queue."""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = rows[0].keys() if rows else []
cols = [k for k in keys if k.lower() in ("queue_id", "stream_id")]
out = collections.defaultdict(lambda: collections.Counter())
for r in rows:
    name = r.get("Kernel_Name", "")[:40]
    out[name][tuple(r[c] for c in cols)] += 1
print(json.dumps({"columns": cols, "kernels": {k: {str(q): n for q, n in v.items()} for k, v in out.items()}}, indent=1))
