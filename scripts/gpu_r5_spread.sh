# Round-5: the spread of the driver-style headline on one box (5 runs of bench.py --steps 20 --warmup 5).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5spread; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b1_s$i.txt 2>&1 || { echo "FAIL $i"; tail -5 $O/b1_s$i.txt; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/b1_s$i.txt') if l.startswith('{')][-1]); w=sorted(d['round_wall_ms'])
print('s$i', round(d['ms_per_step'],3), 'med', round(w[len(w)//2],3), 'max', round(w[-1],3), 'drain', round(d['drain_ms'],2), flush=True)"
done
