# Round-5 same-box A/B of the round's wave priorities: base = ab_base (HEAD: step and Gram at 1, both share MSMs at
# 2), p1 = ab_p1 (step and Gram at 3), p2 = working tree (p1 + the pre-step's commitment MSM at 1); driver-style
# x3 each in rotating order, one 200-round run each, then a kernel timeline of p2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5prio; mkdir -p $O
run() {  # variant tag steps warmup
  v=$1; t=$2; st=$3; w=$4
  case $v in base) D=$R/ab_base;; p1) D=$R/ab_p1;; *) D=$R;; esac
  (cd $D && timeout -k 10 300 python bench.py --steps $st --warmup $w) > $O/${v}_$t.txt 2>&1 || { echo "FAIL $v $t"; tail -5 $O/${v}_$t.txt; return 1; }
  grep '^{' $O/${v}_$t.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$v $t', round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'rb', round(p['recover.readback'],3), 'kw', round(p['verify.krum_wait'],3), 'vj', round(p.get('vrf_join',0),3), 'audit', round(p.get('recover.audit',0),3), flush=True)"
}
for i in 1 2 3; do
  case $i in 1) order="base p1 p2";; 2) order="p2 base p1";; 3) order="p1 p2 base";; esac
  for v in $order; do run $v s$i 20 5 || exit 1; done
done
for v in base p1 p2; do run $v long 200 10 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt" -o run -- python3 "$R/bench.py" --steps 60 --warmup 5 \
  > "$R/$O/kt_bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/$O/kt_bench.txt"; exit 1; }
cd "$R"
T=$(find $O/kt -name '*kernel_trace.csv' | head -1)
S=$(find $O/kt -name '*kernel_stats.csv' | head -1)
cp "$S" $O/kernel_stats.csv
python scripts/kt_timeline.py "$T" 40 43 > $O/kt_timeline.txt
gzip -c "$T" > $O/kernel_trace.csv.gz
rm -rf $O/kt
head -22 $O/kt_timeline.txt
