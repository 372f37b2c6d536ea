# Round-5 fence removal (k_gram_pairs split-K reduce as a second kernel, no per-wave / per-block agent or system
# fences in the evaluation, recovery, audit and commitment sums): the whole GPU suite, the side kernels alone,
# same-box A/B against ab_base (HEAD before it), a kernel timeline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5fence; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 \
  || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error" $O/gputests.txt | tail -20; exit 1; }
echo "gpu tests passed: $(grep -c PASSED $O/gputests.txt)"
timeout -k 10 300 python scripts/kernel_alone.py --reps 20 > $O/alone.txt 2> $O/alone.err || { echo "ALONE FAILED"; tail -5 $O/alone.err; exit 1; }
cat $O/alone.txt
run() {  # variant tag steps warmup
  v=$1; t=$2; st=$3; w=$4
  case $v in base) D=$R/ab_base;; *) D=$R;; esac
  (cd $D && timeout -k 10 300 python bench.py --steps $st --warmup $w) > $O/${v}_$t.txt 2>&1 || { echo "FAIL $v $t"; tail -5 $O/${v}_$t.txt; return 1; }
  grep '^{' $O/${v}_$t.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$v $t', round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'max', d.get('round_wall_max_ms'), 'rb', round(p.get('recover.readback',0),3), flush=True)"
}
for i in 1 2 3; do
  if [ $i = 2 ]; then run new s$i 20 5 || exit 1; run base s$i 20 5 || exit 1
  else run base s$i 20 5 || exit 1; run new s$i 20 5 || exit 1; fi
done
run new long 200 10 || exit 1
run base long 200 10 || exit 1
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
sed -n 1,20p $O/kt_timeline.txt
