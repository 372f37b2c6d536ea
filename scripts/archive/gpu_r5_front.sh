# Round-5 early front (engine._round_front): its chain tests, then same-box A/B against no_early_front
# (driver-style x3 in alternating order + 200 rounds each), then a kernel timeline with it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5front; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_engine_paths.py -x -v --timeout 300 \
  --timeout-method thread -k "early_front or pre_gram or engine_rounds or horizon or exact" > $O/tests.txt 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.txt | tail -20; exit 1; }
echo "tests passed: $(grep -c PASSED $O/tests.txt)"
run() {  # tag steps warmup extra...
  t=$1; st=$2; w=$3; shift 3
  timeout -k 10 300 python bench.py --steps $st --warmup $w "$@" > $O/$t.txt 2>&1 || { echo "FAIL $t"; tail -5 $O/$t.txt; return 1; }
  grep '^{' $O/$t.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$t', round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'max', d.get('round_wall_max_ms'), 'rb', round(p.get('recover.readback',0),3), 'kw', round(p.get('verify.krum_wait',0),3), 'fronts', d['engine_stats'].get('early_fronts'), flush=True)"
}
for i in 1 2 3; do
  if [ $i = 2 ]; then run off_s$i 20 5 --set ablation=no_early_front || exit 1; run on_s$i 20 5 || exit 1
  else run on_s$i 20 5 || exit 1; run off_s$i 20 5 --set ablation=no_early_front || exit 1; fi
done
run on_long 200 10 || exit 1
run off_long 200 10 --set ablation=no_early_front || exit 1
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
