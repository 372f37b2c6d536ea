# Round-5 recovery on the critical chain: k_recover_w's row sums split over the block (RW_CPB 2) and the recovery
# queued behind the speculative MSM on its own stream.  Tests, then same-box A/B against ab_base (HEAD without
# the two), driver-style x3 alternating + 200 rounds, then a kernel timeline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/${TAG:-r5rec}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_engine_paths.py -x -v --timeout 300 \
  --timeout-method thread -k "recover or early_front or pre_gram or engine_rounds or horizon or exact or kzg or noise_aware or committee" > $O/tests.txt 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.txt | tail -20; exit 1; }
echo "tests passed: $(grep -c PASSED $O/tests.txt)"
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
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true \
  --wrap _early_vrf_submit,_spec_head_launch,_prepare_next_in_wait,_open_round,_select_noisers,_launch_krum,_resolve_evals,native.spec_msm,native.after_select,_finish_secagg,_secure_aggregation,_round_front,_noise_ids_np,_krum_static,_on_accept,_spec_aggregate_native,_live_mask,_vrf_key_rows,_finish_verification \
  > $O/host_tl.json 2> $O/host_tl.err || { echo "HOST TL FAILED"; tail -20 $O/host_tl.err; exit 1; }
