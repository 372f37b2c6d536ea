# Round-5 closing evidence on the working tree: the box's CPU (model, AVX-512 IFMA), the whole GPU test suite, the
# 5-seed poisoning run (docs/ROBUSTNESS.md), then driver-style bench runs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5final; mkdir -p $O
{ grep -m1 'model name' /proc/cpuinfo; grep -c processor /proc/cpuinfo; grep -o -m1 -w 'avx512ifma' /proc/cpuinfo || echo no-ifma; } > $O/cpu.txt
cat $O/cpu.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 \
    || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error" $O/gputests.txt | tail -20; exit 1; }
  echo "gpu tests passed: $(grep -c PASSED $O/gputests.txt)"
fi
if [ -z "$SKIP_POISON" ]; then
  timeout -k 10 600 python scripts/poison_diag.py --config mnist100_po30_ep1 --seeds 5 --rounds 100 \
    -o $O/poison30_100_5seeds.json > $O/poison.log 2>&1 || { echo "POISON FAILED"; tail -5 $O/poison.log; exit 1; }
  python -c "
import json,statistics as st; d=json.load(open('$O/poison30_100_5seeds.json'))
runs=d['runs']; a=[r['attack_last10'] for r in runs]; e=[r['err_last10'] for r in runs]; rj=[r['rejection_rate_after_burnin'] for r in runs]
print('attack_last10', [round(x,3) for x in a], 'mean', round(st.mean(a),3), 'sd', round(st.pstdev(a),3), 'err', round(st.mean(e),3), 'rej', round(st.mean(rj),3))"
fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b1_s$i.txt 2>&1 || { echo "BENCH FAILED"; tail -5 $O/b1_s$i.txt; exit 1; }
  grep '^{' $O/b1_s$i.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b1', $i, round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'max', d.get('round_wall_max_ms'))"
done
# the AVX-512 IFMA VRF outputs against the scalar path, same box (BISCOTTI_VRF_SCALAR), and the host timeline
for i in 1 2; do
  BISCOTTI_VRF_SCALAR=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b1_scalar_s$i.txt 2>&1 || { echo "BENCH FAILED"; tail -5 $O/b1_scalar_s$i.txt; exit 1; }
  grep '^{' $O/b1_scalar_s$i.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('scalar', $i, round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'host_cpu', d.get('host_cpu_ms_per_round'))"
done
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true \
  --wrap _early_vrf_submit,_spec_head_launch,_prepare_next_in_wait,_open_round,_select_noisers,_launch_krum,_resolve_evals,native.spec_msm,native.after_select,_finish_secagg,_secure_aggregation,_verification \
  > $O/host_tl.json 2> $O/host_tl.err || { echo "HOST TL FAILED"; tail -20 $O/host_tl.err; exit 1; }
python -c "
import json; d=json.load(open('$O/host_tl.json'))
for r in d[:2]: print('wall', r['wall_us'], r['jobs (kind, submit_us, queued_us, run_us)'])"
