# One host-optimisation iteration on the GPU: engine/pipeline GPU tests, the wrapped host timeline
# (bench settings: lazy_eval), then REPS driver-style benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
TAG=${TAG:-it}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_engine_paths.py tests/test_gpu_bn256.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.txt
fi
W=_spec_head_launch,_queue_pre_step,_aggregate_native,_krum_static,_select_noisers,_noise_ids_np,_launch_krum,_spec_aggregate,_early_vrf_submit,_resolve_evals,_log_round,task.evaluate_async,crypto.commitments_async,crypto.shares_async,_gram_rows,_open_round,_prepare_next_in_wait,_finish_secagg,_secure_aggregation,_verification
timeout -k 10 200 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true --wrap $W > gpurun_out/${TAG}_tl.json 2> gpurun_out/${TAG}_tl.err || { echo "TL FAILED"; tail -5 gpurun_out/${TAG}_tl.err; exit 1; }
python - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_tl.json"))
print("timeline walls", [r["wall_us"] for r in d])
PY
for rep in $(seq 1 ${REPS:-3}); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_b$rep.txt 2>&1 || { echo "BENCH FAILED"; tail -5 gpurun_out/${TAG}_b$rep.txt; exit 1; }
  grep '^{' gpurun_out/${TAG}_b$rep.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('short', round(d['ms_per_step'],3), 'drain', round(d['drain_ms'],2), 'acc', d['final_test_acc'], 'rb', round(p['recover.readback'],3), 'audit', round(p['recover.audit'],3), 'kw', round(p['verify.krum_wait'],3))"
done
if [ "${LONG:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/${TAG}_long.txt 2>&1 || { echo "LONG FAILED"; tail -5 gpurun_out/${TAG}_long.txt; exit 1; }
  grep '^{' gpurun_out/${TAG}_long.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('long', round(d['ms_per_step'],3), 'acc', d['final_test_acc'])"
fi
