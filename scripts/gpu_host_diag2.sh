# Host timeline with engine methods timed as events, then an MSM-library A/B with the old build first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
W=_spec_head_launch,_queue_pre_step,_aggregate_native,_krum_static,_select_noisers,_noise_ids_np,_launch_krum,_agg_index,_predict_miners,_early_vrf_submit,_resolve_evals,_log_round,task.step,task.evaluate_async,crypto.commitments_async,crypto.shares_async,_gram_rows,_open_round,_live_mask,_maybe_fail,_spec_aggregate
timeout -k 10 200 python scripts/host_timeline.py --rounds 4 --warm 30 --wrap $W > gpurun_out/host_tl2.json 2> gpurun_out/host_tl2.err || { echo "TL FAILED"; tail -5 gpurun_out/host_tl2.err; exit 1; }
for rep in 1 2; do for v in old new; do
  if [ $v = old ]; then export BISCOTTI_HIP_LIB=$PWD/exp/libhip_old.so; else unset BISCOTTI_HIP_LIB; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab3_${v}_$rep.txt 2>&1 || { echo "BENCH FAILED"; tail -5 gpurun_out/ab3_${v}_$rep.txt; exit 1; }
  grep '^{' gpurun_out/ab3_${v}_$rep.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rep', round(d['ms_per_step'],3), 'drain', round(d['drain_ms'],2))"
done; done
