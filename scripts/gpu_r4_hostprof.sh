# Host hot spots of the 1-GPU round: cProfile over 200 rounds, and a fine host timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/host_cprofile.py --steps 200 --warmup 10 --rounds 210 > gpurun_out/cprof.txt 2>&1 || { echo "CPROF FAILED"; tail -20 gpurun_out/cprof.txt; exit 1; }
grep -A 60 "==== by tottime" gpurun_out/cprof.txt | head -70
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true --wrap fsm.spec_plan,fsm.make_secagg_block,fsm.route_view,fsm.approve,fsm.commit_block,fsm.begin_round,_krum_static,_spec_head_launch,_spec_aggregate,_aggregate_native,_queue_pre_step,_early_vrf_submit,_open_round,_noise_ids_np,_select_noisers,_log_round,_resolve_evals,task.evaluate_async,_vrf_key_rows > gpurun_out/host_tl2.json 2> gpurun_out/host_tl2.err || { echo "TIMELINE FAILED"; tail -20 gpurun_out/host_tl2.err; exit 1; }
echo timeline ok
