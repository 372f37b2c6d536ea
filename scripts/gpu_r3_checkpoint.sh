# Round-3 checkpoint on one box: every GPU test, the smoke test, two driver-style benches, one long bench,
# a kernel-trace + stats profile of a driver-style bench (database output), and the host timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-cp}
STEPS=tests,smoke,short,long TAG=$TAG bash scripts/gpu_session.sh || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/short2_$TAG.txt 2>&1 || { echo "BENCH2 FAILED"; exit 1; }
grep '^{' gpurun_out/short2_$TAG.txt | tail -1 > gpurun_out/bench_short2_$TAG.json
python -c "import json; d=json.load(open('gpurun_out/bench_short2_$TAG.json')); print('short2', round(d['ms_per_step'],3))"
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_$TAG -o run -- python3 $PWD/bench.py --steps 20 --warmup 5 > gpurun_out/prof_$TAG.txt 2>&1 || { echo "PROF FAILED"; tail -20 gpurun_out/prof_$TAG.txt; exit 1; }
W=_spec_head_launch,_queue_pre_step,_aggregate_native,_krum_static,_select_noisers,_noise_ids_np,_launch_krum,_spec_aggregate,_early_vrf_submit,_log_round,task.evaluate_async,_open_round,_prepare_next_in_wait,_finish_secagg,_secure_aggregation,_verification
timeout -k 10 200 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true --wrap $W > gpurun_out/host_tl_$TAG.json 2> gpurun_out/host_tl_$TAG.err || { echo "TL FAILED"; exit 1; }
echo done
