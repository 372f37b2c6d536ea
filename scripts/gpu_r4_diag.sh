# Driver-style 1-GPU benches, a host timeline of steady-state rounds, and a 4-rank RCCL rehearsal with
# per-thread CPU attribution (helper threads labelled by the library that started them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/diag_bench_$i.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/diag_bench_$i.txt; exit 1; }
  grep '^{' gpurun_out/diag_bench_$i.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('bench', round(d['ms_per_step'],3), 'drain', round(d['drain_ms'],2), 'rb', round(p['recover.readback'],3), 'cpu', round(d['host_cpu_ms_per_round'],2), d['thread_cpu_ms_per_round'])"
done
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --wrap _launch_krum,_spec_aggregate,_aggregate_native,_queue_pre_step,_finish_secagg,_spec_head_launch,_early_vrf_submit,_prepare_next_in_wait,_open_round,_noise_ids_np,_select_noisers,_log_round > gpurun_out/host_tl.json 2> gpurun_out/host_tl.err || { echo "TIMELINE FAILED"; tail -20 gpurun_out/host_tl.err; exit 1; }
echo timeline ok
if [ "${RCCL4:-1}" = 1 ]; then
BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python bench.py --gpus 4 --steps 30 --warmup 5 --set ablation=spec_head_shared > gpurun_out/diag_bench4r.txt 2>&1 || { echo "RCCL4 BENCH FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/diag_bench4r.txt | tail -20; exit 1; }
grep '^{' gpurun_out/diag_bench4r.txt | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bench4r', round(d['ms_per_step'],3))
for p in d['per_rank']: print(p['rank'], round(p['host_cpu_ms_per_round'],2), p['thread_cpu_ms_per_round'])"
fi
