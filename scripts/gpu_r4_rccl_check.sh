set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 5 --set ablation=spec_head_shared > gpurun_out/rccl2_noprio.txt 2>&1 || { echo "RCCL2 FAILED"; tail -20 gpurun_out/rccl2_noprio.txt; exit 1; }
grep '^{' gpurun_out/rccl2_noprio.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl2', round(d['ms_per_step'],3), [round(x,1) for x in d['round_wall_ms']])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b1_prio.txt 2>&1 || { echo "BENCH FAILED"; exit 1; }
grep '^{' gpurun_out/b1_prio.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench1', round(d['ms_per_step'],3))"
