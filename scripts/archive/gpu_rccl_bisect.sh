# 2-rank RCCL rehearsal (two ranks sharing the box's GPU) for several package trees: TREES="exp/t_a exp/t_b ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
R=$PWD
port=29600
for t in ${TREES:-.}; do
  port=$((port + 1))
  name=$(basename $t)
  (cd $R/$t && BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
     --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps ${STEPS:-20} --warmup 5) > gpurun_out/bisect_$name.txt 2>&1 || { echo "FAIL $name"; grep -v "Train Error\|Attack Rate" gpurun_out/bisect_$name.txt | tail -5; exit 1; }
  grep '^{' gpurun_out/bisect_$name.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$name', round(d['ms_per_step'],3), 'kw', round(p.get('verify.krum_wait',0),2), 'cpu', round(d['host_cpu_ms_per_round'],1))"
done
