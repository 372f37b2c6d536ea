# bench.py on N ranks that share the box's one GPU over RCCL (socket transport, distinct NCCL_HOSTIDs):
# a pessimistic rehearsal of the multi-GPU path (the ranks contend for one device)
set -o pipefail
N=${N:-2}
mkdir -p gpurun_out
BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port ${PORT:-29511} bench.py --gpus $N --steps ${STEPS:-60} --warmup 10 \
  > gpurun_out/rccl_bench_$N.txt 2>&1 || { echo "RCCL BENCH FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/rccl_bench_$N.txt | tail -20; exit 1; }
grep '^{' gpurun_out/rccl_bench_$N.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', d['n_gpus'], 'ms/round', round(d['ms_per_step'],3), 'acc', d['final_test_acc'], 'parallelism', d['config']['parallelism'])"
