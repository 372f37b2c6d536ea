# A/B of the 2-rank RCCL rehearsal (two ranks sharing the GPU over RCCL's socket transport):
# current code (default and the no_pipeline ablation) against a staged older tree (OLD=dir).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() {  # name dir extra-args...
  local name=$1 dir=$2; shift 2
  (cd $dir && BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port ${PORT:-29531} bench.py --gpus 2 --steps 30 --warmup 5 "$@") \
    > gpurun_out/rab_$name.txt 2>&1 || { echo "RUN $name FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/rab_$name.txt | tail -15; exit 1; }
  grep '^{' gpurun_out/rab_$name.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$name', round(d['ms_per_step'],3), 'krum_wait', round(p.get('verify.krum_wait',0),3), 'readback', round(p.get('recover.readback',0),3), 'cpu', round(d['host_cpu_ms_per_round'],1))"
}
for v in ${VARIANTS:-new nopipe}; do
  case $v in
    new) run new . ;;
    nopipe) run new_nopipe . --set ablation=no_pipeline ;;
  esac
done
[ -n "$OLD" ] && run old $OLD
true
