# One GPU session on the 1-GPU box: GPU tests, smoke, driver-style and long benches, and the RCCL
# rehearsals (2 and 4 ranks sharing the GPU over RCCL's socket transport).  Every GPU step has its own
# time limit; the first failure ends the script.  STEPS selects a subset: tests,smoke,short,long,rccl2,rccl4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
STEPS=${STEPS:-tests,smoke,short,long,rccl2,rccl4}
TAG=${TAG:-s}
has() { case ",$STEPS," in *",$1,"*) return 0;; *) return 1;; esac; }
if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputests_$TAG.txt 2>&1 || { echo "GPU TESTS FAILED rc=$?"; grep -E "PASS|FAIL|Error" gpurun_out/gputests_$TAG.txt | tail -30; exit 1; }
  grep -cE "PASSED" gpurun_out/gputests_$TAG.txt
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke_$TAG.txt; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.txt
fi
if has short; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_short_$TAG.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_short_$TAG.txt; exit 1; }
  grep '^{' gpurun_out/bench_short_$TAG.txt | tail -1 > gpurun_out/bench_short_$TAG.json
  python -c "import json; d=json.load(open('gpurun_out/bench_short_$TAG.json')); print('short ms/round', round(d['ms_per_step'],3), 'acc', d['final_test_acc'])"
fi
if has long; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 200 --warmup 10 > gpurun_out/bench_long_$TAG.txt 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_long_$TAG.txt; exit 1; }
  grep '^{' gpurun_out/bench_long_$TAG.txt | tail -1 > gpurun_out/bench_long_$TAG.json
  python -c "import json; d=json.load(open('gpurun_out/bench_long_$TAG.json')); print('long ms/round', round(d['ms_per_step'],3), 'acc', d['final_test_acc'], 'phases', {k: round(v,3) for k,v in d['phase_ms_per_round'].items()})"
fi
if has acc10; then   # headline accuracy over 10 independent 100-round runs (final + last-10 mean, mean +- std)
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --seeds 10 > gpurun_out/acc10_$TAG.txt 2>&1 || { echo "ACC10 FAILED"; tail -20 gpurun_out/acc10_$TAG.txt; exit 1; }
  grep '^{' gpurun_out/acc10_$TAG.txt | tail -1 > gpurun_out/acc10_$TAG.json
  python -c "import json; d=json.load(open('gpurun_out/acc10_$TAG.json')); print('acc10 final', d['final_test_acc_mean_std'], 'last10', d['test_acc_last10_mean_std'], 'ms', round(d['ms_per_step'],3))"
fi
for cfgname in poison30 poison30_200; do
  if has $cfgname; then   # BASELINE config 4 over 5 seeds
    timeout -k 10 600 python bench.py --gpus 1 --config $cfgname --steps 20 --warmup 5 --seeds 5 > gpurun_out/${cfgname}_$TAG.txt 2>&1 || { echo "$cfgname FAILED"; tail -20 gpurun_out/${cfgname}_$TAG.txt; exit 1; }
    grep '^{' gpurun_out/${cfgname}_$TAG.txt | tail -1 > gpurun_out/${cfgname}_$TAG.json
    python -c "import json; d=json.load(open('gpurun_out/${cfgname}_$TAG.json')); print('$cfgname acc', d['final_test_acc_mean_std'], 'last10', d['test_acc_last10_mean_std'], 'att', d['attack_rate_last10_mean_std'], 'ms', round(d['ms_per_step'],3))"
  fi
done
for n in 2 4; do
  if has rccl$n; then
    BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29511 + n)) bench.py --gpus $n --steps 40 --warmup 10 \
      > gpurun_out/rccl_bench_${n}_$TAG.txt 2>&1 || { echo "RCCL BENCH $n FAILED"; grep -v "Train Error\|Attack Rate" gpurun_out/rccl_bench_${n}_$TAG.txt | tail -20; exit 1; }
    grep '^{' gpurun_out/rccl_bench_${n}_$TAG.txt | tail -1 > gpurun_out/rccl_bench_${n}_$TAG.json
    python -c "import json; d=json.load(open('gpurun_out/rccl_bench_${n}_$TAG.json')); print('rccl', d['n_gpus'], 'ms/round', round(d['ms_per_step'],3), 'acc', d['final_test_acc'], 'host_cpu', round(d['host_cpu_ms_per_round'],2), 'b0', d['b0'])"
  fi
done
