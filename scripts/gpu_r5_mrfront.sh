# Round-5 early front with several ranks: the multi-rank GPU tests (RCCL and gloo ranks sharing the GPU, chains
# identical to one process), then emulated ranks N = 2 / 4 / 8 against ab_base (HEAD without it) and a rehearsal.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5mrf; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_ml.py -x -v --timeout 300 \
  --timeout-method thread -k "rank or early_front or last_round" > $O/tests.txt 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.txt | tail -20; exit 1; }
echo "tests passed: $(grep -c PASSED $O/tests.txt)"
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', round(max(w), 3), 'fronts', d['engine_stats'].get('early_fronts'), flush=True)
PY
}
for n in 2 4 8; do
  for v in new base; do
    case $v in base) D=$R/ab_base;; *) D=$R;; esac
    (cd $D && timeout -k 10 300 python bench.py --emulate-world $n --steps 20 --warmup 5) > $O/emu${n}_$v.txt 2>&1 || { echo "FAIL emu $n $v"; tail -20 $O/emu${n}_$v.txt; exit 1; }
    summ $O/emu${n}_$v.txt "emu $n $v"
  done
done
for n in 8; do
  for v in base new; do
    case $v in base) D=$R/ab_base;; *) D=$R;; esac
    (cd $D && timeout -k 10 300 python bench.py --emulate-world $n --steps 20 --warmup 5) > $O/emu${n}_${v}2.txt 2>&1 || { echo "FAIL emu $n $v"; exit 1; }
    summ $O/emu${n}_${v}2.txt "emu $n $v (2)"
  done
done
BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared \
  > $O/reh.txt 2>&1 || { echo "FAIL reh"; tail -20 $O/reh.txt; exit 1; }
summ $O/reh.txt "reh"
