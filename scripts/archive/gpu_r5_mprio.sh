# Round-5: the wave priority classes with several ranks (ablation wave_prio_multi) against the default (classes
# off when world > 1): emulated rank 0 of N = 8 / 2 (one process, no transport) and the 2-rank RCCL rehearsal
# (both ranks on the box's one GPU), alternating on the same box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5mprio; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
pr = d.get('per_rank', [d])
p = d['phase_ms_per_round']
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', round(max(w), 3), '>3x', sum(x > 3 * med for x in w),
      'cpu', [round(r['host_cpu_ms_per_round'], 1) for r in pr], 'rb', round(p.get('recover.readback', 0), 3),
      'krum_wait', round(p.get('verify.krum_wait', 0), 3), flush=True)
PY
}
for i in 1 2; do
  for v in off on; do
    A=""; [ $v = on ] && A="--set ablation=wave_prio_multi"
    timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --warmup 5 $A > $O/emu8_${v}_$i.txt 2>&1 || { echo "FAIL emu8 $v $i"; tail -20 $O/emu8_${v}_$i.txt; exit 1; }
    summ $O/emu8_${v}_$i.txt "emu8 $v $i"
  done
done
for v in on off; do
  A=""; [ $v = on ] && A="--set ablation=wave_prio_multi"
  timeout -k 10 300 python bench.py --emulate-world 2 --steps 20 --warmup 5 $A > $O/emu2_$v.txt 2>&1 || { echo "FAIL emu2 $v"; exit 1; }
  summ $O/emu2_$v.txt "emu2 $v"
done
for i in 1 2; do
  for v in on off; do
    A=spec_head_shared; [ $v = on ] && A=spec_head_shared,wave_prio_multi
    BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 60 --warmup 5 --set ablation=$A \
      > $O/reh_${v}_$i.txt 2>&1 || { echo "FAIL reh $v $i"; tail -20 $O/reh_${v}_$i.txt; exit 1; }
    summ $O/reh_${v}_$i.txt "reh $v $i"
  done
done
