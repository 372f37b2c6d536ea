# Round-5 closing evidence on the final code: driver-style x3 and 200 rounds (1 GPU), bench --emulate-world 2/4/8
# (rank 0's per-round cost of an N-GPU job), two 60-round 2-rank RCCL rehearsals (stall check), a host timeline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5close; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
pr = d.get('per_rank', [d])
p = d['phase_ms_per_round']
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', round(max(w), 3), '>3x', sum(x > 3 * med for x in w),
      'thr', [r.get('cgroup_cpu_stat_delta', {}).get('nr_throttled') for r in pr], 'cpu', [round(r['host_cpu_ms_per_round'], 1) for r in pr],
      'rb', round(p.get('recover.readback', 0), 3), 'drain', round(d['drain_ms'], 2), flush=True)
PY
}
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b1_s$i.txt 2>&1 || { echo "FAIL b1 $i"; tail -5 $O/b1_s$i.txt; exit 1; }
  summ $O/b1_s$i.txt "b1 s$i"
done
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > $O/b1_long.txt 2>&1 || { echo "FAIL long"; exit 1; }
summ $O/b1_long.txt "b1 long"
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-world $n --steps 20 --warmup 5 > $O/emu$n.txt 2>&1 || { echo "FAIL emu $n"; tail -20 $O/emu$n.txt; exit 1; }
  summ $O/emu$n.txt "emulated world $n"
done
for i in 1 2; do
  BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared \
    > $O/reh$i.txt 2>&1 || { echo "FAIL reh $i"; tail -20 $O/reh$i.txt; exit 1; }
  summ $O/reh$i.txt "reh $i"
done
timeout -k 10 300 python scripts/host_timeline.py --rounds 4 --warm 30 --set lazy_eval=true \
  --wrap _early_vrf_submit,_spec_head_launch,_prepare_next_in_wait,_open_round,_select_noisers,_launch_krum,native.spec_msm,native.after_select,_finish_secagg,_secure_aggregation,_round_front,_finish_verification \
  > $O/host_tl.json 2> $O/host_tl.err || { echo "HOST TL FAILED"; tail -20 $O/host_tl.err; exit 1; }
python -c "
import json; d=json.load(open('$O/host_tl.json'))
for r in d[:2]: print('wall', r['wall_us'], r['jobs (kind, submit_us, queued_us, run_us)'])"
