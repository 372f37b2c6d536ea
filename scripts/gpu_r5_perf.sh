# Round-5 performance evidence on one box: (1) three 60-round 2-rank RCCL rehearsals (the stall check); (2) a 1-rank
# driver-style A/B of the host-wait spin (5 ms, the one-rank default, vs 200 us: ablation short_spin) and of the
# periodic noise Gram table (vs noise_gram_each_round), 3 rounds of the three;
# (3) bench --emulate-world 2/4/8; (4) the double-FMA multiplier prototype (exact check + throughput); (5) a 1-GPU
# kernel + HIP runtime trace: per-kernel stats, the round timeline, which API call queued each runtime blit;
# (6) the poisoning guard's deterministic run, printed.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5p; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
pr = d.get('per_rank', [d])
p = d['phase_ms_per_round']
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', max(w), '>3x', sum(x > 3 * med for x in w),
      'thr', [r.get('cgroup_cpu_stat_delta', {}).get('nr_throttled') for r in pr], 'cpu', [round(r['host_cpu_ms_per_round'], 1) for r in pr],
      'rccl', [r['thread_cpu_ms_per_round'].get('comm-nccl') for r in pr], 'rb', round(p.get('recover.readback', 0), 3),
      'kw', round(p.get('verify.krum_wait', 0), 3), 'ver', round(p.get('verify', 0), 3), 'drain', round(d['drain_ms'], 2), flush=True)
PY
}
for i in 1 2 3; do
  BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared \
    > $O/reh$i.txt 2>&1 || { echo "FAIL reh $i"; tail -20 $O/reh$i.txt; exit 1; }
  summ $O/reh$i.txt "reh $i"
done
for i in 1 2 3; do
  for v in full short gramall; do
    case $v in short) X="--set ablation=short_spin";; gramall) X="--set ablation=noise_gram_each_round";; *) X="";; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 $X > $O/b1_${v}_$i.txt 2>&1 || { echo "FAIL b1 $v"; exit 1; }
    summ $O/b1_${v}_$i.txt "b1 $v s$i"
  done
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-world $n --steps 20 --warmup 5 > $O/emu$n.txt 2>&1 || { echo "FAIL emu $n"; tail -20 $O/emu$n.txt; exit 1; }
  summ $O/emu$n.txt "emulated world $n"
done
timeout -k 10 120 ./scripts/isa/fpmul_f64 /tmp/fpmul_f64_check.bin > $O/fpmul_f64.jsonl 2>&1 || { echo "F64 BENCH FAILED"; cat $O/fpmul_f64.jsonl; exit 1; }
timeout -k 10 300 python scripts/isa/fpmul_f64_check.py /tmp/fpmul_f64_check.bin >> $O/fpmul_f64.jsonl || { echo "F64 CHECK FAILED"; exit 1; }
rm -f /tmp/fpmul_f64_check.bin
cat $O/fpmul_f64.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine_paths.py -k label_flip -s -q --timeout 280 --timeout-method thread \
  > $O/poison_guard.txt 2>&1 || { echo "POISON GUARD FAILED"; tail -20 $O/poison_guard.txt; exit 1; }
grep "digit-1" $O/poison_guard.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d "$R/$O/kt" -o run -- \
  python3 "$R/bench.py" --steps 60 --warmup 5 > "$R/$O/kt_bench.txt" 2>&1 || { echo PROF FAILED; tail -20 "$R/$O/kt_bench.txt"; exit 1; }
cd "$R"
T=$(find $O/kt -name '*kernel_trace.csv' | head -1)
H=$(find $O/kt -name '*hip_api_trace.csv' | head -1)
S=$(find $O/kt -name '*kernel_stats.csv' | head -1)
cp "$S" $O/kernel_stats.csv
python scripts/kt_timeline.py "$T" 40 43 > $O/kt_timeline.txt
python scripts/blit_attrib.py "$T" "$H" > $O/blits.json
gzip -c "$T" > $O/kernel_trace.csv.gz
rm -rf $O/kt
head -24 $O/kt_timeline.txt
head -30 $O/blits.json
