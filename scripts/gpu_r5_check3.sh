# Round-5 check 3: the collectives serialised on one comm stream (parallel/comm.py _ordered): three 60-round 2-rank
# RCCL rehearsals, a per-rank kernel trace (which streams the RCCL kernels run on), the GPU tests that cover the
# changed paths (evaluation self-reset, multi-rank, engine paths), and a 1-rank A/B of the host-wait spin
# (5 ms full spin, the new one-rank default, vs the 200 us spin-then-sleep of round 4: ablation short_spin).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5c3; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
pr = d.get('per_rank', [d])
p = d['phase_ms_per_round']
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', max(w), '>3x', sum(x > 3 * med for x in w),
      'thr', [r.get('cgroup_cpu_stat_delta', {}).get('nr_throttled') for r in pr], 'pool', d.get('host_threads'),
      'cpu', [round(r['host_cpu_ms_per_round'], 1) for r in pr], 'rccl', [r['thread_cpu_ms_per_round'].get('comm-nccl') for r in pr],
      'rb', round(p.get('recover.readback', 0), 3), 'kw', round(p.get('verify.krum_wait', 0), 3), 'drain', round(d['drain_ms'], 2))
PY
}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ml.py tests/test_gpu_multirank.py tests/test_gpu_engine_paths.py -x -v \
  --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { echo "GPU TESTS FAILED"; grep -E "FAIL|Error" $O/gputests.txt | tail -20; exit 1; }
echo "gpu tests passed: $(grep -c PASSED $O/gputests.txt)"
for i in 1 2 3; do
  BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared \
    > $O/reh$i.txt 2>&1 || { echo "FAIL reh $i"; tail -20 $O/reh$i.txt; exit 1; }
  summ $O/reh$i.txt "reh $i"
done
for i in 1 2 3; do
  for v in full short; do
    if [ $v = short ]; then X="--set ablation=short_spin"; else X=""; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 $X > $O/b1_${v}_$i.txt 2>&1 || { echo "FAIL b1 $v"; exit 1; }
    summ $O/b1_${v}_$i.txt "b1 $v s$i"
  done
done
cd /tmp && export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29519 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 BISCOTTI_RCCL_SHARED_DEVICE=1
pids=""
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/kt_r$r" -o run -- \
    python3 "$R/bench.py" --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared > "$R/$O/kt_r$r.txt" 2>&1 &
  pids="$pids $!"
done
ok=1; for p in $pids; do wait $p || ok=0; done
cd "$R"
[ $ok = 1 ] || { echo "TRACE FAILED"; tail -5 $O/kt_r0.txt $O/kt_r1.txt; exit 1; }
summ $O/kt_r0.txt "traced"
for r in 0 1; do T=$(find $O/kt_r$r -name '*kernel_trace.csv' | head -1); gzip -c "$T" > $O/kt_r$r.csv.gz; rm -rf $O/kt_r$r; done
exit 0
