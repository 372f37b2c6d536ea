# Round-5 stall study, part 2: (1) three 60-round 2-rank RCCL rehearsals with the quota-fitted pool sizing
# (bench._host_threads -> threadcpu.pool_threads), (2) one with the round-4 sizing (host_threads=8 per rank) for
# the throttle counters, (3) a per-rank rocprofv3 kernel trace of a rehearsal at the round-4 sizing (each rank its
# own rocprofv3 process running python directly), (4) a 1-rank driver-style A/B of pool 14 (new) vs 16 (round 4),
# (5) bench --emulate-world 2/4/8 (rank 0's per-round cost of an N-GPU job).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5stall2; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
pr = d.get('per_rank', [d])
print(sys.argv[2], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', max(w), '>3x', sum(x > 3 * med for x in w),
      'thr', [r.get('cgroup_cpu_stat_delta', {}).get('nr_throttled') for r in pr],
      'thr_ms', [round(r.get('cgroup_cpu_stat_delta', {}).get('throttled_usec', 0) / 1e3, 1) for r in pr],
      'pool', d.get('host_threads'), 'cpu', [round(r['host_cpu_ms_per_round'], 1) for r in pr],
      'rccl', [r['thread_cpu_ms_per_round'].get('comm-nccl') for r in pr])
PY
}
reh() {  # $1 tag, rest: bench args
  t=$1; shift
  BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared "$@" \
    > $O/reh_$t.txt 2>&1 || { echo "FAIL $t"; tail -20 $O/reh_$t.txt; return 1; }
  summ $O/reh_$t.txt "reh $t"
}
for i in 1 2 3; do reh fit$i || exit 1; done
reh r4size --set host_threads=8 || exit 1
for i in 1 2 3; do
  for v in 14 16; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --set host_threads=$v > $O/b1_p${v}_$i.txt 2>&1 || { echo "FAIL b1 $v"; exit 1; }
    summ $O/b1_p${v}_$i.txt "b1 pool$v s$i"
  done
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-world $n --steps 20 --warmup 5 > $O/emu$n.txt 2>&1 || { echo "FAIL emu $n"; tail -20 $O/emu$n.txt; exit 1; }
  summ $O/emu$n.txt "emulated world $n"
done
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  export MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 BISCOTTI_RCCL_SHARED_DEVICE=1
  pids=""
  for r in 0 1; do
    RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/kt_r$r" -o run -- \
      python3 "$R/bench.py" --gpus 2 --steps 60 --warmup 5 --set ablation=spec_head_shared --set host_threads=8 \
      > "$R/$O/kt_r$r.txt" 2>&1 &
    pids="$pids $!"
  done
  ok=1; for p in $pids; do wait $p || ok=0; done
  cd "$R"
  [ $ok = 1 ] || { echo "TRACE FAILED"; tail -5 $O/kt_r0.txt $O/kt_r1.txt; exit 1; }
  summ $O/kt_r0.txt "traced"
  for r in 0 1; do T=$(find $O/kt_r$r -name '*kernel_trace.csv' | head -1); gzip -c "$T" > $O/kt_r$r.csv.gz; rm -rf $O/kt_r$r; done
fi
exit 0
