# Round-5 multi-rank stall study: the box's CPU quota and cgroup counters, then a same-box
# alternating A/B of the 2-rank RCCL rehearsal (both ranks on the box's one GPU, socket transport) between
# ab_base (scripts/make_ab_base.sh e45e382: worst round 3.44 ms in round 4) and the working tree, 60 timed rounds
# each, with the cgroup's throttle counters read around every run; VARIANTS adds working-tree runs with other
# RunConfig overrides (e.g. a smaller native pool).  Output: gpurun_out/r5stall/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5stall; mkdir -p $O
{
  echo "nproc $(nproc)"; cat /proc/self/cgroup
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.stat \
           /sys/fs/cgroup/cpuset.cpus.effective; do [ -e $f ] && { echo "== $f"; cat $f; }; done
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
} > $O/box.txt 2>&1
cat $O/box.txt | head -30
cgstat() { python -c "from biscotti_amd.utils import threadcpu as t; import json; print(json.dumps(t.cgroup_cpu_stat()))"; }
run() {  # $1 = variant (base|new), $2 = tag, $3.. = extra bench args
  v=$1; tag=$2; shift 2
  if [ $v = base ]; then D=$R/ab_base; else D=$R; fi
  c0=$(cgstat)
  (cd $D && BISCOTTI_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps ${STEPS:-60} --warmup 5 \
      --set ablation=spec_head_shared "$@") > $O/${v}_$tag.txt 2>&1 || { echo "FAIL $v $tag"; tail -20 $O/${v}_$tag.txt; return 1; }
  c1=$(cgstat)
  python - "$O/${v}_$tag.txt" "$c0" "$c1" "$v $tag" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
c0, c1 = json.loads(sys.argv[2]), json.loads(sys.argv[3])
w = d['round_wall_ms']; med = sorted(w)[len(w) // 2]
cg = {k: c1[k] - c0.get(k, 0) for k in c1}
kw = [r['phase_ms_per_round'].get('verify.krum_wait') for r in d.get('per_rank', [])]
print(sys.argv[4], 'ms', round(d['ms_per_step'], 3), 'med', round(med, 3), 'max', max(w), '>3x', sum(x > 3 * med for x in w),
      '>5x', sum(x > 5 * med for x in w), 'cg', cg, 'krum_wait', kw,
      'cpu', [round(r['host_cpu_ms_per_round'], 1) for r in d.get('per_rank', [])])
json.dump({'bench': d, 'cg_shell': cg}, open(sys.argv[1].replace('.txt', '.json'), 'w'))
EOF
}
for rep in $(seq 1 ${REPS:-3}); do
  if [ $((rep % 2)) = 1 ]; then order="base new"; else order="new base"; fi
  for v in $order; do run $v s$rep || exit 1; done
done
i=0
for var in $VARIANTS; do i=$((i+1)); run new var$i --set $var || exit 1; done
exit 0
