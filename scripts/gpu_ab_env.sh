# Same-box A/B of environment variants of the working tree: each variant is NAME:VAR=val,VAR=val (or
# NAME: for none); driver-style benches, REPS repetitions with the variant order alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"base:"}
i=0
for rep in $(seq 1 ${REPS:-3}); do
  list=$VARIANTS
  if [ $((rep % 2)) = 0 ]; then list=$(echo $VARIANTS | tr ' ' '\n' | tac | tr '\n' ' '); fi
  for v in $list; do
    name=${v%%:*}; envs=${v#*:}
    ( for kv in $(echo $envs | tr ',' ' '); do export "$kv"; done
      timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} ) > gpurun_out/abe_${name}_$rep.txt 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/abe_${name}_$rep.txt; exit 1; }
    grep '^{' gpurun_out/abe_${name}_$rep.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$name $rep', round(d['ms_per_step'],3), 'drain', round(d.get('drain_ms',0),2), 'rb', round(p['recover.readback'],3), 'audit', round(p['recover.audit'],3), 'pv', round(p['pre_vrf'],3))"
  done
done
