# Round-5 speculative-miss path: the horizon test (with spec_tight: the host top-up path in most poisoned rounds), then
# driver-style bench runs with the default horizon and with spec_tight (every miss takes the host path).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5miss; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_paths.py -k horizon -x -v -s --timeout 300 \
  --timeout-method thread > $O/horizon_test.txt 2>&1 || { echo "TEST FAILED"; tail -30 $O/horizon_test.txt; exit 1; }
grep -E "PASSED|misses" $O/horizon_test.txt
run() {  # tag steps warmup extra...
  t=$1; st=$2; w=$3; shift 3
  timeout -k 10 300 python bench.py --steps $st --warmup $w "$@" > $O/$t.txt 2>&1 || { echo "FAIL $t"; tail -5 $O/$t.txt; return 1; }
  grep '^{' $O/$t.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$t', round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'max', d.get('round_wall_max_ms'), 'misses', d['engine_stats'].get('spec_misses',0), 'shares', round(p.get('shares',0),3), 'recover', round(p.get('recover',0),3), flush=True)"
}
for i in 1 2; do
  run def_s$i 20 5 || exit 1
  run tight_s$i 20 5 --set ablation=spec_tight || exit 1
done
run tight_long 100 10 --set ablation=spec_tight || exit 1
run def_long 100 10 || exit 1
