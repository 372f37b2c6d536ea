# Round-5 wave priority of the pre-step's commitment MSM (AHEAD instead of SPEC) after the fence fix: same-box A/B
# against ab_base, driver-style x3 alternating + 200 rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5prio2; mkdir -p $O
run() {  # variant tag steps warmup
  v=$1; t=$2; st=$3; w=$4
  case $v in base) D=$R/ab_base;; *) D=$R;; esac
  (cd $D && timeout -k 10 300 python bench.py --steps $st --warmup $w) > $O/${v}_$t.txt 2>&1 || { echo "FAIL $v $t"; tail -5 $O/${v}_$t.txt; return 1; }
  grep '^{' $O/${v}_$t.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$v $t', round(d['ms_per_step'],3), 'p50', d.get('round_wall_p50_ms'), 'max', d.get('round_wall_max_ms'), 'rb', round(p.get('recover.readback',0),3), flush=True)"
}
for i in 1 2 3 4; do
  if [ $((i % 2)) = 0 ]; then run new s$i 20 5 || exit 1; run base s$i 20 5 || exit 1
  else run base s$i 20 5 || exit 1; run new s$i 20 5 || exit 1; fi
done
run new long 200 10 || exit 1
run base long 200 10 || exit 1
