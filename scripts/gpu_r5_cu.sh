# Round-5: same-box A/B of the speculative share MSM's CU mask (3/4 of the CUs, the default; 7/8; all), 3 rounds
# of the three driver-style runs, then a cProfile of a 200-round bench (the host loop's hot spots).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5cu; mkdir -p $O
for i in 1 2 3; do
  for v in base c78 call; do
    case $v in c78) X="--set ablation=side_cus_7of8";; call) X="--set ablation=side_cus_all";; *) X="";; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 $X > $O/b1_${v}_$i.txt 2>&1 || { echo "FAIL b1 $v"; tail -5 $O/b1_${v}_$i.txt; exit 1; }
    grep '^{' $O/b1_${v}_$i.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_round']; print('$v $i', round(d['ms_per_step'],3), 'p50', d['round_wall_p50_ms'], 'rb', round(p['recover.readback'],3), 'kw', round(p['verify.krum_wait'],3))"
  done
done
timeout -k 10 400 python scripts/host_cprofile.py --steps 200 --warmup 10 > $O/cprof.txt 2> $O/cprof.err || { echo "CPROF FAILED"; tail -5 $O/cprof.err; exit 1; }
head -80 $O/cprof.txt | tail -60
