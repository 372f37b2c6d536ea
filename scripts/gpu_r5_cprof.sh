# Host-side function profile of the headline run (cProfile over 200 timed rounds): where the round's Python time goes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5cp; mkdir -p $O
timeout -k 10 400 python -m cProfile -o $O/prof.out bench.py --steps 200 --warmup 10 > $O/bench.txt 2>&1 || { echo "PROF FAILED"; tail -5 $O/bench.txt; exit 1; }
python - <<'PY' > gpurun_out/r5cp/summary.txt
import pstats
p = pstats.Stats("gpurun_out/r5cp/prof.out")
p.sort_stats("tottime").print_stats(60)
p.sort_stats("cumulative").print_stats(80)
PY
head -90 $O/summary.txt | tail -70
