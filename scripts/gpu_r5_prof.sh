# cProfile of 200 steady-state headline rounds (scripts/prof_rounds.py) -> gpurun_out/r5prof/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5prof; mkdir -p $O
timeout -k 10 300 python scripts/prof_rounds.py --warm 30 --rounds 200 -o $O/prof.txt > $O/out.txt 2>&1 \
  || { echo "PROF FAILED"; tail -20 $O/out.txt; exit 1; }
head -80 $O/prof.txt
