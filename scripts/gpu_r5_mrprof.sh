# Round-5: where one rank of a multi-rank job spends its round's host time (emulated rank 0 of 8 and of 2):
# cProfile of 200 steady-state rounds, plus the same for one rank alone.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; O=gpurun_out/r5mrprof; mkdir -p $O
for n in 8 2; do
  timeout -k 10 300 python scripts/prof_rounds.py --emulate-world $n --warm 30 --rounds 200 -o $O/prof_emu$n.txt > $O/prof_emu$n.log 2>&1 \
    || { echo "FAIL prof emu $n"; tail -20 $O/prof_emu$n.log; exit 1; }
  echo "emu $n done"
done
timeout -k 10 300 python scripts/prof_rounds.py --warm 30 --rounds 200 -o $O/prof_1.txt > $O/prof_1.log 2>&1 || { echo "FAIL prof 1"; exit 1; }
echo "1 done"
