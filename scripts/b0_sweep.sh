set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for b in 14 13 12 11; do
  BSC_TABLE_B0=$b timeout -k 10 300 python bench.py > gpurun_out/b0_$b.txt 2>&1 || { echo "fail $b"; tail -5 gpurun_out/b0_$b.txt; exit 1; }
  echo "B0=$b $(grep '^{' gpurun_out/b0_$b.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["phase_ms_per_round"]["verify.defense"],3), round(d["phase_ms_per_round"]["recover.readback"],3))')"
done
