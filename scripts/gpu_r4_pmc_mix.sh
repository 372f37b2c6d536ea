# VALU work per kernel over a short bench run (rocprofv3 --pmc, its own run; no trace domains)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"; cd "$R"; mkdir -p gpurun_out/pmcmix
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/pmcmix" -o mix -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$R/gpurun_out/pmcmix_bench.txt" 2>&1 || { echo PMC FAILED; tail -5 "$R/gpurun_out/pmcmix_bench.txt"; exit 1; }
cd "$R"
python3 scripts/pmc_round_mix.py gpurun_out/pmcmix 100   # the bench runs 100 rounds (accuracy quote) > gpurun_out/pmc_mix.json
find gpurun_out/pmcmix -name '*counter_collection.csv' -delete
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_mix.json'))
for k in d['kernels'][:14]: print(k['kernel'], k['dispatches'], k['valu_share'], round(k.get('SQ_INSTS_VALU',0)/1e6,2), 'M VALU/round')"
