# round-2 config sweep: headline over 3 seeds, then the BASELINE presets; JSON lines -> gpurun_out/sweep_r2.jsonl
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep_r2.jsonl
if [ -z "$SKIP_HEADLINE" ]; then
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --seeds 3 > gpurun_out/sweep_headline.txt 2>&1 || { echo HEADLINE FAILED; tail -5 gpurun_out/sweep_headline.txt; exit 1; }
  tail -1 gpurun_out/sweep_headline.txt > gpurun_out/sweep_r2.jsonl
fi
timeout -k 10 1000 python scripts/run_configs.py --out gpurun_out/sweep_r2.jsonl --steps 100 --warmup 5 --timeout 240 \
  ${CONFIGS:-mnist10_dp1 fedsys poison30 poison30_200 credit50_3v30 poison50_5v churn10 churn_kill2 lfw100 kzg_audit scale40 scale80 scale200 secagg_off verification_off noising_off credit4}
python - <<'PY'
import json
for ln in open("gpurun_out/sweep_r2.jsonl"):
    ln = ln.strip()
    if not ln.startswith("{"): continue
    d = json.loads(ln)
    c = d.get("config", {})
    if isinstance(c, str):
        print(f"{c:16s} FAILED rc={d.get('rc')} {d.get('error', '')}")
        continue
    print(f"{c.get('name', '?'):16s} {d.get('ms_per_step', float('nan')):8.3f} ms  acc {d.get('final_test_acc')}  last10 {d.get('test_acc_last10_mean')}  attack {d.get('attack_rate_last10_mean')}  {d.get('error', '')}")
PY
