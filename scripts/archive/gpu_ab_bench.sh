# A/B of engine settings on the headline bench: one bench.py per --set variant (VARIANTS, ';'-separated)
set -o pipefail
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:-none}"
i=0
for v in "${VS[@]}"; do
  args=""
  for kv in $v; do [ "$kv" != "none" ] && args="$args --set $kv"; done
  timeout -k 10 240 python bench.py --steps ${STEPS:-60} --warmup 10 $args > gpurun_out/ab_${TAG:-}$i.txt 2>&1 || { echo "variant '$v' FAILED"; tail -5 gpurun_out/ab_${TAG:-}$i.txt; exit 1; }
  python - "$v" gpurun_out/ab_${TAG:-}$i.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["phase_ms_per_round"]
print(f"{sys.argv[1]:40s} ms/round {d['ms_per_step']:.3f} host_cpu {d['host_cpu_ms_per_round']:.1f} acc {d['final_test_acc']:.3f}",
      "vrf_join %.3f verify %.3f next_head %.3f" % (ph.get("vrf_join", 0), ph.get("verify", 0), ph.get("next_head", 0)),
      {k: v for k, v in d.get("engine_stats", {}).items() if k in ("spec_misses", "device_aggregations", "pre_steps")})
PY
  i=$((i+1))
done
