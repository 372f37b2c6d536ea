# Kernel-trace profiles of the driver-style bench for the in-tree kernel library (new) and exp/libhip_old.so
# (old), one rocprofv3 run each (database output; convert with rocpd2csv on the host).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
for v in ${VARIANTS:-new old}; do
  if [ $v = old ]; then export BISCOTTI_HIP_LIB=$R/${OLD:-exp/libhip_old.so}; else unset BISCOTTI_HIP_LIB; fi
  rm -rf gpurun_out/profab_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/profab_$v -o run -- python3 $R/bench.py --steps 20 --warmup 5 > gpurun_out/profab_$v.txt 2>&1 || { echo "PROF $v FAILED"; tail -20 gpurun_out/profab_$v.txt; exit 1; }
  grep '^{' gpurun_out/profab_$v.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3))"
done
