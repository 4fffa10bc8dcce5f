#!/bin/bash
# k_env0 placement sweep (AMX_ENV_WG: 0 = single-wave workgroups at Le 1024; 1/2/4 waves
# per CU with the plan's Le): rocprof kernel stats + the bench line, per config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-c3}; do
  for wg in ${WGS:-0 2}; do
    AMX_ENV_WG=$wg timeout -k 10 300 \
      rocprofv3 --kernel-trace --stats -d gpurun_out/envwg_${cfg}_$wg -o run --output-format csv -- \
      python3 bench.py --config $cfg --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/envwg_${cfg}_$wg.log 2>&1 || { echo "$cfg $wg rc=$?"; exit 1; }
  done
done
