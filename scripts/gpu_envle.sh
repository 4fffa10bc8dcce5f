#!/bin/bash
# Envelope segment length sweep (AMX_ENV_LE) on one config: rocprof kernel stats + bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
for le in ${LES:-1024 768}; do
  AMX_ENV_LE=$le timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/envle_${CFG}_$le -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/envle_${CFG}_$le.log 2>&1 || { echo "$le rc=$?"; exit 1; }
  AMX_ENV_LE=$le timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --no-pipeline > gpurun_out/envle_${CFG}_${le}_bench.log 2>&1 || { echo "$le bench rc=$?"; exit 1; }
done
