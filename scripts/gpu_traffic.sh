#!/bin/bash
# HBM bytes per kernel launch for one bench config: two PMC passes (FETCH_SIZE and
# WRITE_SIZE do not fit one pass), then gpurun_out/traffic_<config>.json (copy it to profiles/ for bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
CFG=${CFG:-c2}
CMD="python3 bench.py --config $CFG --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${CFG}_fetch -o run --output-format csv -- $CMD > gpurun_out/pmc_${CFG}_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${CFG}_write -o run --output-format csv -- $CMD > gpurun_out/pmc_${CFG}_write.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmc_${CFG}_fetch/run_counter_collection.csv gpurun_out/pmc_${CFG}_write/run_counter_collection.csv gpurun_out/traffic_${CFG}.json > gpurun_out/traffic_${CFG}.txt 2>&1
