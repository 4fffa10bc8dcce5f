# round 6: HBM bytes per launch of the dynamic path's kernels (C3, dynamic input): the two
# PMC passes of scripts/gpu_traffic.sh on the dynamic bench command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 bench.py --config c3 --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c3dyn_fetch -o run --output-format csv -- $CMD > gpurun_out/pmc_c3dyn_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c3dyn_write -o run --output-format csv -- $CMD > gpurun_out/pmc_c3dyn_write.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmc_c3dyn_fetch/run_counter_collection.csv gpurun_out/pmc_c3dyn_write/run_counter_collection.csv gpurun_out/traffic_c3_dynamic.json > gpurun_out/traffic_c3_dynamic.txt 2>&1
