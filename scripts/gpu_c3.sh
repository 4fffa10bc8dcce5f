#!/bin/bash
# C3 (multiband + width + analog) bench + rocprof summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01_c3}
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench_c3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
echo "prof_rc=$?" >> gpurun_out/prof_${TAG}.log
