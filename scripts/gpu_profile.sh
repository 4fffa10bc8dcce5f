#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (writes gpurun_out/prof_*)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1
echo "prof_rc=$?" >> gpurun_out/prof_${TAG}.log
