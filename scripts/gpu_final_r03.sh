#!/bin/bash
# End-of-round GPU run (round 3): the GPU suite, smoke, the default bench, a rocprofv3
# kernel-stats profile of C3, and the C3 PMC traffic / FLOP summaries bench.py reads.
# Every step under its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03d}
STEPS="tests smoke" TAG=$TAG bash scripts/gpu_r03.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c3 -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs \
    > gpurun_out/prof_${TAG}_c3.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo "prof done"
CFG=c3 bash scripts/gpu_traffic.sh || { echo "traffic rc=$?"; exit 1; }
echo "traffic done"
CFG=c3 bash scripts/gpu_flops.sh || { echo "flops rc=$?"; exit 1; }
echo "flops done"
