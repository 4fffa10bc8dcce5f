# round 6: the default bench line on the current tree + a kernel-trace profile of the C3 step
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r06f_bench_default.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06f_prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r06f_prof.log 2>&1
