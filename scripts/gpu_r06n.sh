# round 6: kernel profile of the C3 dynamic-mode step (bench --input dynamic)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06n_prof -o dyn -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --input dynamic --no-other-configs --no-cpu-baseline --no-pipeline --steps 40 --warmup 3 --soak 0 > $GRAFT_REPO_ROOT/gpurun_out/r06n_prof.log 2>&1
