# round 6: PMC traffic of the C3 / C2 steps on this tree (two passes each), then the
# default bench line (which reads profiles/traffic_c3.json) and the kernel profile of its
# C3 command
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
CFG=c3 bash scripts/gpu_traffic.sh || exit 1
CFG=c2 bash scripts/gpu_traffic.sh || exit 1
cp gpurun_out/traffic_c3.json profiles/traffic_c3.json && cp gpurun_out/traffic_c2.json profiles/traffic_c2.json || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_default.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06_final_prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r06_final_prof.log 2>&1
