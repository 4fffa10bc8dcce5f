# round 6: the graph-captured dynamic path against the eager one, scratch compared region by region
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/dyn_graph_probe.py > gpurun_out/r06c_dyn_graph_probe.log 2>&1
