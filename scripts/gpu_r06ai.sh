# round 6: per-kernel profiles of the C2 and C3 linear steps on the current tree
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for c in c2 c3; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ai_prof_$c -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 --warmup 3 --soak 0 > $GRAFT_REPO_ROOT/gpurun_out/r06ai_prof_$c.log 2>&1 || exit 1
done
