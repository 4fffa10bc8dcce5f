# round 6: the split quiet start (2 ranks on one GPU over gloo) + the windowed shard tests; then the C3 kernel-trace profile (csv)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu \
  "tests/test_gpu_dist.py::test_two_ranks_match_one" "tests/test_gpu_dynamic.py::test_shard_windows_vs_oracle" \
  > gpurun_out/r06h_dist_tests.log 2>&1
rc=$?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06h_prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r06h_prof.log 2>&1
exit $rc
