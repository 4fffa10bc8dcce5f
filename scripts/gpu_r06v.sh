# round 6: the hand-off recipe in k_peak_reduce and the general limiter's walker -- the
# full GPU suite, then C3 / dynamic benches and the C3 kernel profile
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r06v_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 400 --warmup 10 --soak 0 --no-cpu-baseline --no-other-configs \
  --no-pipeline > gpurun_out/r06v_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 3 --soak 0 --no-cpu-baseline \
  --no-other-configs --no-pipeline > gpurun_out/r06v_dyn.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06v_prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r06v_prof.log 2>&1
