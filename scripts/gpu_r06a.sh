# round 6 first call: the limiter from_rest fix + close() (dist tests, limiter parity),
# then a bare `bench.py --gpus 2` (no launcher: it must start its 2 ranks itself), C3 and C4
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dist.py "tests/test_gpu_parity.py::test_limiter_segments_vs_oracle" \
  > gpurun_out/r06a_tests.log 2>&1 || exit 1
for cfg in c3 c4; do
  timeout -k 10 400 python bench.py --gpus 2 --config $cfg --dist-backend gloo --one-device --steps 10 \
    --warmup 2 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06a_${cfg}_bare_n2.log 2>&1 || exit 1
done
