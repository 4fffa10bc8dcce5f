# round 6: dynamic-mode tests (ceiling bound, graph form, shard windows) on the current tree
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py > gpurun_out/r06i_dynamic_tests.log 2>&1
