# round 6: the whole GPU suite on the tree with the zero kernels, from_rest, close(), dynamic graphs
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r06d_gpu_tests.log 2>&1
