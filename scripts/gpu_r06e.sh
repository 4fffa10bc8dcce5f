# round 6: the multichannel path on the GPU
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_multichannel.py > gpurun_out/r06e_mc_tests.log 2>&1
