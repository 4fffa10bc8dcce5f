# round 5: the whole GPU suite after the envelope fix-up rework
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05ac_gpu_tests.log 2>&1 || exit 1
