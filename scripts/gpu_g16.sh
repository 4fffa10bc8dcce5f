#!/bin/bash
# front1 forms at C3 (measurements): k_gemv16 threads per segment (AMX_G16_PARTS) and
# k_analog_h's block order (AMX_ANALOG_FLAT); parity subset first, then rocprof kernel
# stats per setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or multichunk or front1" > gpurun_out/g16_tests.log 2>&1 || exit 1
for v in "2 1" "4 1"; do
  set -- $v
  AMX_G16_PARTS=$1 AMX_ANALOG_FLAT=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/g16_$1_$2 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs > gpurun_out/g16_$1_$2.log 2>&1 || exit 1
done
