#!/bin/bash
# front1 at C3 (measurements): k_analog_h per chunk (AMX_ANALOG_FLAT=0) against the one
# block sequence over all chunks (default); parity subset first, then rocprof kernel
# stats per setting.  (The k_gemv16 variants DESIGN §3.4 lists were builds of this
# round's history.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or multichunk or front1" > gpurun_out/g16_tests.log 2>&1 || exit 1
for v in 0 1; do
  AMX_ANALOG_FLAT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/analog_flat_$v -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs > gpurun_out/analog_flat_$v.log 2>&1 || exit 1
done
