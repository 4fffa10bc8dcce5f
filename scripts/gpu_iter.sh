#!/bin/bash
# One iteration on the GPU: the GPU suite (unless NO_TESTS), then per config in CFGS a
# rocprof kernel-stats run and a bench line.  TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-iter}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  echo "tests ok: $(tail -1 gpurun_out/${TAG}_tests.log)"
fi
for cfg in ${CFGS:-c3 c2}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_${cfg} -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/${TAG}_prof_${cfg}.log 2>&1 || { echo "prof $cfg rc=$?"; exit 1; }
  timeout -k 10 300 python3 bench.py --config $cfg ${BENCH_ARGS} > gpurun_out/${TAG}_bench_${cfg}.log 2>&1 || { echo "bench $cfg rc=$?"; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/${TAG}_bench_${cfg}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["parity_vs_oracle"]["max_abs_lsb"], d["stages_ms"])')"
done
