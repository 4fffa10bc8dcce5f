#!/bin/bash
# k_env0 with the m table in LDS: GPU suite, then a placement sweep (VARIANTS of
# "lds:wg:lemin") as rocprof kernel stats + bench lines, C3 unless CFGS says otherwise
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-envlds}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
  echo "tests ok"
fi
for cfg in ${CFGS:-c3}; do
  for v in ${VARIANTS:-1:4:1024 1:4:512 1:2:1024 0:2:1024}; do
    IFS=: read lds wg lemin <<< "$v"
    AMX_ENV_LDS=$lds AMX_ENV_WG=$wg AMX_ENV_LEMIN=$lemin timeout -k 10 200 \
      rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${cfg}_${lds}_${wg}_${lemin} -o run --output-format csv -- \
      python3 bench.py --config $cfg --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/${TAG}_${cfg}_${lds}_${wg}_${lemin}.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    echo "$cfg $v done"
  done
done
