#!/bin/bash
# Round-2 full GPU pass: smoke + the whole GPU suite, the four bench configs, then per
# config a kernel-trace profile and the FETCH/WRITE traffic passes.  Stops at the first
# failure; every step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
run() {   # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
    local rc=$?
    echo "${name} rc=$rc"
    return $rc
}
if [ -z "$NO_TESTS" ]; then
  run smoke 300 python __graft_entry__.py smoke || exit $?
  run tests 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread ${PYTEST_ARGS} || exit $?
fi
for c in ${CONFIGS:-c3 c2 c4 c5}; do
  run bench_$c 400 python bench.py --config $c || exit $?
done
for c in ${PROF_CONFIGS:-c3 c2 c4 c5}; do
  run prof_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$c -o run --output-format csv -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline || exit $?
  CFG=$c bash scripts/gpu_traffic.sh || exit $?
  echo "traffic_$c done"
done
