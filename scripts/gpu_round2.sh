#!/bin/bash
# GPU-box check for round 2: smoke, the GPU test suite (incl. slow full-size tests),
# then the default bench (C3) and the C4 / C5 benches.  Each GPU step has its own
# time limit and the steps stop at the first failure; logs go to gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02}
run() {   # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
    local rc=$?
    echo "${name}_rc=$rc" >> gpurun_out/${TAG}_${name}.log
    echo "${name} rc=$rc"
    return $rc
}
run smoke 300 python __graft_entry__.py smoke || exit $?
run tests 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread ${PYTEST_ARGS} || exit $?
[ -n "$NO_BENCH" ] && exit 0
run bench_c3 300 python bench.py || exit $?
run bench_c4 300 python bench.py --config c4 --no-pipeline || exit $?
run bench_c5 400 python bench.py --config c5 --no-pipeline || exit $?
