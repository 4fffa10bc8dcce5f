#!/bin/bash
# GPU-box check: smoke, GPU parity suite, a short bench.  Each GPU step has its
# own time limit; logs go to gpurun_out/ (merged back by gpurun).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc" >> gpurun_out/smoke.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc" >> gpurun_out/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc" >> gpurun_out/bench.log
exit $rc
