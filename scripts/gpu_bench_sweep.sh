#!/bin/bash
# bench at several segment lengths (each run bounded), logs under gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${SEGS:-128 256}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --seg-frames $L ${BENCH_ARGS} > gpurun_out/bench_L$L.log 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/bench_L$L.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
