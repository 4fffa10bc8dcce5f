#!/bin/bash
# Round-3 GPU steps: named test selections and scripts, each under its own time limit,
# logs under gpurun_out/r03_<name>.log; stops at the first failure.
#   STEPS="dyn dynbench" bash scripts/gpu_r03.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
run() {   # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
    local rc=$?
    echo "${name} rc=$rc"
    tail -3 gpurun_out/${TAG}_${name}.log
    return $rc
}
PYT="python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread"
for s in ${STEPS}; do
  case $s in
    dyn)      run dyn 900 $PYT tests/test_gpu_dynamic.py || exit $? ;;
    dynfast)  run dynfast 600 $PYT tests/test_gpu_dynamic.py -k "splits or filter_vs" || exit $? ;;
    dropnew)  run dropnew 600 $PYT tests/test_gpu_dropin.py -k "rates or 192k" || exit $? ;;
    dyn300)   run dyn300 900 $PYT tests/test_gpu_dynamic.py -k "300s" || exit $? ;;
    dynbench) run dynbench 300 python scripts/dyn_bench.py --seconds 300 --reps 3 --cpu-seconds 10 || exit $? ;;
    tests)    run tests 1100 $PYT tests -m gpu || exit $? ;;
    smoke)    run smoke 300 python __graft_entry__.py smoke || exit $? ;;
    bench)    run bench_${CFG:-c3} 400 python bench.py --config ${CFG:-c3} ${BENCH_ARGS} || exit $? ;;
    prof)     run prof_${CFG:-c3} 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_${CFG:-c3} -o run --output-format csv -- \
                  python3 bench.py --config ${CFG:-c3} --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs || exit $? ;;
    flops)    CFG=${CFG:-c3} bash scripts/gpu_flops.sh && echo "flops done" || exit $? ;;
    traffic)  CFG=${CFG:-c3} bash scripts/gpu_traffic.sh && echo "traffic done" || exit $? ;;
    rehearse) run rehearse_${CFG:-c5} 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NR:-4} \
                  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus ${NR:-4} --config ${CFG:-c5} \
                  ${BENCH_ARGS} --dist-backend gloo --one-device --no-cpu-baseline --no-pipeline || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
