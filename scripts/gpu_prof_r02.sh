#!/bin/bash
# Round-2 profile of one config: kernel trace + stats, then separate PMC passes
# (SQ wave states, TA/LDS, FETCH_SIZE, WRITE_SIZE).  Never mixes counters and traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-r02_$CFG}
CMD="python3 bench.py --config $CFG --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- $CMD > gpurun_out/prof_${TAG}.log 2>&1 || exit $?
run() {
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?
  echo "rc=$rc" >> gpurun_out/pmc_${TAG}_$name.log
  return $rc
}
[ -n "$NO_PMC" ] && exit 0
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES && \
run ta TA_BUSY_avr TA_BUSY_max SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE
