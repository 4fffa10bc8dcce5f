#!/bin/bash
# C3 SQ wave-state and LDS / TA counters at the round-3 tree (one C3 bench step set, no
# other configs) -- separate --pmc runs, no traces mixed in
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03e_c3}
CMD="python3 bench.py --config c3 --steps 2 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_${TAG}_sq -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_sq.log 2>&1 || exit $?
echo "sq done"
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc_${TAG}_ta -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_ta.log 2>&1 || exit $?
echo "ta done"
