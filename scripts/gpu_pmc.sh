#!/bin/bash
# PMC passes (one rocprofv3 run per counter group; never combined with traces).
# FETCH_SIZE on gfx950 reports 1/2 of the bytes of wide coalesced reads
# (MI355X_MICROARCH.md "HBM"): bench.py / DESIGN.md apply the x2 correction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?
  echo "rc=$rc" >> gpurun_out/pmc_${TAG}_$name.log
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
