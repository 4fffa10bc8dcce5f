#!/bin/bash
# FLOPs per kernel launch for one bench config: one PMC pass of the 8 VALU FP counters
# (8 SQ counters: the per-pass limit), then gpurun_out/flops_<config>.json (copy it to
# profiles/ for bench.py's chain_flop_frac).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
CMD="python3 bench.py --config $CFG --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 \
    SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 \
    -d gpurun_out/pmc_${CFG}_flops -o run --output-format csv -- $CMD > gpurun_out/pmc_${CFG}_flops.log 2>&1 || exit $?
python3 scripts/pmc_flops.py gpurun_out/pmc_${CFG}_flops/run_counter_collection.csv gpurun_out/flops_${CFG}.json > gpurun_out/flops_${CFG}.txt 2>&1
