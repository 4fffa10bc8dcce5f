#!/bin/bash
# k_env0 at 2 and 4 waves per CU (AMX_ENV_WG): kernel trace + three PMC passes each
# (wave issue / waits; LDS, VMEM and TA; icache and fp64 instruction mix), summarised
# per kernel into gpurun_out/envwg_<wg>_summary.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 bench.py --config c3 --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs"
for WG in ${WGS:-2 4}; do
  export AMX_ENV_WG=$WG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/envwg_${WG}_trace -o run --output-format csv -- $CMD \
      > gpurun_out/envwg_${WG}_trace.log 2>&1 || exit $?
  P=0
  for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM TA_TA_BUSY" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"; do
    P=$((P + 1))
    timeout -s KILL 120 rocprofv3 --pmc $SET -d gpurun_out/envwg_${WG}_pmc$P -o run --output-format csv -- $CMD \
        > gpurun_out/envwg_${WG}_pmc$P.log 2>&1 || exit $?
  done
  python3 scripts/pmc_summary.py gpurun_out/envwg_${WG}_pmc1/run_counter_collection.csv \
      gpurun_out/envwg_${WG}_pmc2/run_counter_collection.csv gpurun_out/envwg_${WG}_pmc3/run_counter_collection.csv \
      > gpurun_out/envwg_${WG}_summary.txt 2>&1
  grep -E "k_env0|k_gain|k_front1" gpurun_out/envwg_${WG}_summary.txt | cut -c1-600
  grep -E "k_env0" gpurun_out/envwg_${WG}_trace/run_kernel_stats.csv
done
