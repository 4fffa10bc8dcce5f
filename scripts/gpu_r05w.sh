# round 5: SQ counters of k_xrms (separate --pmc passes)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
CMD="python3 bench.py --config c3 --steps 2 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
timeout -k 10 120 rocprofv3 --kernel-include-regex k_xrms --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/r05w_sq -o run --output-format csv -- $CMD > gpurun_out/r05w_sq.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-include-regex k_xrms --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/r05w_lds -o run --output-format csv -- $CMD > gpurun_out/r05w_lds.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-include-regex k_xrms --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_FLAT SQ_INSTS_BRANCH -d gpurun_out/r05w_act -o run --output-format csv -- $CMD > gpurun_out/r05w_act.log 2>&1 || exit 1
