# round 5 end: SQ counters of the four largest C3 kernels (separate --pmc passes), for the next round's plan
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
CMD="python3 bench.py --config c3 --steps 2 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
R="k_up<4>|k_front2|k_gain_overlay|k_env0"
timeout -k 10 120 rocprofv3 --kernel-include-regex "$R" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/r05at_sq -o run --output-format csv -- $CMD > gpurun_out/r05at_sq.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-include-regex "$R" --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/r05at_lds -o run --output-format csv -- $CMD > gpurun_out/r05at_lds.log 2>&1 || exit 1
