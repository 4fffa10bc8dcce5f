# round 4: SQ counters of the dynamic-mode filter kernels after the branch-free lp_val (C3 --input dynamic), two passes
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/r04s_dyn_sq -o run --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 2 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04s_dyn_sq.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d gpurun_out/r04s_dyn_lds -o run --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 2 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04s_dyn_lds.log 2>&1
