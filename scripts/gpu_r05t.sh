# round 5: the fix-up stage, HEAD library vs the active-band tables (same box, alternating)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
H=audio-mastering-engine_amd/lib_var/libamx_head.so
B="--config c3 --steps 200 --warmup 10 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05t_head1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05t_new1.log 2>&1 || exit 1
AMX_ENV_BANDTAB=0 timeout -k 10 300 python bench.py $B > gpurun_out/r05t_tab31.log 2>&1 || exit 1
AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05t_head2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05t_new2.log 2>&1 || exit 1
AMX_LIB=$H timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t_prof -o head --output-format csv -- python3 bench.py $B > gpurun_out/r05t_prof_head.log 2>&1 || exit 1
