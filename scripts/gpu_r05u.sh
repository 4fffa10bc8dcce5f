# round 5: isolate the fix-up stage's slowdown (HEAD / bitmask product / fix-up without band flags, 3-band table)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
H=audio-mastering-engine_amd/lib_var/libamx_head.so
V=audio-mastering-engine_amd/lib_var/libamx_fixb0.so
B="--config c3 --steps 200 --warmup 10 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05u_head.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05u_new.log 2>&1 || exit 1
AMX_ENV_BANDTAB=0 timeout -k 10 300 python bench.py $B > gpurun_out/r05u_tab3.log 2>&1 || exit 1
AMX_ENV_BANDTAB=0 AMX_LIB=$V timeout -k 10 300 python bench.py $B > gpurun_out/r05u_fixb0.log 2>&1 || exit 1
