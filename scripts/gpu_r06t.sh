# round 6: k_lp_seg phase times per segment (libamx_lptime)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_lptime.so timeout -k 10 300 python -u scripts/lp_seg_times.py > gpurun_out/r06t_seg_times.txt 2>&1
