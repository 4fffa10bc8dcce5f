# round 6: per-frame times of k_lp_seg after the range emit
# counters (libamx_lpprof), on the current tree
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_lptime.so timeout -k 10 300 python -u scripts/lp_seg_times.py > gpurun_out/r06am_seg_times.txt 2>&1 || exit 1
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_lpprof.so timeout -k 10 300 python bench.py --config c3 --input dynamic \
  --steps 1 --warmup 0 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06am_lpprof_raw.log 2>&1
grep LPPROF gpurun_out/r06am_lpprof_raw.log | tail -8400 > gpurun_out/r06am_lpprof.txt
