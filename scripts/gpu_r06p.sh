# round 6: per-frame counters of k_lp_seg (measurement build lpprof: device printf per
# frame -- detect calls, groups scanned, skip votes, serial steps, envelope slots, ticks)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_lpprof.so timeout -k 10 300 python bench.py --config c3 --input dynamic \
  --steps 1 --warmup 0 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06p_lpprof_raw.log 2>&1
grep LPPROF gpurun_out/r06p_lpprof_raw.log | tail -8000 > gpurun_out/r06p_lpprof.txt
