# round 6: the boundary records' hand-off (AMX_LP_HANDOFF: sc1 record stores, one relaxed
# agent count, one acquire; hand0 = the __threadfence form) -- dynamic + dist tests, the
# C3 dynamic step A/B, and the per-segment phase times (libamx_lptime, rebuilt on this tree)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py tests/test_gpu_dist.py > gpurun_out/r06u_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06u_summary.txt
for v in hand0 new hand0 new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  AMX_LIB=$lib timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06u_dyn_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r06u_dyn_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['ms_per_step'], s['ln_filter1'], s['ln_filter2'])")" >> gpurun_out/r06u_summary.txt
done
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_lptime.so timeout -k 10 300 python -u scripts/lp_seg_times.py > gpurun_out/r06u_seg_times.txt 2>&1
