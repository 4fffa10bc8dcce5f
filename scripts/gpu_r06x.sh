# round 6: the 192 kHz upsampler's outputs staged in LDS and written as contiguous
# blocks (AMX_LN_UPS_LDS; ups0 = direct per-thread stores) -- dynamic tests and the
# multichannel / parity tests that reach the upsampler, then the C3 dynamic step A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py > gpurun_out/r06x_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06x_summary.txt
for v in ups0 new ups0 new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  AMX_LIB=$lib timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06x_dyn_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r06x_dyn_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['ms_per_step'], s['ln_filter1'], s['ln_filter2'])")" >> gpurun_out/r06x_summary.txt
done
