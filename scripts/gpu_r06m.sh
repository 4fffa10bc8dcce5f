# round 6: k_rms 2048-frame tiles at 48 / 44.1 kHz (rms4k: 4096) and the whole-quad
# k_analog_h (anv0: the general form) on C3, same box; parity and the dist tests on the
# new library (the N = 2 linear cases now also against the oracle)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/r06m_summary.txt
for v in rms4k anv0 new rms4k anv0 new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  AMX_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 300 --warmup 10 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06m_c3_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r06m_c3_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms']['front1'], d['stages_ms']['rms'])")" >> gpurun_out/r06m_summary.txt
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multichannel.py tests/test_gpu_dist.py > gpurun_out/r06m_tests.log 2>&1
