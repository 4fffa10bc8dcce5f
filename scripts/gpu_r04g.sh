# round 4: sharded dynamic mode tests + the whole suite, then k_up_poly with / without
# the one-output-ahead row loads (AMX_UP_PF) at 44.1 kHz: kernel stats and step times
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dynamic.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04g_gpu_dyn.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04g_gpu_tests.log 2>&1
rc=$?
for name in base pf0; do
  lib=""
  [ "$name" != base ] && lib=$PWD/audio-mastering-engine_amd/lib_var/libamx_$name.so
  AMX_LIB=$lib timeout -k 10 300 python scripts/rate_probe.py --rates 44100,48000 > gpurun_out/r04g_rate_$name.log 2>&1 || exit 1
  AMX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_prof_$name -o run --output-format csv -- python3 scripts/rate_probe.py --rates 44100 > gpurun_out/r04g_prof_$name.log 2>&1 || exit 1
done
exit $rc
