# round 5: k_envfix segments per wave (64 product / 16 / 4 variants) -- fix-up tests, then C4 / C5 / C3 fix stage
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V16=audio-mastering-engine_amd/lib_var/libamx_spw16.so
V4=audio-mastering-engine_amd/lib_var/libamx_spw4.so
K="fixup_paths or active_bands"
AMX_LIB=$V16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/r05x_tests16.log 2>&1 || exit 1
AMX_LIB=$V4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/r05x_tests4.log 2>&1 || exit 1
for cfg in c4 c5 c3; do
  B="--config $cfg --steps 20 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
  timeout -k 10 300 python bench.py $B > gpurun_out/r05x_${cfg}_64.log 2>&1 || exit 1
  AMX_LIB=$V16 timeout -k 10 300 python bench.py $B > gpurun_out/r05x_${cfg}_16.log 2>&1 || exit 1
  AMX_LIB=$V4 timeout -k 10 300 python bench.py $B > gpurun_out/r05x_${cfg}_4.log 2>&1 || exit 1
done
