# round 5: k_gain_overlay envelope step with the raw fp64 min against HEAD -- fix-up tests, C3 / C4 / C3 dynamic fix stage
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
H=audio-mastering-engine_amd/lib_var/libamx_head.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fixup_paths or golden or multichunk" > gpurun_out/r05ar_tests.log 2>&1 || exit 1
for cfg in c3 c4; do
  B="--config $cfg --steps 60 --warmup 5 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
  AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05ar_${cfg}_head.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $B > gpurun_out/r05ar_${cfg}_new.log 2>&1 || exit 1
done
B="--config c3 --input dynamic --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05ar_c3dyn_head.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05ar_c3dyn_new.log 2>&1 || exit 1
