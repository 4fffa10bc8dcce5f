# round 5: k_peak_reduce with the slots reduced in parallel against HEAD -- tests, C3 / C2 A/B, profile
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
H=audio-mastering-engine_amd/lib_var/libamx_head.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ebu.py -x -q --timeout 200 --timeout-method thread -k "loudness or pipeline or tp_decision or ebu or batch or short" > gpurun_out/r05am_tests.log 2>&1 || exit 1
for cfg in c3 c2; do
  B="--config $cfg --steps 300 --warmup 20 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
  AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05am_${cfg}_head.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $B > gpurun_out/r05am_${cfg}_new.log 2>&1 || exit 1
  AMX_LIB=$H timeout -k 10 300 python bench.py $B > gpurun_out/r05am_${cfg}_head2.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $B > gpurun_out/r05am_${cfg}_new2.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05am_prof -o c3 --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05am_prof.log 2>&1 || exit 1
