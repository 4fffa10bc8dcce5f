# round 4: k_ln_up_static (the M == 1 rates' 192 kHz stream for the dynamic-mode filter):
# dynamic-mode parity, then the C3 dynamic step over segment shapes (AMX_LN_SEG frames per
# segment, AMX_LN_WARM warm-up frames, AMX_LN_P persistent waves)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread -k "dynamic or rates" > gpurun_out/r04m_dyn_tests.log 2>&1 || exit 1
for cfg in "4 3 1024" "3 2 1024" "4 2 1024" "3 1 1024" "2 2 2048" "2 1 2048" "1 1 4096"; do
  set -- $cfg
  AMX_LN_SEG=$1 AMX_LN_WARM=$2 AMX_LN_P=$3 timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04m_dyn_seg$1_warm$2_p$3.log 2>&1 || exit 1
done
