# round 4: k_env0l (the compressor's m table in LDS) -- parity with it forced on, then
# the C3 bench with k_env0 / k_env0l at 2 and 4 waves per CU
set -o pipefail
AMX_ENV_LDS=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "golden or fixup or multichunk or pipeline_vs_oracle or full_size" > gpurun_out/r04h_env0l_parity.log 2>&1 || exit 1
for cfg in "0 2" "1 2" "1 4"; do
  set -- $cfg
  AMX_ENV_LDS=$1 AMX_ENV_WG=$2 timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-other-configs --no-pipeline --soak 1 > gpurun_out/r04h_bench_lds$1_wg$2.log 2>&1 || exit 1
done
AMX_ENV_LDS=1 AMX_ENV_WG=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04h_prof_env0l -o run --output-format csv -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-other-configs --no-pipeline --soak 0.2 > gpurun_out/r04h_prof_env0l.log 2>&1
