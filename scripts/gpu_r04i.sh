# round 4: k_env0l with a batched table fill -- C3 bench at 2 / 4 waves per CU + kernel stats
set -o pipefail
for cfg in "1 2" "1 4"; do
  set -- $cfg
  AMX_ENV_LDS=$1 AMX_ENV_WG=$2 timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-other-configs --no-pipeline --soak 1 > gpurun_out/r04i_bench_lds$1_wg$2.log 2>&1 || exit 1
done
AMX_ENV_LDS=1 AMX_ENV_WG=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i_prof_env0l -o run --output-format csv -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-other-configs --no-pipeline --soak 0.2 > gpurun_out/r04i_prof_env0l.log 2>&1
