# round 5: single-graph N>1 step (RCCL captured), k_lp_fill + skipping scan + sparse emit,
# loudness-failure fallback; then the benches
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dist.py tests/test_gpu_dropin.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 200 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05b_bench_c3_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --force-exchange --steps 300 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05b_bench_c2_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 300 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05b_bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05b_bench_c3_dyn.log 2>&1 || exit 1
AMX_LP_FILL=0 timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05b_bench_c3_dyn_nofill.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r05b_bench_default.log 2>&1
