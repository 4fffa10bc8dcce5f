# round 4: k_ln_up_static with the next window loaded ahead: the dynamic tests
# (oracle, sharded, graph steps) and the C3 / C5 dynamic bench
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dist.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04ai_dyn_tests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04ai_dyn_c3.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline > gpurun_out/r04ai_dyn_c5.log 2>&1
