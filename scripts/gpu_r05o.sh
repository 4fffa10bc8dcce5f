# round 5: k_ln_up_static over 4-frame blocks (one window, 16-B loads)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dropin.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "dynamic or above or fill or shard or window or parallel or filter or rates" > gpurun_out/r05o_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05o_bench_c3_dyn.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05o_prof -o c3dyn --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05o_prof_c3dyn.log 2>&1
