# round 5: the 192 kHz measurement through the identity resampler (k_up<1>: one pass)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dropin.py tests/test_gpu_dist.py tests/test_gpu_ebu.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "dynamic or above or 192k or shard or window or parallel or filter or rates or sine or tp_decision or two_ranks or rccl" > gpurun_out/r05q_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05q_bench_c3_dyn.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05q_prof -o c3dyn --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05q_prof_c3dyn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c5 --strong --input dynamic --steps 10 --warmup 2 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05q_bench_c5_dyn.log 2>&1
