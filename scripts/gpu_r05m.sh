# round 5: pass 2 reuses the frame statistics; the 192 kHz alimiter bound from the filter ceiling
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dropin.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "dynamic or above or fill or shard or window or parallel or filter or rccl or two_ranks or capture" > gpurun_out/r05m_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05m_bench_c3_dyn.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05m_prof -o c3dyn --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05m_prof_c3dyn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c5 --strong --input dynamic --steps 10 --warmup 2 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05m_bench_c5_dyn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --force-exchange --steps 400 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05m_bench_c2_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 300 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05m_bench_c3_fx.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05m_prof -o c2fx --output-format csv -- python3 bench.py --config c2 --force-exchange --steps 40 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05m_prof_c2fx.log 2>&1
