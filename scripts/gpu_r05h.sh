# round 5: fused carry+peaks exchange kernel; slot restore after pipelined replay; traces of the fx step
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "rccl or two_ranks" > gpurun_out/r05h_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 300 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05h_bench_c3_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --force-exchange --steps 400 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05h_bench_c2_fx.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r05h_prof -o c2fx --output-format csv -- python3 bench.py --config c2 --force-exchange --steps 31 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05h_prof_c2fx.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r05h_prof -o c2 --output-format csv -- python3 bench.py --config c2 --steps 31 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05h_prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05h_prof -o c3dyn --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05h_prof_c3dyn.log 2>&1
