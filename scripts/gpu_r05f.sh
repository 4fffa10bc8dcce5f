# round 5: separate dynamic graph diagnostics; inputs above 192 kHz; fx benches
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python scripts/dyn_graph_probe2.py > gpurun_out/r05f_probe2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05f_prof -o probe2 --output-format csv -- python3 scripts/dyn_graph_probe2.py > gpurun_out/r05f_probe2_prof.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_dist.py -x -v --timeout 600 --timeout-method thread -k "above_192k or rates or 192k_dynamic or rccl or two_ranks" > gpurun_out/r05f_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 300 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05f_bench_c3_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --force-exchange --steps 400 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05f_bench_c2_fx.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05f_prof -o c2fx --output-format csv -- python3 bench.py --config c2 --force-exchange --steps 30 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05f_prof_c2fx.log 2>&1
