# round 4 end-of-round set: the whole GPU suite, smoke, the default bench line, kernel stats
# of the C3 step (linear) and of C3 in loudnorm dynamic mode
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04o_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04o_smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r04o_bench_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04o_prof_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o_prof_c3dyn -o run --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 5 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04o_prof_c3dyn.log 2>&1
