# round 5 checkpoint: the whole GPU suite, smoke, the default bench line, C3 dynamic profile
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05n_smoke.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r05n_bench_default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05n_prof -o c3dyn --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05n_prof_c3dyn.log 2>&1
