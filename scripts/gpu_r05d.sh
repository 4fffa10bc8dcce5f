# round 5: skip test without flags (margin), vectorized k_lp_fill; dynamic tests; C3 dynamic
# kernel stats; C2 force-exchange kernel trace (where the N>1 step's extra time goes)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dynamic.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1 || exit 1
B="bench.py --config c3 --input dynamic --steps 6 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05d_prof -o dyn --output-format csv -- python3 $B > gpurun_out/r05d_prof_dyn.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05d_prof -o c2fx --output-format csv -- python3 bench.py --config c2 --force-exchange --steps 30 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05d_prof_c2fx.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05d_prof -o c2 --output-format csv -- python3 bench.py --config c2 --steps 30 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05d_prof_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05d_bench_c3_dyn.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c5 --strong --input dynamic --steps 10 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05d_bench_c5s_dyn.log 2>&1
