# round 4: k_ln_up_static with packed dots, k_lp_stats 4 frames per workgroup: dynamic tests, C3 dynamic bench + kernel stats
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread -k "dynamic or rates" > gpurun_out/r04u_dyn_tests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04u_dyn_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u_prof_c3dyn -o run --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 5 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04u_prof_c3dyn.log 2>&1
