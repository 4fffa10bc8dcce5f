# round 5: k_lp_seg at 256 lanes per segment (variant build) against the 128-lane product
set -o pipefail
export TMPDIR=/tmp
V=audio-mastering-engine_amd/lib_var/libamx_nt256.so
AMX_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamic.py -x -v --timeout 300 --timeout-method thread -k "filter or parallel or quiet or final" > gpurun_out/r05p_nt256_tests.log 2>&1 || exit 1
AMX_LIB=$V timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05p_nt256_c3_dyn.log 2>&1 || exit 1
AMX_LIB=$V timeout -k 10 300 python bench.py --config c5 --strong --input dynamic --steps 10 --warmup 2 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05p_nt256_c5_dyn.log 2>&1 || exit 1
AMX_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05p_prof -o nt256 --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05p_prof_nt256.log 2>&1
