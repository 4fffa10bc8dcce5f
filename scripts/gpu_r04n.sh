# round 4: the dynamic-mode filter's segment shape chosen by the plan (Fs from the track
# length, Wf 2, up to 2048 waves) against round 3's (Fs 4, Wf 3, 1024 waves): C3 and C5 strong
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamic.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "dynamic or parallel or quiet" > gpurun_out/r04n_dyn_tests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04n_dyn_c3_auto.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline > gpurun_out/r04n_dyn_c5_auto.log 2>&1 || exit 1
AMX_LN_SEG=4 AMX_LN_WARM=3 AMX_LN_P=1024 timeout -k 10 400 python bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline > gpurun_out/r04n_dyn_c5_r3shape.log 2>&1
