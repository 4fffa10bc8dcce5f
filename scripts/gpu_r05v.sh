# round 5: k_xrms (crossover pass 2 + rms fused) -- parity, C3 A/B against the split kernels, profile
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "xrms or active_bands or multichunk or golden or fixup_paths" > gpurun_out/r05v_tests.log 2>&1 || exit 1
B="--config c3 --steps 200 --warmup 10 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
timeout -k 10 300 python bench.py $B > gpurun_out/r05v_c3.log 2>&1 || exit 1
AMX_XRMS=0 timeout -k 10 300 python bench.py $B > gpurun_out/r05v_c3_split.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05v_c3_b.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05v_prof -o c3 --output-format csv -- python3 bench.py --config c3 --steps 50 --warmup 5 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05v_prof.log 2>&1 || exit 1
