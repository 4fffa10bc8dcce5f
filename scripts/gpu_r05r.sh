# round 5: active-band envelope tables -- parity, then C3 A/B (AMX_ENV_BANDTAB=0 keeps the 3-band table)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="--config c3 --steps 300 --warmup 20 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "active_bands or fixup_paths or chain" > gpurun_out/r05r_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05r_c3.log 2>&1 || exit 1
AMX_ENV_BANDTAB=0 timeout -k 10 300 python bench.py $B > gpurun_out/r05r_c3_tab3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $B > gpurun_out/r05r_c3_b.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05r_prof -o c3 --output-format csv -- python3 bench.py --config c3 --steps 100 --warmup 5 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05r_prof.log 2>&1
