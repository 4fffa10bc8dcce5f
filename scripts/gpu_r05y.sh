# round 5: envelope fix-up as parallel chains (k_envheads + k_envchain) -- parity, C3 / C4 / C5 timing, C4 full size
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fixup_paths or active_bands or golden or multichunk" > gpurun_out/r05y_tests.log 2>&1 || exit 1
for cfg in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05y_${cfg}.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 500 --timeout-method thread -k c4 > gpurun_out/r05y_fullsize_c4.log 2>&1 || exit 1
