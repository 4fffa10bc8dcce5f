# round 5: optimistic parallel re-run pass + chains -- parity, C3 / C4 / C5 / C3 dynamic timing
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dynamic.py -x -v --timeout 200 --timeout-method thread -k "fixup_paths or active_bands or golden or multichunk or filter or quiet" > gpurun_out/r05ab_tests.log 2>&1 || exit 1
for cfg in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ab_${cfg}.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ab_c3_dyn.log 2>&1 || exit 1
