# round 5: re-run loop with loads two / three windows ahead -- parity, then W 2304 / 1536 / 1024 at C3 / C4 / C5 and C3 dynamic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fixup_paths or active_bands or golden or multichunk" > gpurun_out/r05ah_tests.log 2>&1 || exit 1
for w in 2304 1536 1024; do
  for cfg in c3 c4 c5; do
    timeout -k 10 300 python bench.py --config $cfg --env-warm $w --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ah_${cfg}_w$w.log 2>&1 || exit 1
  done
  timeout -k 10 300 python bench.py --config c3 --input dynamic --env-warm $w --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ah_c3dyn_w$w.log 2>&1 || exit 1
done
