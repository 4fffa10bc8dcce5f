# round 4: k_gain_overlay with its checkpoint and r loads outside branches: compressor / golden
# parity, then the C3 bench and kernel stats
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "golden or fixup or multichunk or pipeline_vs_oracle or full_size or batch" > gpurun_out/r04z_parity.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-other-configs --no-pipeline --soak 1 > gpurun_out/r04z_bench_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04z_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04z_prof_c3.log 2>&1
