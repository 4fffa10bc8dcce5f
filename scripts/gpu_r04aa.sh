# round 4: k_up<L> with the C A^n rows loaded one output ahead: loudness / pipeline parity,
# C3 bench and kernel stats
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ebu.py \
  -k "loudness or pipeline or tp_decision or full_size or ebu or 3341 or 3342" > gpurun_out/r04aa_parity.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-other-configs --no-pipeline --soak 1 > gpurun_out/r04aa_bench_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04aa_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04aa_prof_c3.log 2>&1
