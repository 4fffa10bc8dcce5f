# round 4: k_gain_overlay with the gain chains interleaved (AMX_GO_ILP 2 / 4 variant
# libraries) against the in-tree build: C3 bench + the compressor / golden parity
set -o pipefail
for name in base go2 go4; do
  lib=""
  [ "$name" != base ] && lib=$PWD/audio-mastering-engine_amd/lib_var/libamx_$name.so
  AMX_LIB=$lib timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-other-configs --no-pipeline --soak 1 > gpurun_out/r04c_bench_$name.log 2>&1 || exit 1
done && \
AMX_LIB=$PWD/audio-mastering-engine_amd/lib_var/libamx_go4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "golden or fixup or pipeline_vs_oracle" > gpurun_out/r04c_go4_parity.log 2>&1 && \
AMX_LIB=$PWD/audio-mastering-engine_amd/lib_var/libamx_go2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "golden or fixup" > gpurun_out/r04c_go2_parity.log 2>&1
