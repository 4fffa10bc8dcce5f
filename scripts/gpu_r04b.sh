# round 4: k_env0 layouts on realistic bands (env_mb2), k_env0t parity and C3 timing
# against k_env0, then the parity tests the first pass did not reach
set -o pipefail
python scripts/env_mb_data.py /tmp/env_mb_data.bin > gpurun_out/env_mb2.txt 2>&1 && \
timeout -k 10 200 ./scripts/env_mb2.bin /tmp/env_mb_data.bin >> gpurun_out/env_mb2.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_compressor_row_tiled_speculation > gpurun_out/r04b_env0t.log 2>&1 && \
for RK in 0 2 4; do
  AMX_ENV_RK=$RK timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-other-configs --no-pipeline --soak 1 > gpurun_out/r04b_bench_rk$RK.log 2>&1 || exit 1
done && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dynamic.py::test_graph_step_dynamic_gate_linear_batch \
  tests/test_gpu_dynamic.py::test_graph_step_with_dynamic \
  "tests/test_gpu_dist.py::test_two_ranks_match_one[dynamic]" \
  tests/test_gpu_parity.py::test_front1_variants_vs_oracle \
  tests/test_gpu_dynamic.py::test_filter_300s_vs_oracle > gpurun_out/r04b_tests.log 2>&1
