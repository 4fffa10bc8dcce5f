# round 4: k_env0 layouts on realistic bands (env_mb2), then the parity tests the first
# pass did not reach
set -o pipefail
python scripts/env_mb_data.py /tmp/env_mb_data.bin > gpurun_out/env_mb2.txt 2>&1 && \
timeout -k 10 200 ./scripts/env_mb2.bin /tmp/env_mb_data.bin >> gpurun_out/env_mb2.txt 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dynamic.py::test_graph_step_dynamic_gate_linear_batch \
  tests/test_gpu_dynamic.py::test_graph_step_with_dynamic \
  "tests/test_gpu_dist.py::test_two_ranks_match_one[dynamic]" \
  tests/test_gpu_parity.py::test_front1_variants_vs_oracle \
  tests/test_gpu_dynamic.py::test_filter_300s_vs_oracle > gpurun_out/r04b_tests.log 2>&1
