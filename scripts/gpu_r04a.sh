# round 4, first GPU pass: the k_env0 instruction-mix microbenchmark, then the new
# parity tests (RCCL forced exchange, 22.05 / 11.025 kHz loudnorm, dynamic mode
# chunk-sharded, the gated 192 kHz side plans)
set -o pipefail
timeout -k 10 120 ./scripts/env_mb.bin > gpurun_out/env_mb.txt 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dist.py::test_rccl_forced_exchange_world1 \
  "tests/test_gpu_parity.py::test_loudness_192k_rates_vs_oracle" \
  tests/test_gpu_dropin.py::test_master_audio_rates_inexact_192k_resampler \
  tests/test_gpu_dynamic.py::test_master_audio_dynamic \
  tests/test_gpu_dynamic.py::test_graph_step_dynamic_gate_linear_batch \
  tests/test_gpu_dynamic.py::test_graph_step_with_dynamic \
  "tests/test_gpu_dist.py::test_two_ranks_match_one[dynamic]" > gpurun_out/r04a_tests.log 2>&1
