# round 4: the sharded dynamic mode (segment hand-off, 192 kHz measurement and alimiter over the ranks), then the whole suite
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dynamic.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04f_gpu_dyn.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04f_gpu_tests.log 2>&1
