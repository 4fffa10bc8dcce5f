# round 4: the sharded dynamic mode's quiet-start fallback (2 gloo ranks on one GPU)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "dynamic" > gpurun_out/r04ah_dist_dynamic.log 2>&1
