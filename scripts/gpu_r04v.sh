# round 4: the shard entry points through the C ABI, ranks simulated in one process
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_dynamic.py -x -v --timeout 300 --timeout-method thread -k "shard_parts" > gpurun_out/r04v_shard_parts.log 2>&1
