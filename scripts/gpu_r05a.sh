# round 5: baseline of the tree + RCCL hipGraph capture probe at world 1
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python scripts/rccl_capture_probe.py > gpurun_out/r05a_rccl_probe.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 200 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05a_bench_c3_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 200 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05a_bench_c3.log 2>&1 || exit 1
