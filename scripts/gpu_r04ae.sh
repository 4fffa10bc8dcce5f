# round 4: the default bench line on the final tree (what the driver runs at round end)
set -o pipefail
timeout -k 10 500 python bench.py > gpurun_out/r04ae_bench_default.log 2>&1
