# round 5 end: PMC traffic per config (separate FETCH_SIZE / WRITE_SIZE passes), smoke, the default bench,
# its rocprofv3 summary, C3 in dynamic mode
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c3 c2 c4 c5; do CFG=$c bash scripts/gpu_traffic.sh || exit 1; done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ae_smoke.log 2>&1 || exit 1
for c in c3 c2 c4 c5; do cp gpurun_out/traffic_$c.json profiles/traffic_$c.json; done
timeout -k 10 900 python -u bench.py > gpurun_out/r05ae_bench_default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ae_prof -o c3 --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ae_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ae_c3_dyn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c5 --strong --input dynamic --steps 10 --warmup 2 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ae_c5_dyn.log 2>&1 || exit 1
