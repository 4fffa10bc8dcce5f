# round 5 end (final tree, envelope step unified): whole GPU suite, PMC traffic (C3, C4), smoke, default bench, its rocprofv3 summary
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05as_gpu_tests.log 2>&1 || exit 1
for c in c3; do CFG=$c bash scripts/gpu_traffic.sh || exit 1; cp gpurun_out/traffic_$c.json profiles/traffic_$c.json; done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05as_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r05as_bench_default.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05as_prof -o c3 --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05as_prof.log 2>&1 || exit 1
