# round 5: the default bench with the dominant kernel timed over back-to-back launches, next to its rocprofv3 summary
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py > gpurun_out/r05al_bench_default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05al_prof -o c3 --output-format csv -- python3 bench.py --no-other-configs --no-pipeline > gpurun_out/r05al_prof.log 2>&1 || exit 1
