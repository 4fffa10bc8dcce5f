# round 5: the envelope warm-up W re-tuned for the parallel fix-up (bench --env-warm), C3 / C4 / C5 / C3 dynamic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for w in 2304 1536 1024 768; do
  for cfg in c3 c4 c5; do
    timeout -k 10 300 python bench.py --config $cfg --env-warm $w --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ag_${cfg}_w$w.log 2>&1 || exit 1
  done
done
