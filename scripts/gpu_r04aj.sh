# round 4: kernel stats of the C2 and C5 steps on the final tree
set -o pipefail
export TMPDIR=/tmp
for cfg in c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04aj_prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04aj_prof_$cfg.log 2>&1 || exit 1
done
