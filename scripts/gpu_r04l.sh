# round 4: loudnorm dynamic mode's segment shape (AMX_LN_SEG frames per segment, AMX_LN_WARM
# warm-up frames) on the C3 dynamic-mode step
set -o pipefail
for cfg in "4 3" "2 3" "2 2" "3 2" "1 2"; do
  set -- $cfg
  AMX_LN_SEG=$1 AMX_LN_WARM=$2 timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04l_dyn_seg$1_warm$2.log 2>&1 || exit 1
done
