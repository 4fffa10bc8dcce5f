# round 4: lp_detect's load-ahead depth (AMX_LP_PD 4 in-tree, 6 / 8 variant builds): C3 / C5 dynamic bench
set -o pipefail
for name in base pd6 pd8; do
  lib=""
  [ "$name" != base ] && lib=$PWD/audio-mastering-engine_amd/lib_var/libamx_$name.so
  AMX_LIB=$lib timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04x_dyn_c3_$name.log 2>&1 || exit 1
  AMX_LIB=$lib timeout -k 10 400 python bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline > gpurun_out/r04x_dyn_c5_$name.log 2>&1 || exit 1
done
