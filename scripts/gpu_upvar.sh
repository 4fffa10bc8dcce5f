#!/bin/bash
# 192 kHz kernel variants: library build (register budget, block) x K segment length.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-"w4t8 384" "w4t4 384" "w5t4 384" "w4t8 192" "w4t8 480"}; do
  set -- $v
  AMX_LIB=$PWD/audio-mastering-engine_amd/lib_var/libamx_$1.so AMX_UP_LOUT=$2 timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/upvar_$1_$2 -o run --output-format csv -- \
    python3 bench.py --config c3 --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/upvar_$1_$2.log 2>&1 || exit $?
done
