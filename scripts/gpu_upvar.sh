#!/bin/bash
# Kernel variants: library builds in audio-mastering-engine_amd/lib_var/ (libamx_<name>.so)
# x 192 kHz K segment length.  VARIANTS="name:lout name:lout ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
for v in ${VARIANTS:-v1:480}; do
  name=${v%%:*}; lout=${v##*:}
  AMX_LIB=$PWD/audio-mastering-engine_amd/lib_var/libamx_$name.so AMX_UP_LOUT=$lout timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/upvar_${name}_$lout -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/upvar_${name}_$lout.log 2>&1 || echo "$name rc=$?"
done
