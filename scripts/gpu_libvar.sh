#!/bin/bash
# Library variants (audio-mastering-engine_amd/lib_var/libamx_<name>.so, "base" = the
# in-tree build): rocprof kernel stats of one config per variant.  VARIANTS="base name ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-libvar}
for name in ${VARIANTS:-base}; do
  lib=""
  [ "$name" != base ] && lib=$PWD/audio-mastering-engine_amd/lib_var/libamx_$name.so
  AMX_LIB=$lib timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${CFG}_$name -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-pipeline > gpurun_out/${TAG}_${CFG}_$name.log 2>&1 || { echo "$name rc=$?"; exit 1; }
  echo "$name done"
done
