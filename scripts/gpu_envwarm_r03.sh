#!/bin/bash
# C3 ms per step against the envelope warm-up W (bench.py --env-warm), round-3 guess
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wu in ${WARMS:-1536 1792 2048 2304}; do
  timeout -k 10 200 python3 bench.py --config c3 --env-warm $wu --no-cpu-baseline --no-pipeline --no-other-configs > gpurun_out/envwarm_$wu.log 2>&1 || exit 1
  python3 -c "
import json,sys
d = json.loads([l for l in open('gpurun_out/envwarm_$wu.log') if l.startswith('{')][-1])
print($wu, d['ms_per_step'], d['stages_ms']['env'], d['stages_ms']['fix'], d['env_fixup'])
"
done
