#!/bin/bash
# k_env0 variants on one config: "guess:warm:wg[:il[:lemin]]" (AMX_ENV_GUESS, --env-warm,
# AMX_ENV_WG, AMX_ENV_IL, AMX_ENV_LEMIN), each a bounded bench run without the CPU leg;
# then one line per run with ms/step, the env / fix stage times and the fix-up counters.
#   VARIANTS="1:2304:2 1:1792:2 0:2304:2" CFG=c3 bash scripts/gpu_envsweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
for V in ${VARIANTS:-1:2304:2}; do
  IFS=: read G W WG IL LM <<< "$V"
  log=gpurun_out/envsweep_${CFG}_${G}_${W}_${WG}_${IL:-0}_${LM:-1024}.log
  AMX_ENV_GUESS=$G AMX_ENV_WG=$WG AMX_ENV_IL=${IL:-0} AMX_ENV_LEMIN=${LM:-1024} timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 \
      --no-cpu-baseline --no-pipeline --no-other-configs --env-warm $W > $log 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "$V rc=$rc"; tail -5 $log; exit $rc; }
  python3 - "$log" "$V" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
st = d["stages_ms"]
print("%-12s ms/step %.4f  env %.4f  fix %.4f  fixup %s" % (sys.argv[2], d["ms_per_step"], st["env"], st["fix"],
      json.dumps(d.get("env_fixup"))))
EOF
done
