cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for cfg in c4 c5; do for wu in 2048 2304; do
  timeout -k 10 300 python3 bench.py --config $cfg --env-warm $wu --no-cpu-baseline --no-pipeline --no-other-configs > gpurun_out/envwarm_${cfg}_$wu.log 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/envwarm_${cfg}_$wu.log') if l.startswith('{')][-1])
print('$cfg', $wu, d['ms_per_step'], d['stages_ms'].get('env'), d['stages_ms'].get('fix'), d.get('env_fixup'))
"
done; done
