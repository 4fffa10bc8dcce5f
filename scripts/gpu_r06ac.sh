# round 6: k_lp_fill -- the partial frame's division under its branch (new) against the
# unconditional one (lpf0), and the grid at 65 536 workgroups (lpfg); C3 dynamic step
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py -k "not shard" > gpurun_out/r06ac_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06ac_summary.txt
for v in lpf0 new lpfg lpf0 new lpfg; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  AMX_LIB=$lib timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ac_dyn_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r06ac_dyn_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['ms_per_step'], s['ln_filter1'], s['ln_filter2'])")" >> gpurun_out/r06ac_summary.txt
done
for v in lpf0 lpfg; do
  cd /tmp && AMX_LIB=$GRAFT_REPO_ROOT/audio-mastering-engine_amd/lib_var/libamx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ac_prof_$v -o dyn -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --input dynamic --no-other-configs --no-cpu-baseline --no-pipeline --steps 20 --warmup 3 --soak 0 > $GRAFT_REPO_ROOT/gpurun_out/r06ac_prof_$v.log 2>&1 || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ac_prof_new -o dyn -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --input dynamic --no-other-configs --no-cpu-baseline --no-pipeline --steps 20 --warmup 3 --soak 0 > $GRAFT_REPO_ROOT/gpurun_out/r06ac_prof_new.log 2>&1
