# round 6: k_lp_fill with 8 positions per thread (new) against 4 (base = the previous commit) -- dynamic
# tests, then the C3 dynamic step A/B and the per-kernel profile
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py tests/test_gpu_dist.py > gpurun_out/r06au_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06au_summary.txt
for v in base new base new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  AMX_LIB=$lib timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06au_dyn_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r06au_dyn_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['ms_per_step'], s['ln_filter1'], s['ln_filter2'])")" >> gpurun_out/r06au_summary.txt
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06au_prof -o dyn -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --input dynamic --no-other-configs --no-cpu-baseline --no-pipeline --steps 40 --warmup 3 --soak 0 > $GRAFT_REPO_ROOT/gpurun_out/r06au_prof.log 2>&1
