# round 6: prefetch waits (late tile masks, 3-deep analog pipeline) -- parity on the new
# library, then C3 / C2 timing A/B against the variant builds on the same box
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multichannel.py -k "golden or multichunk or analog or chain or fixup or active" \
  > gpurun_out/r06j_parity.log 2>&1 || exit 1
for v in new old vt0 an2 new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  for cfg in c3 c2; do
    AMX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 400 --warmup 10 --soak 0 \
      --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06j_${cfg}_$v.log 2>&1 || exit 1
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06j_prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r06j_prof.log 2>&1
