# round 6: k_decide's sequential bin sums read 8 terms per LDS round trip (new) against the
# tree before (base) -- the loudness / parity tests, then the C2 and C3 step A/B and profiles
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_ebu.py tests/test_gpu_fullsize.py > gpurun_out/r06ak_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06ak_summary.txt
for v in base new base new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  for c in c2 c3; do
    AMX_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 1500 --warmup 3 --soak 0 \
      --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ak_${c}_$v.log 2>&1 || exit 1
    echo "$c $v $(tail -1 gpurun_out/r06ak_${c}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'].get('decide'))")" >> gpurun_out/r06ak_summary.txt
  done
done
for v in base new; do
  if [ "$v" = new ]; then lib=""; else lib="$GRAFT_REPO_ROOT/audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  cd /tmp && AMX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ak_prof_$v -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --no-other-configs --no-cpu-baseline --no-pipeline --steps 300 --soak 0 > $GRAFT_REPO_ROOT/gpurun_out/r06ak_prof_$v.log 2>&1 || exit 1
done
