# round 6: k_gain_overlay's prefetch kept in flight (checkpoint before the next band's
# loads, unconditional r rows, scalar plan-table reads) -- parity, then C3 / C4 / C5 and
# the C3 kernel profile; the previous library (libamx_old: round-6 HEAD before the
# prefetch work) once more on C3 beside it
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multichannel.py \
  > gpurun_out/r06k_parity.log 2>&1 || exit 1
for cfg in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 5 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06k_${cfg}.log 2>&1 || exit 1
done
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_old.so timeout -k 10 300 python bench.py --config c3 --steps 400 --warmup 10 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06k_c3_old.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 400 --warmup 10 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06k_c3_new.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06k_prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --no-other-configs --no-cpu-baseline --no-pipeline --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r06k_prof.log 2>&1
