# round 6: k_gain_overlay variants (AMX_GO_V bits: 1 checkpoint before the next band's
# loads, 2 unconditional r rows, 4 scalar plan tables) and the persistent k_rms (rms0:
# one tile per workgroup) on C3, same box; then the golden / parity tests on the new library
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in go0 go1 go2 go4 rms0 new go0 rms0 new; do
  if [ "$v" = new ]; then lib=""; else lib="audio-mastering-engine_amd/lib_var/libamx_$v.so"; fi
  AMX_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 300 --warmup 10 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06l_c3_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r06l_c3_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms']['rms'], d['stages_ms']['apply'])")" >> gpurun_out/r06l_summary.txt
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multichannel.py > gpurun_out/r06l_parity.log 2>&1
