# round 6: envelope groups per pass (AMX_LP_EG 4 = new, 6, 8) -- dynamic tests on eg8, then
# the C3 dynamic step and C5 strong dynamic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=audio-mastering-engine_amd/lib_var
AMX_LIB=$V/libamx_eg8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py -k "not shard" > gpurun_out/r06aj_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06aj_summary.txt
run() {  # name lib config-args
  AMX_LIB=$2 timeout -k 10 300 python bench.py $3 --input dynamic --steps 20 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06aj_dyn_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06aj_dyn_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'))")" >> gpurun_out/r06aj_summary.txt
}
for r in 1 2; do
  run c3_new "" "--config c3" || exit 1
  run c3_eg6 $V/libamx_eg6.so "--config c3" || exit 1
  run c3_eg8 $V/libamx_eg8.so "--config c3" || exit 1
done
run c5s_new "" "--config c5 --strong" || exit 1
run c5s_eg6 $V/libamx_eg6.so "--config c5 --strong" || exit 1
run c5s_eg8 $V/libamx_eg8.so "--config c5 --strong" || exit 1
