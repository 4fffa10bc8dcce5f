# round 6: k_lp_seg at two waves per SIMD (AMX_LP_WPE 2: no spill) with 4 (w2e4) or 8 (w2e8)
# envelope groups per pass, against the default (new: 3 waves, 4 groups); C3 dynamic over
# track lengths and C5 strong dynamic; dynamic tests on w2e8 first
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=audio-mastering-engine_amd/lib_var
AMX_LIB=$V/libamx_w2e8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py -k "not shard" > gpurun_out/r06at_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06at_summary.txt
run() {  # name lib args
  AMX_LIB=$2 timeout -k 10 300 python bench.py $3 --input dynamic --steps 10 --warmup 2 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06at_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06at_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'))")" >> gpurun_out/r06at_summary.txt
}
for s in 120 300 600 1200; do
  run new_$s "" "--config c3 --seconds $s" || exit 1
  run w2e4_$s $V/libamx_w2e4.so "--config c3 --seconds $s" || exit 1
  run w2e8_$s $V/libamx_w2e8.so "--config c3 --seconds $s" || exit 1
done
run c5s_new "" "--config c5 --strong" || exit 1
run c5s_w2e4 $V/libamx_w2e4.so "--config c5 --strong" || exit 1
run c5s_w2e8 $V/libamx_w2e8.so "--config c5 --strong" || exit 1
