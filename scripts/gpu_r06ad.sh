# round 6: k_lp_seg at 512 lanes per segment (nt512: the plan's default P, Fs 9; nt512 with
# AMX_LN_P=768: Fs 5, 600 workgroups) against 256 lanes (new); nt512f adds k_lp_fill's
# 65 536-workgroup grid.  Dynamic tests on nt512 first
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_nt512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dynamic.py -k "not shard" > gpurun_out/r06ad_tests.log 2>&1 || exit 1
rm -f gpurun_out/r06ad_summary.txt
run() {  # name lib extra-env
  env AMX_LIB=$2 $3 timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 40 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ad_dyn_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06ad_dyn_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['ms_per_step'], s['ln_filter1'], s['ln_filter2'])")" >> gpurun_out/r06ad_summary.txt
}
V=audio-mastering-engine_amd/lib_var
for r in 1 2; do
  run new "" "" || exit 1
  run nt512 $V/libamx_nt512.so "" || exit 1
  run nt512p768 $V/libamx_nt512.so AMX_LN_P=768 || exit 1
  run nt512f $V/libamx_nt512f.so "" || exit 1
done
