# round 6: k_lp_seg lanes per segment against the plan's P -- C3 dynamic (256 lanes = new,
# 512 at P 384 / 256 / 512, 1024 at P 192) and C5 strong dynamic (256, 512)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/r06ae_summary.txt
run() {  # name lib extra-env config-args
  env AMX_LIB=$2 $3 timeout -k 10 300 python bench.py $4 --input dynamic --steps 20 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ae_dyn_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06ae_dyn_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'))")" >> gpurun_out/r06ae_summary.txt
}
V=audio-mastering-engine_amd/lib_var
run c3_nt1024 $V/libamx_nt1024.so "" "--config c3" || exit 1
for r in 1 2; do
  run c3_new "" "" "--config c3" || exit 1
  run c3_nt512 $V/libamx_nt512.so "" "--config c3" || exit 1
  run c3_nt512p256 $V/libamx_nt512.so AMX_LN_P=256 "--config c3" || exit 1
  run c3_nt512p512 $V/libamx_nt512.so AMX_LN_P=512 "--config c3" || exit 1
  run c3_nt1024 $V/libamx_nt1024.so "" "--config c3" || exit 1
done
run c5s_new "" "" "--config c5 --strong" || exit 1
run c5s_nt512 $V/libamx_nt512.so "" "--config c5 --strong" || exit 1
run c5s_nt512p768 $V/libamx_nt512.so AMX_LN_P=768 "--config c5 --strong" || exit 1
