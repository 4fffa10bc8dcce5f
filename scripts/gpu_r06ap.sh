# round 6: AMX_LN_P 768 (the default) against 1024 over track lengths (C3 settings, dynamic
# input) and C5 strong dynamic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/r06ap_summary.txt
run() {  # name env args
  env $2 timeout -k 10 300 python bench.py $3 --input dynamic --steps 10 --warmup 2 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ap_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06ap_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'))")" >> gpurun_out/r06ap_summary.txt
}
for s in 120 240 420 600 900 1200; do
  run p768_$s AMX_LN_P=768 "--config c3 --seconds $s" || exit 1
  run p1024_$s AMX_LN_P=1024 "--config c3 --seconds $s" || exit 1
done
run c5s_p768 AMX_LN_P=768 "--config c5 --strong" || exit 1
run c5s_p1024 AMX_LN_P=1024 "--config c5 --strong" || exit 1
run c5s_p768b AMX_LN_P=768 "--config c5 --strong" || exit 1
run c5s_p1024b AMX_LN_P=1024 "--config c5 --strong" || exit 1
