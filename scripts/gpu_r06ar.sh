# round 6: k_lp_seg's warm-up frames per segment (AMX_LN_WARM 2 = the default, 1, 3) over
# track lengths (C3 settings, dynamic input) and C5 strong dynamic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/r06ar_summary.txt
run() {  # name env args
  env $2 timeout -k 10 300 python bench.py $3 --input dynamic --steps 10 --warmup 2 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ar_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06ar_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'))")" >> gpurun_out/r06ar_summary.txt
}
for s in 120 300 600 1200; do
  for w in 2 1 3; do run w${w}_$s AMX_LN_WARM=$w "--config c3 --seconds $s" || exit 1; done
done
for w in 2 1 3; do run c5s_w$w AMX_LN_WARM=$w "--config c5 --strong" || exit 1; done
