# round 6: k_lp_seg's workgroup budget P (AMX_LN_P; the plan's Fs follows it) -- more,
# shorter segments than the three-waves-per-SIMD budget, the extra workgroups dispatched as
# early ones finish; C3 dynamic and C5 strong dynamic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/r06ao_summary.txt
run() {  # name env config-args
  env $2 timeout -k 10 300 python bench.py $3 --input dynamic --steps 20 --warmup 3 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06ao_$1.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/r06ao_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'), (d.get('dynamic') or {}).get('reruns'))")" >> gpurun_out/r06ao_summary.txt
}
for r in 1 2; do
  run c3_p768 AMX_LN_P=768 "--config c3" || exit 1
  run c3_p1024 AMX_LN_P=1024 "--config c3" || exit 1
  run c3_p1536 AMX_LN_P=1536 "--config c3" || exit 1
  run c3_p2048 AMX_LN_P=2048 "--config c3" || exit 1
done
run c5s_p768 AMX_LN_P=768 "--config c5 --strong" || exit 1
run c5s_p1536 AMX_LN_P=1536 "--config c5 --strong" || exit 1
run c5s_p3072 AMX_LN_P=3072 "--config c5 --strong" || exit 1
