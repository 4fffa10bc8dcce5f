# round 6: 256 (new) against 512 lanes per segment over track lengths (C3 settings, dynamic
# input): where the wider segment stops paying for its longer segments
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/r06af_summary.txt
run() {  # name lib seconds
  AMX_LIB=$2 timeout -k 10 300 python bench.py --config c3 --seconds $3 --input dynamic --steps 10 --warmup 2 --soak 0 \
    --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r06af_dyn_$1_$3.log 2>&1 || exit 1
  echo "$1 $3 $(tail -1 gpurun_out/r06af_dyn_$1_$3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stages_ms', {}); print(d['ms_per_step'], s.get('ln_filter1'), s.get('ln_filter2'))")" >> gpurun_out/r06af_summary.txt
}
V=audio-mastering-engine_amd/lib_var
for s in 120 240 420 600 900 1200; do
  run new "" $s || exit 1
  run nt512 $V/libamx_nt512.so $s || exit 1
done
