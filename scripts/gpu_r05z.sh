# round 5: k_envchain grid 1024 / 2048 (product) / 4096 waves at C3 / C5; C3 dynamic with the round's chain changes
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cfg in c3 c5; do
  B="--config $cfg --steps 30 --warmup 3 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
  timeout -k 10 300 python bench.py $B > gpurun_out/r05z_${cfg}_2048.log 2>&1 || exit 1
  AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_cw4096.so timeout -k 10 300 python bench.py $B > gpurun_out/r05z_${cfg}_4096.log 2>&1 || exit 1
  AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_cw1024.so timeout -k 10 300 python bench.py $B > gpurun_out/r05z_${cfg}_1024.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05z_c3_dyn.log 2>&1 || exit 1
