# round 4: k_lp_seg at 3 waves per SIMD (168 VGPRs, spills) with one-frame segments and up to
# 3072 waves, against the in-tree 2-wave form: C3 / C5 dynamic bench
set -o pipefail
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env AMX_LIB=$lib "$@" timeout -k 10 240 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.3 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04af_c3_$name.log 2>&1 || return 1
  env AMX_LIB=$lib "$@" timeout -k 10 400 python bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline > gpurun_out/r04af_c5_$name.log 2>&1
}
V=$PWD/audio-mastering-engine_amd/lib_var/libamx_wpe3.so
run base "" && \
run wpe3_p3072 $V AMX_LN_P=3072 && \
run wpe3_seg1_p3072 $V AMX_LN_P=3072 AMX_LN_SEG=1 AMX_LN_WARM=2 && \
run base_seg1 "" AMX_LN_SEG=1 AMX_LN_WARM=2
