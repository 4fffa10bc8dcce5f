# round 5: pipelined two-slot N>1 replay, windowed sharded dynamic mode, fill pre-pass tests;
# k_lp_seg phase costs from measurement variants (rocprofv3 kernel stats)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dynamic.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r05c_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 300 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05c_bench_c3_fx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --force-exchange --steps 400 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05c_bench_c2_fx.log 2>&1 || exit 1
B="bench.py --config c3 --input dynamic --steps 6 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_prof_dyn -o base --output-format csv -- python3 $B > gpurun_out/r05c_prof_base.log 2>&1 || exit 1
for v in nosnap noemit nodetect; do
  AMX_LIB=$PWD/audio-mastering-engine_amd/lib_var/libamx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_prof_dyn -o $v --output-format csv -- python3 $B > gpurun_out/r05c_prof_$v.log 2>&1 || exit 1
done
AMX_LP_FILL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_prof_dyn -o nofill --output-format csv -- python3 $B > gpurun_out/r05c_prof_nofill.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_prof_dyn -o c5 --output-format csv -- python3 bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05c_prof_c5.log 2>&1
