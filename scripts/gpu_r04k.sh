# round 4: kernel stats of the C3 step (linear, the headline) and of C3 in loudnorm dynamic mode
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04k_prof_c3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_prof_c3dyn -o run --output-format csv -- python3 bench.py --config c3 --input dynamic --steps 5 --warmup 1 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04k_prof_c3dyn.log 2>&1
