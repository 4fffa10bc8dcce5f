cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03e_c3 -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --soak 0 --no-cpu-baseline --no-pipeline --no-other-configs \
    > gpurun_out/prof_r03e_c3.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo "prof done"
CFG=c3 bash scripts/gpu_traffic.sh || { echo "traffic rc=$?"; exit 1; }
echo "traffic done"
CFG=c3 bash scripts/gpu_flops.sh || { echo "flops rc=$?"; exit 1; }
echo "flops done"
