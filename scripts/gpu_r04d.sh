# round 4: the whole GPU suite, smoke, and the N > 1 rehearsal on one GPU (gloo)
set -o pipefail
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04d_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04d_smoke.log 2>&1 && \
bash scripts/gpu_rehearse.sh > gpurun_out/r04d_rehearse.txt 2>&1
