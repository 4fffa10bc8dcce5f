# round 4: the whole GPU suite + smoke on the final tree, and the N > 1 rehearsal on one GPU
# (gloo: C3 at 4 ranks, C4 at 2, C3 loudnorm dynamic mode at 2 -- the sharded filter)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04y_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y_smoke.log 2>&1 || exit 1
bash scripts/gpu_rehearse.sh > gpurun_out/r04y_rehearse.txt 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --config c3 --input dynamic --gpus 2 --dist-backend gloo --one-device --steps 5 --warmup 1 --soak 0 > gpurun_out/r04y_rehearse_c3_dynamic_n2.log 2>&1
