#!/bin/bash
# N > 1 rehearsal on one GPU (gloo, every rank on cuda:0): the bench's distributed path
# for C3 at N = 4 and C4 at N = 2 -- what the driver's RCCL scaling run executes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 4 --dist-backend gloo --one-device --steps 10 --warmup 2 --soak 0 > gpurun_out/rehearse_c3_n4.log 2>&1 || { echo "c3 n4 rc=$?"; exit 1; }
echo "c3 n4 ok"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --config c4 --gpus 2 --dist-backend gloo --one-device --steps 5 --warmup 1 --soak 0 > gpurun_out/rehearse_c4_n2.log 2>&1 || { echo "c4 n2 rc=$?"; exit 1; }
echo "c4 n2 ok"
