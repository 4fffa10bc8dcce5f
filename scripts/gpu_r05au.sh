# round 5 end: the N = 2 bench path rehearsed on one GPU (gloo, both ranks on device 0), C3 and C4
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cfg in c3 c4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config $cfg --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05au_${cfg}_n2.log 2>&1 || exit 1
done
