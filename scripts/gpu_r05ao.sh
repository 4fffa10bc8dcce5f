# round 5 end: the N > 1 step rehearsed at one rank with every collective over RCCL (C3, C2)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cfg in c3 c2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --config $cfg --force-exchange --steps 300 --warmup 20 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r05ao_${cfg}_fx.log 2>&1 || exit 1
done
