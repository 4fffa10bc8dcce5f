# round 4: loudnorm dynamic mode in the bench -- C3 (5 min 48 kHz) and C5 strong (one
# 60-min 96 kHz track) at N = 1, then C5 strong over 2 gloo ranks on one GPU (the
# segment-sharded filter, 192 kHz measurement and alimiter over the ranks)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --input dynamic --steps 10 --warmup 2 --soak 0.5 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04j_bench_c3_dynamic.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --config c5 --strong --input dynamic --steps 3 --warmup 1 --soak 0 --no-cpu-baseline > gpurun_out/r04j_bench_c5_strong_dynamic.log 2>&1 || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --config c5 --strong --input dynamic --gpus 2 --dist-backend gloo --one-device --steps 2 --warmup 1 --soak 0 > gpurun_out/r04j_rehearse_c5_strong_dynamic_n2.log 2>&1
[ $? -eq 0 ] && timeout -k 10 300 python bench.py --config c3 --force-exchange --steps 50 --warmup 3 --soak 1 --no-cpu-baseline --no-other-configs --no-pipeline > gpurun_out/r04j_bench_c3_force_exchange.log 2>&1
