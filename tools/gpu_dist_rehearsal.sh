#!/bin/bash
# torchrun path of bench.py with 2 ranks on a one-GPU box (gloo for the barrier / max-time
# reduction; both ranks share cuda:0), then the same with --gpus 1 for comparison
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > gpurun_out/dist2.log 2>&1 || { tail -30 gpurun_out/dist2.log; exit 1; }
grep '^{' gpurun_out/dist2.log | cut -c1-600
