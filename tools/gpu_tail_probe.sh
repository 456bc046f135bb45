#!/bin/bash
# verify-kernel wave-quantisation probe: device-resident rate at several launch sizes
# (1M = 3.81 rounds of 4,096 resident waves), then two ranks sharing the GPU (gloo)
mkdir -p gpurun_out
: > gpurun_out/tail.log
for n in 1000000 1048576 786432 2000000 1000000; do
  timeout -k 10 200 python bench.py --n $n --steps 10 --warmup 2 --no-cpu-baseline --no-latency --no-sha --no-host-path > gpurun_out/tail_$n.log 2>&1 || { tail -5 gpurun_out/tail_$n.log; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open('gpurun_out/tail_$n.log') if l.startswith('{')][-1]);print($n, d['value'], d['roofline']['avg_kernel_ms'], d['ms_per_step'])" >> gpurun_out/tail.log
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo > gpurun_out/dist2.log 2>&1 || { tail -30 gpurun_out/dist2.log; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/dist2.log') if l.startswith('{')][-1]);print('2rank', d['value'], d['roofline']['avg_kernel_ms'], d['ms_per_step'])" >> gpurun_out/tail.log
cat gpurun_out/tail.log
