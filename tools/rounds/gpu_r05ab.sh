#!/bin/bash
# Round 5: differential parity sweeps at scale (tools/parity_sweep.py): 2M (then 6M, seed 2606, 1M exact) seeded, GPU-signed tuples with
# 18 kinds of corruption / edge form through every verify kernel, 200k through the exact kernel and
# 3k registered keys through the three keyed paths, each against the oracle (16 threads).
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/parity_sweep.py --n 2000000 --threads 16 > gpurun_out/r05ab_sweep.log 2>&1 && timeout -k 10 900 python -u tools/parity_sweep.py --n 6000000 --seed 2606 --exact 1000000 --threads 16 > gpurun_out/r05ab_sweep2.log 2>&1
rc=$?
grep -v "^W2026\|^E2026" gpurun_out/r05ab_sweep.log gpurun_out/r05ab_sweep2.log | tail -24
exit $rc
