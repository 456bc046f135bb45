#!/bin/bash
# Round 5: differential parity sweep on the final build after the keyed lanes kernel's changes
# (ping-pong comb, Z^2/Z^3 beside X3/Y3): 1M seeded tuples (18 corruption kinds) through the
# selected, throughput, pair and half kernels, 50k through the exact kernel, and 6,000 registered
# keys through the keyed wave (67 / 500) and four-lane paths, against the oracle.
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/parity_sweep.py --n 1000000 --keyed 6000 --hash 0 --exact 50000 > gpurun_out/r05aq_parity.log 2>&1 || { tail -15 gpurun_out/r05aq_parity.log; exit 1; }
tail -12 gpurun_out/r05aq_parity.log
