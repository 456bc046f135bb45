#!/bin/bash
# Round 5: a larger differential parity sweep on the final tree: 6M seeded tuples (seed 2606) through
# the selected, throughput, pair and half kernels, 400k through the exact kernel, 20,000 registered
# keys (10 GB of comb tables) through the keyed wave (67 / 500) and four-lane paths, and 200k GPU-hashed
# messages + 50k VerifyProposal-layout requests, against the oracle and hashlib.
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/parity_sweep.py --n 6000000 --seed 2606 --keyed 20000 --exact 400000 --hash 200000 --framed 50000 > gpurun_out/r05as_parity.log 2>&1 || { tail -15 gpurun_out/r05as_parity.log; exit 1; }
tail -16 gpurun_out/r05as_parity.log
