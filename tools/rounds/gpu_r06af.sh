#!/bin/bash
# Round 6: differential parity sweep on the final kernels after the quad table build (seed 2608): every verify kernel incl.
# the wide half kernel (quad ladders, affine join), exact, keyed, GPU-hashed and VerifyProposal layouts.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06af
timeout -k 10 900 python -u tools/parity_sweep.py --n 2000000 --seed 2608 --threads 16 > gpurun_out/${T}_sweep.log 2>&1 || { tail -30 gpurun_out/${T}_sweep.log; exit 1; }
tail -c 4000 gpurun_out/${T}_sweep.log
