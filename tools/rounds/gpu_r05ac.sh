#!/bin/bash
# Round 5: the parity sweep's hash + verify sections (tools/parity_sweep.py --hash/--framed): 300k
# messages of 0-4096 B hashed on the GPU (config 5's HBM and streamed paths) and 50k signed
# requests in the VerifyProposal layout (fused half kernel at 10k per call, and one 50k call),
# with corrupted bodies, signatures and keys, against hashlib + the oracle; plus a 500k tuple pass.
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/parity_sweep.py --n 500000 --seed 2607 --exact 50000 --hash 300000 --framed 50000 --threads 16 > gpurun_out/r05ac_sweep.log 2>&1
rc=$?
grep -v "^W2026\|^E2026\|amdgpu.ids" gpurun_out/r05ac_sweep.log | tail -16
exit $rc
