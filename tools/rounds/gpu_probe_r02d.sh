#!/bin/bash
# all-exceptional batches (tests + timing), then full-size SHA-256 PMC passes
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "exceptional" > gpurun_out/exc_tests.log 2>&1 || { tail -30 gpurun_out/exc_tests.log; exit 1; }
tail -1 gpurun_out/exc_tests.log
timeout -k 10 300 python -c "
import json, torch, bench
from smartbft_amd import GpuVerifier
print(json.dumps(bench.adversarial(GpuVerifier(device_mask=1), torch.device('cuda:0'))))" > gpurun_out/adversarial.log 2>&1 || { cat gpurun_out/adversarial.log; exit 1; }
grep -v amdgpu.ids gpurun_out/adversarial.log
N=2097152
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/shaF_pmc1 -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/shaF_pmc1.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/shaF_pmc2 -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/shaF_pmc2.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS -d gpurun_out/shaF_pmc3 -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/shaF_pmc3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/shaF_stats -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/shaF_stats.log 2>&1 || exit $?
echo done
