#!/bin/bash
# rocprofv3 passes on the SHA-256 kernel (tools/sha_ab.py, 262,144 config-5 messages): stats,
# then one PMC pass per counter group (never combined with tracing domains)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=262144
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sha_stats -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/sha_stats.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/sha_pmc1 -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/sha_pmc1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/sha_pmc2 -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/sha_pmc2.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM -d gpurun_out/sha_pmc3 -o run --output-format csv -- python3 tools/sha_ab.py $N > gpurun_out/sha_pmc3.log 2>&1 || exit $?
ls gpurun_out/sha_pmc1 gpurun_out/sha_stats
