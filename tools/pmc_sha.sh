#!/bin/bash
# PMC passes over the SHA-256 probe (one counter group per pass).
mkdir -p gpurun_out/pmc_sha; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_sha/p$i -o run --output-format csv -- python3 tools/sha_probe.py --messages 131072 > gpurun_out/pmc_sha/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc_sha/p$i.log; exit 1; }
done
echo done
