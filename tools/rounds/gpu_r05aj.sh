#!/bin/bash
# Round 5: the registered-client keyed kernel's comb phase with every tuple's u2 Q read from one
# key's table (lib_khot, -DSBFT_KEYED_HOT_TABLE, timing only) against the real per-key tables
# (lib_kprobe): is the comb bound by the table loads?
mkdir -p gpurun_out
for v in kprobe khot kprobe khot; do
  SBFT_GV_SELFTEST=0 KEYED_PROBE_NOCHECK=1 SBFT_GV_LIB=$PWD/tools/variants/lib_$v.so timeout -k 10 300 python tools/keyed_lanes_probe.py > gpurun_out/r05aj_$v.log 2>&1 || { tail -5 gpurun_out/r05aj_$v.log; exit 1; }
  echo "== $v"; grep keyed-probe gpurun_out/r05aj_$v.log | tail -5
done
