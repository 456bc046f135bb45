#!/bin/bash
# Round 5: byte_of's select chain kept in registers (SBFT_BYTE_OF_REGS, default 1) against the
# build where LLVM turns it into a 32-B stack array and an indexed scratch load (lib_bo0,
# -DSBFT_BYTE_OF_REGS=0): keyed / sign GPU tests on the new build, then the keyed wave kernel's
# rocprof average and config-4 latencies, interleaved on one box.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_plugin.py tests/test_gpu_split.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ag_tests.log 2>&1 || { tail -15 gpurun_out/r05ag_tests.log; exit 1; }
tail -1 gpurun_out/r05ag_tests.log
out=gpurun_out/r05ag_ab.txt; : > $out
for rep in 1 2 3; do
  for v in cur bo0; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -k 10 240 python tools/latency_probe.py --calls 200 > gpurun_out/r05ag_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05ag_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05ag_${v}_$rep.log $v $rep >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
q = d["commit_quorum_n100"]; h = d["commit_quorum_n100_hook"]; c = d["commit_quorum_n100_concurrent_singles"]["coalesced"]
pp = d["commit_quorum_n100_pipelined"]["gpu"]
print(sys.argv[2], "rep", sys.argv[3], "batch67 p50", q["c_harness"]["p50_ms"], "| hook p50/p99", h["p50_ms"], h["p99_ms"],
      "| singles coalesced p50/p99", c["p50_ms"], c["p99_ms"], "| pipelined", pp["decisions_per_s"])
PY
    timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ag_st_${v}_$rep -o st --output-format csv -- python3 tools/latency_probe.py --calls 50 > gpurun_out/r05ag_p_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05ag_p_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05ag_st_${v}_$rep/st_kernel_stats.csv $v $rep >> $out <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "keyed_wave" in r["Name"] or "sign_wave" in r["Name"]:
        print(sys.argv[2], "rep", sys.argv[3], r["Name"].split("(")[0], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2), "min_us", round(float(r["MinNs"]) / 1e3, 2))
PY
  done
done
unset SBFT_GV_LIB
cat $out
