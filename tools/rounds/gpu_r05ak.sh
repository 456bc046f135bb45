#!/bin/bash
# Round 5: the registered-client keyed kernel's comb additions in the pipelined ILP product form
# (SBFT_KEYED_LANES_ILP=1, p29_add_aff_lean_ilp) against the chain form: phase probes of both
# (lib_kprobe / lib_kprobe0), interleaved on one box; then the GPU tests of the keyed and config
# paths on the new default build and the registered-client config-3 latency.
mkdir -p gpurun_out
out=gpurun_out/r05ak_ab.txt; : > $out
for rep in 1 2; do
  for v in kprobe kprobe0; do
    SBFT_GV_LIB=$PWD/tools/variants/lib_$v.so timeout -k 10 300 python tools/keyed_lanes_probe.py > gpurun_out/r05ak_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05ak_${v}_$rep.log; exit 1; }
    echo "== $v rep $rep" >> $out; grep keyed-probe gpurun_out/r05ak_${v}_$rep.log | tail -5 >> $out
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_configs.py tests/test_gpu_plugin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ak_tests.log 2>&1 || { tail -15 gpurun_out/r05ak_tests.log; exit 1; }
tail -1 gpurun_out/r05ak_tests.log >> $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ak_lat -o st --output-format csv -- python3 tools/latency_probe.py --calls 100 > gpurun_out/r05ak_lat.log 2>&1 || { tail -5 gpurun_out/r05ak_lat.log; exit 1; }
python3 - gpurun_out/r05ak_lat/st_kernel_stats.csv gpurun_out/r05ak_lat.log >> $out <<'PY'
import csv, json, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "keyed" in r["Name"] or "half_kernel<true>" in r["Name"]:
        print(r["Name"].split("(")[0], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1), "min_us", round(float(r["MinNs"]) / 1e3, 1))
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("registered p50/p99", d["verify_proposal_10k_registered_clients"]["p50_ms"], d["verify_proposal_10k_registered_clients"]["p99_ms"],
      "| generic", d["verify_proposal_10k"]["p50_ms"], "| batch67", d["commit_quorum_n100"]["c_harness"]["p50_ms"])
PY
cat $out
