#!/bin/bash
# Round 5: the default bench line on the final tree (after the keyed lanes kernel's Z^2/Z^3 change).
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r05at_bench.log 2>&1 || { tail -5 gpurun_out/r05at_bench.log; exit 1; }
python3 - gpurun_out/r05at_bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
L = d["latency"]
print("value", d["value"], "frac", d["roofline"]["frac"], "| vp10k", L["verify_proposal_10k"]["p50_ms"], L["verify_proposal_10k"]["p99_ms"],
      "| registered", L["verify_proposal_10k_registered_clients"]["p50_ms"], L["verify_proposal_10k_registered_clients"]["p99_ms"],
      "| batch67", L["commit_quorum_n100"]["c_harness"]["p50_ms"], "| pipelined", L["commit_quorum_n100_pipelined"]["gpu"]["decisions_per_s"])
PY
