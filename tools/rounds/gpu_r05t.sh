#!/bin/bash
# Round 5: VerifyProposal with the parsed offsets staged while the payload copy is still being
# staged by the helper: the proposal-path GPU tests, then the SBFT_VP_TRACE splits and p50.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_plugin.py tests/test_gpu_split.py tests/test_gpu_faults.py tests/test_gpu_keyed.py tests/test_gpu_runtime.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05t_tests.log 2>&1 || { tail -15 gpurun_out/r05t_tests.log; exit 1; }
tail -2 gpurun_out/r05t_tests.log
SBFT_VP_TRACE=1 timeout -k 10 180 python tools/latency_probe.py --calls 100 > gpurun_out/r05t_lat.log 2> gpurun_out/r05t_trace.log || { tail -5 gpurun_out/r05t_trace.log; exit 1; }
python3 - <<'PY'
import re, json, statistics as st
rows=[l for l in open("gpurun_out/r05t_trace.log") if l.startswith("vp ") and "launch=0.0 " not in l]
keys=["submit","parse","copy_wait_sync","stage","launch","rest"]
vals={k:[] for k in keys}
for l in rows:
    for k in keys:
        m=re.search(k+r"=([0-9.]+)", l)
        if m: vals[k].append(float(m.group(1)))
print(len(rows), "calls;", {k:(round(st.median(v),1) if v else None) for k,v in vals.items()})
d=json.loads([l for l in open("gpurun_out/r05t_lat.log") if l.startswith("{")][-1])
print("vp10k", d["verify_proposal_10k"]["p50_ms"], d["verify_proposal_10k"]["p99_ms"], "registered", d["verify_proposal_10k_registered_clients"]["p50_ms"])
PY
