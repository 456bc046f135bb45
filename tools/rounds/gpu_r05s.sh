#!/bin/bash
# Round 5: where a config-3 VerifyProposal's host time goes (SBFT_VP_TRACE splits per call).
mkdir -p gpurun_out
SBFT_VP_TRACE=1 timeout -k 10 180 python tools/latency_probe.py --calls 100 > gpurun_out/r05s_lat.log 2> gpurun_out/r05s_trace.log || { tail -5 gpurun_out/r05s_trace.log; exit 1; }
python3 - <<'PY'
import re, statistics as st
rows=[l for l in open("gpurun_out/r05s_trace.log") if l.startswith("vp ") and "launch=0.0 " not in l]
keys=["submit","parse","copy_wait_sync","stage","launch","rest"]
vals={k:[] for k in keys}
for l in rows:
    for k in keys:
        m=re.search(k+r"=([0-9.]+)", l)
        if m: vals[k].append(float(m.group(1)))
print(len(rows), "calls;", {k:(round(st.median(v),1) if v else None) for k,v in vals.items()})
PY
