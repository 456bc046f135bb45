#!/bin/bash
# SBFT_HELPER_NEAR=1 (the payload-copy helper on a CPU sharing the caller's L3) against the default,
# interleaved, config-3 latency and the VerifyProposal host phases (SBFT_VP_TRACE).
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r04w_ab.txt
: > $out
for rep in 1 2 3; do
  for v in near default; do
    if [ $v = near ]; then export SBFT_HELPER_NEAR=1; else unset SBFT_HELPER_NEAR; fi
    SBFT_VP_TRACE=1 timeout -k 10 180 python tools/latency_probe.py --calls 200 > gpurun_out/r04w_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r04w_${v}_$rep.log; exit 1; }
    python - gpurun_out/r04w_${v}_$rep.log $v $rep >> $out <<'PY'
import json, re, statistics, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in lines if l.startswith("{")][-1])
L = d["verify_proposal_10k"]
vp = [l for l in lines if l.startswith("vp ")][:200]  # the generic calls come first
def med(key):
    return statistics.median(float(re.search(key + r"=([\d.]+)", l).group(1)) for l in vp[5:])
print(sys.argv[2], "rep", sys.argv[3], "vp10k p50/p99", L["p50_ms"], L["p99_ms"],
      "| parse %.1f copy_wait %.1f rest %.1f us" % (med("parse"), med("copy_wait_sync"), med("rest")))
PY
  done
done
cat $out
