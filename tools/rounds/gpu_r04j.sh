#!/bin/bash
# Software-pipelined safegcd (SBFT_INV_PIPE=1, the build) against the previous form (pipe0):
# the GPU suite on the build, then interleaved A/B of config 3 (generic and registered-client
# VerifyProposal, both in-process through SBFT_GV_LIB), config 4's one-batch call (the keyed
# wavefront kernel, through the harness with the library swapped in LD_LIBRARY_PATH) and the
# throughput kernel.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04j_tests.log; [ $rc -ne 0 ] && exit $rc
mkdir -p /tmp/pipe0lib && ln -sf $V/lib_pipe0.so /tmp/pipe0lib/libsbft_gpuverify.so
Q="--no-sha --no-host-path --no-cpu-baseline --no-pipelined --steps 10 --warmup 3"
out=gpurun_out/r04j_ab.txt
: > $out
for rep in 1 2; do
  for v in cur pipe0; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; LP=; else export SBFT_GV_LIB=$V/lib_pipe0.so; LP=/tmp/pipe0lib; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/r04j_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r04j_${v}_$rep.log; exit 1; }
    python - gpurun_out/r04j_${v}_$rep.log $v $rep >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
L = d["latency"]
print(sys.argv[2], "rep", sys.argv[3], "value", round(d["value"] / 1e6, 2), "M/s kernel_ms", d["roofline"]["avg_kernel_ms"],
      "| vp10k p50/p99", L["verify_proposal_10k"]["p50_ms"], L["verify_proposal_10k"]["p99_ms"],
      "| registered p50/p99", L["verify_proposal_10k_registered_clients"]["p50_ms"], L["verify_proposal_10k_registered_clients"]["p99_ms"])
PY
    echo "$v rep $rep harness quorum-batch: $(LD_LIBRARY_PATH=$LP timeout -k 10 60 tools/latency_harness quorum-batch 67 400)" >> $out || exit 1
  done
done
unset SBFT_GV_LIB
cat $out
