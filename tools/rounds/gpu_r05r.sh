#!/bin/bash
# Round 5: the LLVM AMDGPU max-ILP scheduler (-mllvm -amdgpu-sched-strategy=max-ilp, variant
# tools/variants/lib_ilp.so) against the default build, interleaved on one box: half-kernel
# stats (10k VerifyProposal), throughput bench (1M), config-3 p50.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
B="--no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined --steps 10 --warmup 3"
out=gpurun_out/r05r_ab.txt; : > $out
for rep in 1 2; do
  for v in cur ilp; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -k 10 300 python bench.py $B > gpurun_out/r05r_bench_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05r_bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/r05r_bench_${v}_$rep.log') if l.startswith('{')][-1])
print('$v rep $rep bench', d['value'], 'kernel_ms', d['roofline']['avg_kernel_ms'])" >> $out
    timeout -k 10 180 python tools/latency_probe.py --calls 200 > gpurun_out/r05r_lat_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05r_lat_${v}_$rep.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05r_lat_${v}_$rep.log') if l.startswith('{')][-1])
L=d['verify_proposal_10k']; print('$v rep $rep vp10k p50/p99', L['p50_ms'], L['p99_ms'])" >> $out
  done
done
unset SBFT_GV_LIB
for v in cur ilp; do
  case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05r_stats_$v -o st --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05r_stats_$v.log 2>&1 || { tail -5 gpurun_out/r05r_stats_$v.log; exit 1; }
done
unset SBFT_GV_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_verify.py tests/test_gpu_fixup.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r05r_tests_cur.log 2>&1; echo "cur tests rc=$?" >> $out
cat $out
