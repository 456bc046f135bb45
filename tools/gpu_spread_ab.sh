#!/bin/bash
# Throughput-launch grid A/B (SBFT_VERIFY_SPREAD=0/1, interleaved) on the config-2 bench, after
# the grid-shape parity test.
mkdir -p gpurun_out
out=gpurun_out/r02i_spread_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -m gpu -x -q -k "grid_shapes or bench_workload" --timeout 200 --timeout-method thread > gpurun_out/spread_tests.log 2>&1 || { tail -5 gpurun_out/spread_tests.log; exit 1; }
tail -1 gpurun_out/spread_tests.log >> $out
for rep in 1 2 3; do
  for sp in 0 1; do
    SBFT_VERIFY_SPREAD=$sp timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency --no-sha --no-host-path > gpurun_out/b_$sp.log 2>&1 || exit 1
    python - $sp gpurun_out/b_$sp.log >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(json.dumps({"spread": int(sys.argv[1]), "value": d["value"], "kernel_ms": d["roofline"]["avg_kernel_ms"],
                  "step_ms": d["ms_per_step"], "parity": d["parity"]["full_size_mismatches"]}))
PY
  done
done
cat $out
