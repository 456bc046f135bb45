#!/bin/bash
# A/B of the generic comb's window width (tools/build_variants.sh wNN:-DSBFT_GCOMB_W=NN): per
# variant the first-use table build, golden-vector parity on the pair kernel, a 10k-tuple call,
# then the config-2 bench (verify only; full-size parity is checked inside bench.py).
mkdir -p gpurun_out
out=gpurun_out/gcomb_ab.txt
: > $out
for v in "$@"; do
  lib=$PWD/tools/variants/lib_$v.so
  SBFT_GV_LIB=$lib timeout -k 10 120 python tools/gcomb_probe.py >> $out 2>&1 || { echo "probe $v failed" >> $out; exit 1; }
  SBFT_GV_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency --no-sha --no-host-path > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed" >> $out; exit 1; }
  python - "$v" gpurun_out/bench_$v.log >> $out <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps({"variant": sys.argv[1], "value": d["value"], "kernel_ms": d["roofline"]["avg_kernel_ms"],
                  "step_ms": d["ms_per_step"], "frac": d["roofline"]["frac"], "parity": d["parity"]}))
PY
done
cat $out
