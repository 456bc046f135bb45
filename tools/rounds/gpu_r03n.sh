#!/bin/bash
# Lane-local pair ladder (p29_dbl_pl / p29_add_aff_pl) and alpha = 3a' by one carry pass
# (f29_triple): full GPU suite, then same-box A/B of config 2 and config 3/4 latency against
# nopl (-DSBFT_PAIR_LANE_LOCAL=0: the both-lanes pair forms) and notc (-DSBFT_TRIPLE_CARRY=0),
# and a kernel trace of the latency probe (the pair kernel's own time).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V=$PWD/tools/variants
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur nopl notc; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
    timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_${v}_$rep.log; exit 1; }
    python - $v gpurun_out/lat_${v}_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
unset SBFT_GV_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lat_prof -o run --output-format csv -- python3 tools/latency_probe.py --calls 50 > gpurun_out/lat_prof.log 2>&1 || { tail -3 gpurun_out/lat_prof.log; exit 1; }
echo done
