#!/bin/bash
# Why config 3 reads ~40 us slower inside bench.py than in tools/latency_probe.py: probe on a
# fresh process, then right after a heavy bench run (configs 2/5, adversarial), then after a
# 20 s pause, then the bench's own latency section alone (--latency-only style: all heavy parts off).
mkdir -p gpurun_out
export TMPDIR=/tmp
probe() {
  timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_$1.log 2>&1 || { tail -5 gpurun_out/lat_$1.log; exit 1; }
  python - $1 gpurun_out/lat_$1.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
}
probe fresh1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_full.log 2>&1 || { tail -3 gpurun_out/bench_full.log; exit 1; }
python - gpurun_out/bench_full.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
l = [x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1]
d = json.loads(l)["latency"]
print("in_bench", *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
probe after_bench
sleep 20
probe after_pause
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sha --no-host-path --no-pipelined --steps 1 --warmup 1 > gpurun_out/bench_light.log 2>&1 || { tail -3 gpurun_out/bench_light.log; exit 1; }
python - gpurun_out/bench_light.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
l = [x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1]
d = json.loads(l)["latency"]
print("in_light_bench", *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
echo done
