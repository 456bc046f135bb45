#!/bin/bash
# A/B of the host-buffer path of config 2: sub-batch pipelining of pageable inputs (staged into
# page-locked memory) on (1) / off (0); bench.py host_buffer_path.
mkdir -p gpurun_out
for v in 1 0 1; do
  SBFT_PIPE_PAGEABLE=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-sha > gpurun_out/hp_$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
t = open(f"gpurun_out/hp_{v}.log").read()
d = json.loads(t[t.index('{"metric"'):].split("\n")[0])
h = d["host_buffer_path"]
print("pipe_pageable", v, "pageable", h["value"], "mismatches", h["mismatches"], "pinned", h["pinned"]["value"])
PY
done
