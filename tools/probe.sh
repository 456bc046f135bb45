#!/bin/bash
# Probe of the GPU box: toolchains, host CPU, device. Output under gpurun_out/probe.txt.
mkdir -p gpurun_out
{
  echo "== go"; (go version || echo "go: absent") 2>&1
  echo "== nproc"; nproc
  echo "== cpu"; grep -m1 "model name" /proc/cpuinfo; grep -c ^processor /proc/cpuinfo
  echo "== taskset"; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
  echo "== openssl"; openssl version; ls /usr/lib/x86_64-linux-gnu/libcrypto.so* 2>&1
  echo "== rocm-smi"; timeout 30 rocm-smi --showproductname 2>&1 | head -20
  echo "== valu_peak"; timeout -k 10 120 ./tools/valu_peak
} > gpurun_out/probe.txt 2>&1
cat gpurun_out/probe.txt
