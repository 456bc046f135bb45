#!/bin/bash
# A/B the SHA-256 kernel variants under tools/variants/ on the config-5 hashing stage
# (tools/sha_probe.py), after the GPU SHA tests on the default build.
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -k "sha or proposal" > gpurun_out/sha_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sha_tests.log; [ $rc -gt 1 ] && exit $rc
for lib in tools/variants/*.so; do
  [ -e "$lib" ] || continue
  echo "== $lib"
  SBFT_GV_LIB=$PWD/$lib timeout -k 10 300 python tools/sha_probe.py > gpurun_out/shavar_$(basename $lib).log 2>&1 || { echo "fail $?"; tail -5 gpurun_out/shavar_$(basename $lib).log; exit 1; }
  tail -1 gpurun_out/shavar_$(basename $lib).log | cut -c1-160
done
