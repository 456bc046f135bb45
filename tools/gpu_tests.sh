#!/bin/bash
# Run the GPU test suite (optionally filtered: PYTEST_K="expr").
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=10 -k "$PYTEST_K" > gpurun_out/tests.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=10 > gpurun_out/tests.log 2>&1
fi
rc=$?; grep -v "^W2026\|^E2026" gpurun_out/tests.log | tail -40; exit $rc
