#!/bin/bash
# Quick GPU-box check: the GPU test suite (optionally filtered with PYTEST_K), then smoke and a
# short bench. Every GPU step has its own time limit; the script stops at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/round.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/$name.log" | tail -6 | tee -a gpurun_out/round.log
    echo "rc=$rc" | tee -a gpurun_out/round.log
    return $rc
}
if [ -n "$PYTEST_K" ]; then
  step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" || exit $?
else
  step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
fi
[ -n "$NO_BENCH" ] && exit 0
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py ${BENCH_ARGS} || exit $?
echo "== done" | tee -a gpurun_out/round.log
