#!/bin/bash
# Baseline GPU check: parity tests -> smoke -> full bench (latency + sha + cpu baseline).
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
rm -f gpurun_out/round.log
step tests 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py ${BENCH_ARGS} || exit $?
echo "== done" | tee -a gpurun_out/round.log
