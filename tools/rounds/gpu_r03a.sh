#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/round.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/$name.log" | tail -8 | tee -a gpurun_out/round.log
    echo "rc=$rc" | tee -a gpurun_out/round.log
    return $rc
}
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step rehearsal 400 python bench.py --gpus 1 --logical-slots 8 --steps 5 --warmup 2 || exit $?
echo "== done"
