#!/bin/bash
# Same-box A/B: one verify stream over 1M tuples against K concurrent streams sharing the same
# 1M (rehearsal path: K slots x n/K tuples) and K x 1M; plus the plugin tests after the
# incremental commit-collection change.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/round.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/$name.log" | tail -4 | cut -c1-400 | tee -a gpurun_out/round.log
    echo "rc=$rc" | tee -a gpurun_out/round.log
    return $rc
}
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
step plugin 300 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
for rep in 1 2; do
step b1_$rep 300 python bench.py $Q || exit $?
step s2half_$rep 300 python bench.py $Q --logical-slots 2 --n 500000 || exit $?
step s4q_$rep 300 python bench.py $Q --logical-slots 4 --n 250000 || exit $?
step s2full_$rep 300 python bench.py $Q --logical-slots 2 || exit $?
done
echo "== done"
