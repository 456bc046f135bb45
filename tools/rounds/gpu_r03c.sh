#!/bin/bash
# Same-box A/B of the step's launch shape: 1M tuples as one launch, as S sub-batches on one
# stream, and as S sub-batches over SS concurrent streams (forked and joined every step).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/$name.log | head -1)" | tee -a gpurun_out/ab.log
    return $rc
}
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
step b1_$rep 300 python bench.py $Q || exit $?
step s4x1_$rep 300 python bench.py $Q --split 4 || exit $?
step s4x4_$rep 300 python bench.py $Q --split 4 --split-streams 4 || exit $?
step s4x2_$rep 300 python bench.py $Q --split 4 --split-streams 2 || exit $?
step s8x4_$rep 300 python bench.py $Q --split 8 --split-streams 4 || exit $?
step s2x2_$rep 300 python bench.py $Q --split 2 --split-streams 2 || exit $?
step r4q_$rep 300 python bench.py $Q --logical-slots 4 --n 250000 || exit $?
done
