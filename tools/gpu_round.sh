#!/bin/bash
# Full GPU-box round: parity tests -> smoke -> bench -> rocprofv3 kernel stats -> PMC passes.
# Every GPU step has its own time limit; the script stops at the first crash/timeout.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/round.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/round.log
    echo "rc=$rc" | tee -a gpurun_out/round.log
    return $rc
}
step tests 900 python -m pytest tests -m gpu -q --maxfail=5; rc=$?
[ $rc -gt 1 ] && exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py || exit $?
step valu_peak 120 ./tools/valu_peak || exit $?
if [ -x tools/fmul_bench ]; then step fmul_bench 300 ./tools/fmul_bench || exit $?; fi
step prof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit $?
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_valu -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
echo "== done" | tee -a gpurun_out/round.log
