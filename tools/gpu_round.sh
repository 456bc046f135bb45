#!/bin/bash
# Full GPU-box round: parity tests -> smoke -> bench -> variants -> rocprofv3 stats -> PMC passes.
# Every GPU step has its own time limit; the script stops at the first crash/timeout.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/round.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/$name.log" | tail -4 | tee -a gpurun_out/round.log
    echo "rc=$rc" | tee -a gpurun_out/round.log
    return $rc
}
step tests 900 python -m pytest tests -m gpu -q --maxfail=5; rc=$?
[ $rc -gt 1 ] && exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py || exit $?
for lib in tools/variants/*.so; do
  [ -e "$lib" ] || continue
  SBFT_GV_LIB=$PWD/$lib step var_$(basename $lib .so) 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined || exit $?
done
if [ -z "$SKIP_PROF" ]; then
step prof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined || exit $?
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined || exit $?
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined || exit $?
step pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_valu -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined || exit $?
step pmc_busy 600 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d gpurun_out/pmc_busy -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined || exit $?
fi
echo "== done" | tee -a gpurun_out/round.log
