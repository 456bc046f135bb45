#!/bin/bash
# Round-5 evidence on the final build (+ the registered-client keyed kernel's ping-pong comb, 48 per workgroup; the half kernel's entries read before the doublings): the whole GPU suite, smoke, the default bench line,
# rocprofv3 kernel-trace stats over 20 timed steps (tools/trace_summary.py compares the same
# dispatches with the bench's HIP events), the PMC passes (separate runs, counters within the
# per-block limits), and kernel stats of the latency path (configs 3/4).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/r05an.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/r05an_$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/r05an_$name.log" | tail -3 | tee -a gpurun_out/r05an.log
    echo "rc=$rc" | tee -a gpurun_out/r05an.log
    return $rc
}
B="--no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined"
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py || exit $?
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05an_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 $B || exit $?
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B || exit $?
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B || exit $?
step pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_valu -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B || exit $?
step pmc_busy 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d gpurun_out/pmc_busy -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B || exit $?
step prof_lat 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05an_proflat -o run --output-format csv -- python3 tools/latency_probe.py --calls 100 || exit $?
echo "== done" | tee -a gpurun_out/r05an.log
