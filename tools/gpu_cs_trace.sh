mkdir -p gpurun_out
SBFT_CS_TRACE=1 SBFT_KEYED_TRACE=1 timeout -k 10 60 tools/latency_harness quorum-gpu 66 30 22 15 > gpurun_out/trace_22_15.txt 2>&1 || exit $?
SBFT_CS_TRACE=1 SBFT_KEYED_TRACE=1 timeout -k 10 60 tools/latency_harness quorum-gpu 66 30 66 50 > gpurun_out/trace_66_50.txt 2>&1 || exit $?
tail -40 gpurun_out/trace_22_15.txt
