#!/bin/bash
# Round 5: the 3.7 MB payload copy from pageable memory, the runtime's pageable copy against our
# own staging (T pool threads, C-byte chunks into page-locked memory, each chunk's DMA queued as
# soon as it is staged), tools/h2d_pinned.
mkdir -p gpurun_out
timeout -k 10 300 ./tools/h2d_pinned > gpurun_out/r05u_h2d.txt 2>&1 || { tail -5 gpurun_out/r05u_h2d.txt; exit 1; }
cat gpurun_out/r05u_h2d.txt
