#!/bin/bash
# A/B of two builds of the keyed kernels (tools/build_variants.sh a:... b:...): kernel durations
# from rocprofv3 over tools/keyed_probe.py. Result r02g: the four-lane kernel with every mixed
# addition product in f29_mul_ilp form took 112.8 us per 4096 signatures against 110.9 us for the
# interleaved form; kept the interleaved form.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "$@"; do
  SBFT_GV_LIB=$PWD/tools/variants/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run --output-format csv -- python3 tools/keyed_probe.py > gpurun_out/kp_$v.log 2>&1 || exit $?
done
for v in "$@"; do echo "== $v"; grep -h "keyed" gpurun_out/prof_$v/run_kernel_stats.csv | cut -c1-60,200-; done
