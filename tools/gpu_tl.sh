#!/bin/bash
# bench line + one-step per-stream timeline and kernel stats of the default config-2 step.
#   usage: bash tools/gpu_tl.sh TAG [env assignments...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cut -c1-200 gpurun_out/bench_$TAG.json
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1 || exit $?
python tools/timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/tl_$TAG.txt
python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_$TAG.txt
head -4 gpurun_out/tl_$TAG.txt
