#!/bin/bash
# full -m gpu suite then the config-2 bench (no CPU baseline) and the config-4 bench
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh $TAG || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
grep -o '"value[^,]*\|"ms_per_step[^,]*\|"step_frac[^,]*' gpurun_out/bench_c2_$TAG.json
