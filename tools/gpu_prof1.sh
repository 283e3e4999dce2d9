#!/bin/bash
# one workload: bench line + rocprof kernel stats.  usage: bash tools/gpu_prof1.sh WORKLOAD TAG [bench args]
W=$1; TAG=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline "$@" > gpurun_out/bench_${W}_$TAG.json 2> gpurun_out/bench_${W}_$TAG.err || exit $?
grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/bench_${W}_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${W}_$TAG -o run -- \
    python bench.py --workload $W --no-cpu-baseline --no-graph --steps 10 --warmup 3 "$@" > /dev/null 2> gpurun_out/prof_${W}_$TAG.err || exit $?
python tools/prof_summary.py gpurun_out/prof_${W}_$TAG/run_kernel_stats.csv 13 30 | cut -c1-170
