#!/bin/bash
# Round-2 evidence in one call: default bench line, graph-replay kernel trace (stats + one-step
# timeline), PMC traffic of the roofline kernels (dominant and largest HBM-bound launch),
# whole-step PMC (traffic + MFMA counters) and one line per BASELINE config.  usage: TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-250 gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bprof_$TAG.json 2> gpurun_out/bprof_$TAG.err || exit $?
python tools/timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/tl_$TAG.txt
python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_$TAG.txt
head -3 gpurun_out/ks_$TAG.txt | cut -c1-150
for which in roofline roofline_hbm; do
  DOM=$(python -c "import json; print(json.loads(open('gpurun_out/bench_$TAG.json').readline())['$which']['kernel'])")
  DOM="$DOM" bash tools/gpu_pmc.sh ${TAG}_$which || exit 1
done
bash tools/gpu_pmc_step.sh $TAG || exit 1
bash tools/gpu_workloads.sh $TAG || exit 1
timeout -k 10 300 python bench.py --workload dino --mode semi_supervised --dtype fp8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_fp8_$TAG.json 2>&1; echo "fp8 rc=$?"; cut -c1-200 gpurun_out/bench_fp8_$TAG.json
