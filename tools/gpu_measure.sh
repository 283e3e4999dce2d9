#!/bin/bash
# Measurement pass: counter list, default bench (with CPU baseline), rocprof kernel trace of a
# 30-step bench.  usage: bash tools/gpu_measure.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1; echo "list rc=$?"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bprof_$TAG.json 2> gpurun_out/bprof_$TAG.err
rc=$?; echo "prof rc=$rc"; cut -c1-400 gpurun_out/bprof_$TAG.json
python tools/prof_summary.py $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) 36 > gpurun_out/kstats_$TAG.txt 2>&1; head -30 gpurun_out/kstats_$TAG.txt | cut -c1-200
