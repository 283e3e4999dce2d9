#!/bin/bash
# The whole -m gpu suite in one pytest process, then the default bench line.  usage: bash tools/gpu_suite5.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/suite_$TAG.log 2>&1
rc=$?; grep -aE "^E  |passed|failed|FAILED|Error" gpurun_out/suite_$TAG.log | cut -c1-300 | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-330 gpurun_out/bench_$TAG.json
