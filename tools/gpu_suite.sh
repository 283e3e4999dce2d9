#!/bin/bash
# The whole -m gpu suite in one pytest process, then the default bench line.
#   usage: bash tools/gpu_suite.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf -s \
    > gpurun_out/suite_$TAG.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -aE "^E  |passed|failed|FAILED" gpurun_out/suite_$TAG.log | cut -c1-300 | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench rc=$?"; cut -c1-300 gpurun_out/bench_$TAG.json
