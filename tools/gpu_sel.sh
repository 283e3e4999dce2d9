#!/bin/bash
# Selected GPU tests (verbose, one pytest process), then the default bench line.
#   usage: bash tools/gpu_sel.sh TAG [pytest args...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -v -s -m gpu --timeout 300 --timeout-method thread -rf \
    > gpurun_out/sel_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -aE "PASSED|FAILED|ERROR|^E  |passed|failed" gpurun_out/sel_$TAG.log | cut -c1-250 | tail -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench rc=$?"; cut -c1-400 gpurun_out/bench_$TAG.json
