#!/bin/bash
# selected test files, then the config-2 bench (no CPU baseline).  usage: TAG files...
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/tsel_$TAG.log 2>&1
rc=$?; grep -E "^E  |passed|failed|FAILED" gpurun_out/tsel_$TAG.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
grep -o '"value[^,]*\|"ms_per_step[^,]*\|"step_frac[^,]*' gpurun_out/bench_c2_$TAG.json
