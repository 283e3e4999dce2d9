#!/bin/bash
# Round-6 GPU check: selected tests (one pytest process, verbose, per-test timeout), the RCCL
# world-1 test in its own process, then the default bench line.
#   usage: bash tools/gpu_r6.sh TAG "pytest targets" [rccl]
TAG=$1; TARGETS=$2; RCCL=$3
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest $TARGETS -v -s -m gpu --timeout 400 --timeout-method thread -rf \
    > gpurun_out/r6_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -aE "PASSED|FAILED|ERROR|^E  |passed|failed" gpurun_out/r6_$TAG.log | cut -c1-250 | tail -60
[ $rc -le 1 ] || exit $rc
if [ -n "$RCCL" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -v -s -m gpu --timeout 240 --timeout-method thread -rf \
      > gpurun_out/r6_${TAG}_rccl.log 2>&1
  rc=$?; echo "rccl rc=$rc"; grep -aE "PASSED|FAILED|ERROR|^E  |passed|failed" gpurun_out/r6_${TAG}_rccl.log | cut -c1-250 | tail -20
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench rc=$?"; cut -c1-400 gpurun_out/bench_$TAG.json
