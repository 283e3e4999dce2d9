#!/bin/bash
# GPU test pass: the named test files first (verbose), then the whole -m gpu suite.
# usage: bash tools/gpu_tests.sh TAG [test files...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -v -m gpu --timeout 300 --timeout-method thread -rf \
      > gpurun_out/tfirst_$TAG.log 2>&1
  rc=$?; echo "first rc=$rc"; grep -E "PASSED|FAILED|ERROR|^E  |passed|failed" gpurun_out/tfirst_$TAG.log | cut -c1-250 | tail -60
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf \
    > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "all rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | tail -30
exit $rc
