#!/bin/bash
# The whole -m gpu suite in one pytest process (round 6).
#   usage: bash tools/gpu_suite6.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1120 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rf \
    > gpurun_out/suite_$TAG.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -aE "^E  |passed|failed|FAILED" gpurun_out/suite_$TAG.log | cut -c1-300 | tail -30
exit $rc
