#!/bin/bash
# bisect the host segfault seen when tests/test_gpu_step.py runs before tests/test_gpu_graph.py
#   usage: bash tools/gpu_r6seg.sh pytest-targets...
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "$@" -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/seg.log 2>&1
rc=$?; echo "rc=$rc :: $(grep -aE 'passed|failed|Fatal' gpurun_out/seg.log | tail -1)"; exit $rc
