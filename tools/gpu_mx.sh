#!/bin/bash
# MX (block-scaled fp8) conv kernels: tests, mismatch pattern, standalone timings vs bf16.
#   usage: bash tools/gpu_mx.sh TAG
TAG=${1:-x}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --tb=line --timeout 120 --timeout-method thread tests/test_gpu_mx.py > gpurun_out/mx_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/mx_$TAG.log | cut -c1-300
[ $rc -le 1 ] || exit $rc
timeout -k 10 90 python tools/mxdebug.py | cut -c1-200 || exit $?
timeout -k 10 120 python tools/mxbench.py && timeout -k 10 120 python tools/mxbench.py --n 28672
