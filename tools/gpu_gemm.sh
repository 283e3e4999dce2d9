#!/bin/bash
# GEMM loop: GEMM/Linear parity tests, then op replay timings of the step's GEMM launches
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -m gpu -x -k "gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/opbench.py --filter gemm > gpurun_out/opbench_$TAG.txt 2>&1
echo "opbench rc=$?"; cat gpurun_out/opbench_$TAG.txt | grep -v amdgpu.ids
