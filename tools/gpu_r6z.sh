#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_mx.py tests/test_gpu_lbwd.py -v -s -m gpu --timeout 600 --timeout-method thread -rf > gpurun_out/r6z.log 2>&1
rc=$?; grep -aE "FAILED|^E  |passed|failed|rel|band|ratio" gpurun_out/r6z.log | cut -c1-220 | tail -25; exit $rc
