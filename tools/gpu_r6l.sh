#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread -rf tests/test_gpu_lbwd.py tests/test_gpu_augment.py > gpurun_out/r6l.log 2>&1
rc=$?; grep -aE "FAILED|^E  |passed|failed" gpurun_out/r6l.log | cut -c1-200 | tail -20; [ $rc = 0 ] || exit $rc
bash tools/gpu_lbpmc.sh r6p1
