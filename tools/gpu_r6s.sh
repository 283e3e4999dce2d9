#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv1_routes.py tests/test_gpu_c1r3_codes.py tests/test_gpu_c1_gram.py tests/test_gpu_cl.py tests/test_gpu_step.py -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/r6s.log 2>&1
rc=$?; grep -aE "FAILED|^E  |passed|failed" gpurun_out/r6s.log | cut -c1-200 | tail -12; [ $rc = 0 ] || exit $rc
bash tools/gpu_r6o.sh s1 3 default rcp0
