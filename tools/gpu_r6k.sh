#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread -rf tests/test_gpu_benchsize.py -k "bf16_step_vs_fp32_step_config2" tests/test_gpu_lbwd.py tests/test_gpu_augment.py > gpurun_out/r6k.log 2>&1
rc=$?; grep -aE "PASSED|FAILED|^E  |passed|failed" gpurun_out/r6k.log | cut -c1-200 | tail -20; [ $rc = 0 ] || exit $rc
bash tools/gpu_evid6.sh r6e1
