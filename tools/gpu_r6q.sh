#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lbwd.py tests/test_gpu_benchsize.py -v -s -m gpu --timeout 300 --timeout-method thread -rf -k "lbwd or layer_bwd or fused or bf16_step_vs_fp32_step_config2" > gpurun_out/r6q.log 2>&1
rc=$?; grep -aE "FAILED|^E  |passed|failed|dX vs" gpurun_out/r6q.log | cut -c1-200 | tail -12; [ $rc = 0 ] || exit $rc
bash tools/gpu_lbpmc.sh r6p2
