#!/bin/bash
# multi-window BN-backward apply: exactness tests, step tests, same-box A/B
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_benchsize.py tests/test_gpu_cl.py tests/test_gpu_step.py > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -aE "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab3.sh $TAG - AVDINO_APPLY_WPT=1 AVDINO_APPLY_WPT=2
