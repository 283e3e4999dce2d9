#!/bin/bash
# conv1 apply pass in registers: exactness tests, kernel timings, same-box step A/B
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cl.py tests/test_gpu_benchsize.py -k "recompute or moments" > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -aE "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/c1mbench.py | tee gpurun_out/c1m_$TAG.txt || exit 1
AVDINO_C1_APPLY_REG=1 timeout -k 10 120 python tools/c1mbench.py | tee -a gpurun_out/c1m_$TAG.txt || exit 1
bash tools/gpu_ab3.sh $TAG -
