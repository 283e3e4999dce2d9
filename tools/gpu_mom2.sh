#!/bin/bash
# moments-pass kernel: parity tests, conv1 kernel timings, same-box step A/B.
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cl.py -k "recompute" tests/test_gpu_benchsize.py -k "recompute or moments" > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -aE "^E  |passed|failed|FAILED|moments rel" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/c1mbench.py | tee gpurun_out/c1m_$TAG.txt || exit 1
bash tools/gpu_ab3.sh $TAG AVDINO_L1_MOMENTS5=0 AVDINO_L1_MOMENTS5=1
