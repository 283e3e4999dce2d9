#!/bin/bash
# conv kernel loop: conv parity tests, then op replay timings of the conv launches (new path,
# and the legacy kernels for comparison).  usage: bash tools/gpu_ws.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cl.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/opbench.py --filter cl_conv > gpurun_out/opbench_$TAG.txt 2>&1
echo "opbench rc=$?"; cat gpurun_out/opbench_$TAG.txt
AVDINO_CONV_LEGACY=1 timeout -k 10 300 python tools/opbench.py --filter cl_conv > gpurun_out/opbench_${TAG}_legacy.txt 2>&1
echo "legacy rc=$?"; head -30 gpurun_out/opbench_${TAG}_legacy.txt
