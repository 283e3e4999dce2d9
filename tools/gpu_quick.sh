#!/bin/bash
# quick loop: channels-last parity tests + op replay timings.  usage: bash tools/gpu_quick.sh TAG [filter]
TAG=$1; FILT=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_cl.py -q -m gpu -x > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/opbench.py --filter "$FILT" > gpurun_out/opbench_$TAG.txt 2>&1
echo "opbench rc=$?"; head -45 gpurun_out/opbench_$TAG.txt
