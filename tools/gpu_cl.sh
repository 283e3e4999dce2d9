#!/bin/bash
# channels-last path: kernel parity, step parity, then a profiled bench.  usage: bash tools/gpu_cl.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_cl.py tests/test_gpu_step.py -q -m gpu -rf -x > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED|Error" gpurun_out/t_$TAG.log | cut -c1-300 | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1
echo "prof rc=$?"; grep metric gpurun_out/b_$TAG.log | cut -c1-300
