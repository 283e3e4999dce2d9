#!/bin/bash
# 5x5 conv1 moments pass: its tests, the bf16 step tests, same-box A/B vs the stored-y path.
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cl.py -k "recompute" > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests1 rc=$rc"; grep -E "^E  |passed|failed|FAILED|pass-4" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    -s tests/test_gpu_benchsize.py -k "moments or bf16_step or conv1" tests/test_gpu_step.py tests/test_gpu_graph.py > gpurun_out/t2_$TAG.log 2>&1
rc=$?; echo "tests2 rc=$rc"; grep -aE "^E  |passed|failed|FAILED|moments rel|per-channel|^d4|group" gpurun_out/t2_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab3.sh $TAG AVDINO_L1_MOMENTS5=0 AVDINO_L1_MOMENTS5=1
