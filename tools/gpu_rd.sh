#!/bin/bash
# dgrad + BN-backward reduce fusion: its kernel tests, the step tests, same-box A/B, kernel stats.
#   usage: bash tools/gpu_rd.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_benchsize.py tests/test_gpu_step.py > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_abenv.sh $TAG AVDINO_DGRAD_BNREDUCE=0 AVDINO_DGRAD_BNREDUCE=1 AVDINO_DGRAD_BNREDUCE=0 AVDINO_DGRAD_BNREDUCE=1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1
echo "prof rc=$?"; grep metric gpurun_out/b_$TAG.log | cut -c1-200
