#!/bin/bash
# GPU-box cycle: parity tests, then a profiled 1-GPU bench.  usage: bash tools/gpu_check.sh TAG [bench args]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_step.py -q -m gpu -rf > gpurun_out/t_$TAG.log 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -30
if [ $rc -le 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/b_$TAG.log 2>&1
  echo "prof rc=$?"
  grep metric gpurun_out/b_$TAG.log | cut -c1-400
fi
