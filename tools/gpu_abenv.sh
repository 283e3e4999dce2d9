#!/bin/bash
# Same-box A/B of environment switches on the whole step (bench.py, no CPU baseline), interleaved.
#   usage: bash tools/gpu_abenv.sh TAG "VAR=a" "VAR=b" ...   ("-" = no extra variable)
TAG=$1; shift
mkdir -p gpurun_out
for e in "$@"; do
  if [ "$e" = - ]; then envs=(); else envs=($e); fi
  v=$(env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$e $v" | tee -a gpurun_out/abe_$TAG.txt
done
