#!/bin/bash
# Same-box A/B of bench.py flag sets on the whole step (no CPU baseline), interleaved.
#   usage: bash tools/gpu_abflag.sh TAG "flags a" "flags b" ...   ("-" = no extra flags)
TAG=$1; shift
mkdir -p gpurun_out
for e in "$@"; do
  if [ "$e" = - ]; then fl=(); else fl=($e); fi
  v=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 "${fl[@]}" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$e $v" | tee -a gpurun_out/abf_$TAG.txt
done
