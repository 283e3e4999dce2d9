#!/bin/bash
# config-2 bench A/B over env settings given as args ("VAR=a" "VAR=b" ...), each run twice
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/ab2.json 2> gpurun_out/ab2.err || { tail -5 gpurun_out/ab2.err; exit 1; }
    echo "$cfg $(grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/ab2.json | tr '\n' ' ')"
  done
done
