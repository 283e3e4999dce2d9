#!/bin/bash
# config-2 bench A/B over an env switch.  usage: bash tools/gpu_ab_env.sh VAR
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0 1 0; do
  env $1=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  echo "$1=$v $(grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/ab_$v.json | tr '\n' ' ')"
done
