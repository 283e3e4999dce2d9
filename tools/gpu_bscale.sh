#!/bin/bash
# config-2 step time vs batch (graph replay): the intercept is the per-step fixed cost
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 128 256 512 1024; do
  timeout -k 10 300 python bench.py --batch $b --no-cpu-baseline --steps 30 > gpurun_out/bscale_$b.json 2> gpurun_out/bscale_$b.err || exit $?
  echo "B=$b $(grep -o '"ms_per_step[^,]*' gpurun_out/bscale_$b.json)"
done
