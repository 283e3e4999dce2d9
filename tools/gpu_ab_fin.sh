#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 2048 0 100000 2048 0; do
  AVDINO_FIN1_ROWS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/abf_$v.json 2> gpurun_out/abf_$v.err || { tail -5 gpurun_out/abf_$v.err; exit 1; }
  echo "FIN1_ROWS=$v $(grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/abf_$v.json | tr '\n' ' ')"
done
