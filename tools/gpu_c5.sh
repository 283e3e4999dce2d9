#!/bin/bash
# Config 5 (semi-supervised, B = 4096) bf16 and fp8 bench lines, alternating, N rounds.
#   usage: bash tools/gpu_c5.sh TAG ROUNDS
TAG=$1; ROUNDS=${2:-1}
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 "$ROUNDS"); do
  for dt in bf16 fp8; do
    timeout -k 10 300 python bench.py --mode semi_supervised --dtype $dt --no-cpu-baseline > gpurun_out/c5_${dt}_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
    echo "$dt $(python -c "import json; d=json.load(open('gpurun_out/c5_${dt}_$TAG.json')); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/c5_$TAG.txt
  done
done
