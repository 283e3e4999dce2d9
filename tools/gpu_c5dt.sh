#!/bin/bash
# Config 5 (B = 4096, semi-supervised) bf16 vs fp8, same box, alternating, plus the probe line.
#   usage: bash tools/gpu_c5dt.sh TAG ROUNDS
TAG=$1; ROUNDS=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 "$ROUNDS"); do
  for dt in bf16 fp8; do
    timeout -k 10 300 python bench.py --mode semi_supervised --dtype $dt --no-cpu-baseline > gpurun_out/c5dt_$TAG.json 2> gpurun_out/c5dt_$TAG.err || { tail -5 gpurun_out/c5dt_$TAG.err; exit 1; }
    echo "$dt $(python -c "import json; d=json.loads(open('gpurun_out/c5dt_$TAG.json').readline()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/c5dt_$TAG.txt
  done
done
timeout -k 10 400 python bench.py --mode semi_supervised --probe --no-cpu-baseline > gpurun_out/c5probe_$TAG.json 2> gpurun_out/c5probe_$TAG.err || { tail -5 gpurun_out/c5probe_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/c5probe_$TAG.json
