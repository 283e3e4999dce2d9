#!/bin/bash
# Config 5 step (C5_DTYPE, default fp8) under environment variants, interleaved.
#   usage: bash tools/gpu_c5env.sh TAG ROUNDS "-" "VAR=value ..." ...
TAG=$1; ROUNDS=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --mode semi_supervised --dtype ${C5_DTYPE:-fp8} --no-cpu-baseline > gpurun_out/c5env_$TAG.json 2> gpurun_out/c5env_$TAG.err || { tail -5 gpurun_out/c5env_$TAG.err; exit 1; }
    echo "[$v] $(python -c "import json; d=json.load(open('gpurun_out/c5env_$TAG.json')); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/c5env_$TAG.txt
  done
done
