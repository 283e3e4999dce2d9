#!/bin/bash
# Same-box A/B of environment switches on the default bench line: each argument is one
# variant, a space-separated list of VAR=value ("-" = no change); runs A B A B ...
#   usage: bash tools/gpu_ab_env.sh TAG ROUNDS "-" "AVDINO_NO_PIVOT=1"
TAG=$1; ROUNDS=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
    line=$(env $envs timeout -k 10 240 python bench.py --no-cpu-baseline --steps 60 2> gpurun_out/ab_$TAG.err) || { tail -5 gpurun_out/ab_$TAG.err; exit 1; }
    val=$(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])")
    echo "[$v] $val" | tee -a gpurun_out/ab_$TAG.txt
  done
done
