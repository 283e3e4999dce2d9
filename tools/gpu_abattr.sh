#!/bin/bash
# Same-box interleaved A/B of engine route attributes on the whole step (tools/ab_attr.py).
#   usage: bash tools/gpu_abattr.sh TAG ROUNDS "spec A" "spec B" ...   ("-" = defaults)
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq $R); do
  for spec in "$@"; do
    if [ "$spec" = "-" ]; then args=(); else args=($spec); fi
    v=$(timeout -k 10 300 python tools/ab_attr.py "${args[@]}" -- --no-cpu-baseline --steps 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['avg_launch_us'], d['roofline']['frac'])") || exit 1
    echo "[$spec] $v" | tee -a gpurun_out/abattr_$TAG.txt
  done
done
