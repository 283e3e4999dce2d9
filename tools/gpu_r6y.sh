#!/bin/bash
# config 5 fp8: the 56^2 layer backward through the fused bf16 launch vs the MX kernels
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for spec in "-" "ConvBranch.FP8_FUSED_BWD=True"; do
    if [ "$spec" = "-" ]; then args=(); else args=($spec); fi
    v=$(timeout -k 10 300 python tools/ab_attr.py "${args[@]}" -- --no-cpu-baseline --steps 20 --mode semi_supervised --dtype fp8 2>gpurun_out/aby.err | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'][:44], d['roofline']['avg_launch_us'], d['roofline']['frac'])") || { tail -5 gpurun_out/aby.err; exit 1; }
    echo "[$spec] $v" | tee -a gpurun_out/aby.txt
  done
done
