#!/bin/bash
# GEMM launch-plan A/B: opbench over the step's GEMMs per environment setting.
#   usage: bash tools/gpu_gemm_ab.sh TAG "VAR=a VAR2=b" "VAR=c" ...
TAG=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/gemm_ab_$TAG.txt
  env $cfg timeout -k 10 200 python tools/opbench.py --reps 20 --filter gemm >> gpurun_out/gemm_ab_$TAG.txt 2>&1 || exit $?
done
grep -E "^==|serial" gpurun_out/gemm_ab_$TAG.txt
