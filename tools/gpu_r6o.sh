#!/bin/bash
# config 2 alternating library variants on one box, no tests (A/B timing only)
#   usage: bash tools/gpu_r6o.sh TAG ROUNDS v1 v2 ...
TAG=$1; R=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
VD=multimodal-ssl-avmnist_amd/avdino/variants
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=$VD/libavdino_$v.so; fi
    line=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 2>gpurun_out/abo_$TAG.err) || { tail -5 gpurun_out/abo_$TAG.err; exit 1; }
    echo "$v $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'][:44], r['avg_launch_us'], r.get('isolated_avg_launch_us'), r['frac'])")" | tee -a gpurun_out/abo_$TAG.txt
  done
done
