#!/bin/bash
# Config 4 (SimCLR) step: same-box alternating A/B of library variants (bench.py --workload
# simclr, no CPU baseline).  usage: bash tools/gpu_c4ab.sh TAG lib1.so|default lib2.so ...
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/$lib; fi
  line=$(timeout -k 10 300 python bench.py --workload simclr --no-cpu-baseline --steps 30 2> gpurun_out/c4ab_$TAG.err) || { tail -5 gpurun_out/c4ab_$TAG.err; exit 1; }
  echo "$line" >> gpurun_out/c4ab_${TAG}_lines.jsonl
  echo "$lib $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/c4ab_$TAG.txt
done
