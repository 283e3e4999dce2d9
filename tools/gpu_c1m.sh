#!/bin/bash
# conv1 kernel timings per library variant.  usage: bash tools/gpu_c1m.sh TAG v0 v1 ...
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$v.so timeout -k 10 120 python tools/c1mbench.py 2>&1 | tail -1 | tee -a gpurun_out/c1m_$TAG.txt || exit 1
done
