#!/bin/bash
# tools/c1s3bench.py over library variants (same box).  usage: bash tools/gpu_c1s3ab.sh TAG lib1.so|default ...
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/$lib; fi
  echo "== $lib" | tee -a gpurun_out/c1s3ab_$TAG.txt
  timeout -k 10 120 python -u tools/c1s3bench.py 2>/dev/null | tee -a gpurun_out/c1s3ab_$TAG.txt || exit 1
done
