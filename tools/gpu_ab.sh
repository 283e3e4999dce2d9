#!/bin/bash
# Same-box A/B of library variants on the standalone op benchmark.
#   usage: FILT=cl_conv bash tools/gpu_ab.sh TAG lib1.so lib2.so ...   ("default" = the in-tree lib)
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/$lib; fi
  echo "== $lib" >> gpurun_out/ab_$TAG.txt
  timeout -k 10 300 python tools/opbench.py --filter "${FILT:-cl_conv}" 2>/dev/null | grep -v amdgpu >> gpurun_out/ab_$TAG.txt || exit $?
done
cat gpurun_out/ab_$TAG.txt
