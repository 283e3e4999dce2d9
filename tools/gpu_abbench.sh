#!/bin/bash
# Same-box A/B of library variants on the whole step (bench.py, no CPU baseline), interleaved.
#   usage: bash tools/gpu_abbench.sh TAG lib1.so lib2.so ...   ("default" = the in-tree lib)
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/$lib; fi
  v=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$lib $v" | tee -a gpurun_out/abb_$TAG.txt
done
