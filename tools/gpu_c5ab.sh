#!/bin/bash
# Config 5 fp8 step, library variants interleaved (+ the MX / fp8 GPU tests under each variant).
#   usage: bash tools/gpu_c5ab.sh TAG ROUNDS variant ...   ("default" = the in-tree lib)
TAG=$1; ROUNDS=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
lib_of() { if [ "$1" = default ]; then echo multimodal-ssl-avmnist_amd/avdino/libavdino.so; else echo multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$1.so; fi; }
for v in "$@"; do
  [ "$v" = default ] && continue
  AVDINO_LIB=$(lib_of $v) timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/c5ab_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/c5ab_${TAG}_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/c5ab_${TAG}_$v.log)"
done
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    AVDINO_LIB=$(lib_of $v) timeout -k 10 300 python bench.py --mode semi_supervised --dtype fp8 --no-cpu-baseline > gpurun_out/c5ab_$TAG.json 2> gpurun_out/c5ab_$TAG.err || { tail -5 gpurun_out/c5ab_$TAG.err; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('gpurun_out/c5ab_$TAG.json')); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/c5ab_$TAG.txt
  done
done
