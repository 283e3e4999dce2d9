#!/bin/bash
# times the conv launches for each libavdino variant.  usage: bash tools/gpu_wsvar.sh TAG v...
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cl.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$v.so timeout -k 10 300 python tools/opbench.py --filter ${FILT:-cl_conv_} > gpurun_out/opbench_${TAG}_$v.txt 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v "2048x\|x1->" gpurun_out/opbench_${TAG}_$v.txt | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
done
