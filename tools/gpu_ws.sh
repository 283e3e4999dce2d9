#!/bin/bash
# conv_ws variants: cl tests under each variant library, per-launch opbench of the conv
# launches, then an interleaved whole-step A/B.
#   usage: [WS_TESTS="variant ..."] bash tools/gpu_ws.sh TAG variant ...
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $WS_TESTS; do
  lib=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$v.so
  [ "$v" = default ] && lib=multimodal-ssl-avmnist_amd/avdino/libavdino.so
  AVDINO_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cl.py tests/test_gpu_benchsize.py -k "ws or dgrad or wgrad or cl_" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ws_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/ws_${TAG}_$v.log; exit 1; }
  tail -1 gpurun_out/ws_${TAG}_$v.log
done
timeout -k 10 180 python tools/opbench.py --filter cl_conv > gpurun_out/wsop_${TAG}_default.txt 2>&1 || exit $?
for v in "$@"; do
  AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$v.so timeout -k 10 180 python tools/opbench.py --filter cl_conv > gpurun_out/wsop_${TAG}_$v.txt 2>&1 || exit $?
done
libs=""; for v in "$@"; do libs="$libs libavdino_$v.so"; done
bash tools/gpu_abbench.sh ws_$TAG default $libs default $libs
