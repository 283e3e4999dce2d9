#!/bin/bash
# audio conv1 routed passes: the GPU tests of the Gram statistics / window moments / first-layer
# float64 checks, c1wbench per library variant and moments route, then a bench A/B.
#   usage: bash tools/gpu_c1w.sh TAG [variant ...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c1_gram.py tests/test_gpu_conv1_routes.py \
    tests/test_gpu_c1r3_codes.py tests/test_gpu_benchsize.py -k "c1 or conv1 or gram or routes or simclr" -v -s -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/c1w_$TAG.log 2>&1
rc=$?; grep -aE "PASSED|FAILED|ERROR|^E  |passed|failed|: [0-9.]+e-|loss|vs" gpurun_out/c1w_$TAG.log | cut -c1-200 | tail -80
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/c1wbench.py || exit $?
AVDINO_C1_MOMWIN=0 timeout -k 10 120 python tools/c1wbench.py || exit $?
for v in "$@"; do
  AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$v.so timeout -k 10 120 python tools/c1wbench.py || exit $?
done
bash tools/gpu_ab_env.sh c1w_$TAG 2 "-" "AVDINO_C1_MOMWIN=0"
