#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lbwd.py -v -s -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/r6ad.log 2>&1
rc=$?; grep -aE "FAILED|^E  |passed|failed|dX vs" gpurun_out/r6ad.log | cut -c1-200 | tail -8; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/lbwd_ap.py 2>&1 | grep -v amdgpu.ids
AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_reuse0.so timeout -k 10 200 python tools/lbwd_ap.py 2>&1 | grep -v amdgpu.ids | sed 's/^/reuse0 /'
bash tools/gpu_r6o.sh ru 3 default reuse0
