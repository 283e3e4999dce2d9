#!/bin/bash
# lbwd tests, then a same-box interleaved A/B of the config-2 step: fused layer backward (row
# pairs, default lib), fused without row pairs (variant lib rp0), three launches (LAYER_BWD off)
TAG=$1; R=${2:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lbwd.py -v -s -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/r6_${TAG}_lbwd.log 2>&1
rc=$?; echo "lbwd tests rc=$rc"; grep -aE "PASSED|FAILED|^E  |passed|failed|layer bwd|dX vs" gpurun_out/r6_${TAG}_lbwd.log | cut -c1-250 | tail -20
[ $rc -le 1 ] || exit $rc
for r in $(seq $R); do
  for v in fused rp0 off; do
    unset AVDINO_LIB; spec=()
    [ $v = rp0 ] && export AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_rp0.so
    [ $v = off ] && spec=("ConvBranch.LAYER_BWD=False")
    line=$(timeout -k 10 300 python tools/ab_attr.py "${spec[@]}" -- --no-cpu-baseline --steps 40 2>gpurun_out/ab_$TAG.err) || { tail -5 gpurun_out/ab_$TAG.err; exit 1; }
    echo "$v $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'][:48], r['avg_launch_us'], r.get('isolated_avg_launch_us'), r['frac'])")" | tee -a gpurun_out/ab_$TAG.txt
  done
done
