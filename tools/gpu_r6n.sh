#!/bin/bash
# lbwd variants (library builds under variants/): tests of each, then config 2 alternating
#   usage: bash tools/gpu_r6n.sh TAG ROUNDS v1 v2 ...   (v = default or a variants/ name)
TAG=$1; R=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
VD=multimodal-ssl-avmnist_amd/avdino/variants
for v in "$@"; do
  [ $v = default ] && continue
  AVDINO_LIB=$VD/libavdino_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lbwd.py -q -s -m gpu --timeout 200 --timeout-method thread -rf > gpurun_out/r6n_${TAG}_$v.log 2>&1
  rc=$?; echo "$v lbwd tests rc=$rc $(grep -aE "passed|failed|dX vs" gpurun_out/r6n_${TAG}_$v.log | tail -3)"; [ $rc = 0 ] || exit $rc
done
for r in $(seq $R); do
  for v in "$@"; do
    if [ $v = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=$VD/libavdino_$v.so; fi
    line=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 2>gpurun_out/abn_$TAG.err) || { tail -5 gpurun_out/abn_$TAG.err; exit 1; }
    echo "$v $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'][:44], r['avg_launch_us'], r.get('isolated_avg_launch_us'), r['frac'])")" | tee -a gpurun_out/abn_$TAG.txt
  done
done
