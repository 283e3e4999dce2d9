#!/bin/bash
# lbwd double-buffer variant: its tests, then config 2 alternating default / db1 on one box
TAG=$1; R=${2:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
V=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_db1.so
AVDINO_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_lbwd.py -v -s -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/r6m_$TAG.log 2>&1
rc=$?; echo "db1 lbwd tests rc=$rc"; grep -aE "FAILED|^E  |passed|failed|dX vs|bit" gpurun_out/r6m_$TAG.log | cut -c1-200 | tail -12; [ $rc = 0 ] || exit $rc
for r in $(seq $R); do
  for v in default db1; do
    if [ $v = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=$V; fi
    line=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 2>gpurun_out/abm_$TAG.err) || { tail -5 gpurun_out/abm_$TAG.err; exit 1; }
    echo "$v $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'][:44], r['avg_launch_us'], r.get('isolated_avg_launch_us'), r['frac'])")" | tee -a gpurun_out/abm_$TAG.txt
  done
done
