#!/bin/bash
# isolated + in-graph time of the audio conv1 apply pass: current library vs variants/libavdino_c1old.so
export TMPDIR=/tmp
mkdir -p gpurun_out
K="c1_apply_codes[7168x112x112x1->8 k5]"
for r in 1 2 3; do
  for v in default c1old; do
    if [ $v = default ]; then unset AVDINO_LIB; else export AVDINO_LIB=multimodal-ssl-avmnist_amd/avdino/variants/libavdino_$v.so; fi
    line=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --dominant "$K" 2>gpurun_out/abu.err) || { tail -5 gpurun_out/abu.err; exit 1; }
    echo "$v $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'][:40], r['avg_launch_us'], r.get('isolated_avg_launch_us'))")" | tee -a gpurun_out/abu.txt
  done
done
