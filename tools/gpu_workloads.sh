#!/bin/bash
# one bench line per BASELINE config shape on 1 GPU.  usage: bash tools/gpu_workloads.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/workloads_$TAG.jsonl
: > $O
for args in "--workload dino --mode mse" "--workload dino --mode infonce" \
            "--workload dino --mode semi_supervised" "--workload uni" "--workload simclr"; do
  timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline >> $O 2> gpurun_out/workloads_$TAG.err
  rc=$?; echo "$args rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<PY
import json
for l in open("$O"):
    d = json.loads(l)
    print(f'{d["value"]:10.1f} pairs/s {d["ms_per_step"]:8.2f} ms  {d["config"]["workload"][:90]}')
PY
