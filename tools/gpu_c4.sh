#!/bin/bash
# configs 1 and 4 with enough warm-up for every SimCLR modality pair's graph capture
TAG=$1
mkdir -p gpurun_out
for args in "--workload simclr --steps 60 --warmup 12" "--workload uni --steps 200 --warmup 5"; do
  timeout -k 10 300 python bench.py $args --no-cpu-baseline >> gpurun_out/c14_$TAG.jsonl 2> gpurun_out/c14_$TAG.err; rc=$?
  echo "$args rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cut -c1-200 gpurun_out/c14_$TAG.jsonl
