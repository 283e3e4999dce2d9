#!/bin/bash
# 2-rank gloo rehearsal of the data-parallel bench (both ranks on the one GPU): the default
# workload, InfoNCE with all-gathered negatives (config 3) and SimCLR (config 4), each with
# the captured step (host points around the collectives) and bucketed gradient all-reduce.
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
port=29541
for wl in "--mode mse" "--mode infonce" "--workload simclr"; do
  name=$(echo $wl | tr -d ' -')
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 2 --steps 5 --warmup 3 --batch 128 $wl --dist-backend gloo \
      --no-cpu-baseline > gpurun_out/r2_${name}_$TAG.json 2> gpurun_out/r2_${name}_$TAG.err
  rc=$?; echo "$wl rc=$rc"; cut -c1-200 gpurun_out/r2_${name}_$TAG.json
  grep -o '"graph": [a-z]*' gpurun_out/r2_${name}_$TAG.json
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r2_${name}_$TAG.err; exit $rc; }
  port=$((port+1))
done
