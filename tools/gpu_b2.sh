#!/bin/bash
# bench with small warm-ups (graph capture inside the warm-up) and the 2-rank gloo rehearsal
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 5 --warmup $w --no-cpu-baseline > gpurun_out/bw${w}_$TAG.json 2> gpurun_out/bw${w}_$TAG.err
  rc=$?; echo "warmup $w rc=$rc"; cut -c1-120 gpurun_out/bw${w}_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bw${w}_$TAG.err; exit $rc; }
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 256 --dist-backend gloo \
    > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err
rc=$?; echo "bench2 rc=$rc"; cut -c1-300 gpurun_out/bench2_$TAG.json; tail -3 gpurun_out/bench2_$TAG.err
