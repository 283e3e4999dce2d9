#!/bin/bash
# Round-end style check on the 1-GPU box: GPU parity tests, smoke, default bench (with the CPU
# baseline), and a 2-rank gloo rehearsal of the N>1 bench path (both ranks on cuda:0).
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -rf > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 256 --dist-backend gloo \
    > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err
rc=$?; echo "bench2 rc=$rc"; cut -c1-300 gpurun_out/bench2_$TAG.json; tail -3 gpurun_out/bench2_$TAG.err
