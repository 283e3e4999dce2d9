#!/bin/bash
# graph tests + full GPU suite + bench (graph / eager)
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh $TAG tests/test_gpu_graph.py tests/test_gpu_boundary.py tests/test_gpu_simclr.py
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_g_$TAG.json 2> gpurun_out/bench_g_$TAG.err
echo "bench graph rc=$?"; cut -c1-300 gpurun_out/bench_g_$TAG.json; grep -o '"step_roofline.*' gpurun_out/bench_g_$TAG.json | cut -c1-500; tail -3 gpurun_out/bench_g_$TAG.err
timeout -k 10 600 python bench.py --no-cpu-baseline --no-graph > gpurun_out/bench_e_$TAG.json 2> gpurun_out/bench_e_$TAG.err
echo "bench eager rc=$?"; cut -c1-300 gpurun_out/bench_e_$TAG.json; grep -o '"timed_region.*' gpurun_out/bench_e_$TAG.json | cut -c1-300
timeout -k 10 600 python bench.py --no-cpu-baseline --workload uni > gpurun_out/bench_u_$TAG.json 2> gpurun_out/bench_u_$TAG.err
echo "bench uni rc=$?"; cut -c1-200 gpurun_out/bench_u_$TAG.json; grep -o '"timed_region.*' gpurun_out/bench_u_$TAG.json | cut -c1-200
