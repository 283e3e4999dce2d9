#!/bin/bash
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cl.py tests/test_gpu_benchsize.py tests/test_gpu_simclr.py tests/test_gpu_uni.py tests/test_gpu_graph.py -q -m gpu --timeout 300 --timeout-method thread -rf -x > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload simclr --no-cpu-baseline > gpurun_out/bench_simclr_$TAG.json 2>/dev/null
echo "bench rc=$?"; grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/bench_simclr_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_simclr_$TAG -o run -- \
    python bench.py --workload simclr --no-cpu-baseline --no-graph --steps 10 --warmup 3 > /dev/null 2>&1
echo "prof rc=$?"
python tools/prof_summary.py gpurun_out/prof_simclr_$TAG/run_kernel_stats.csv 13 16 | cut -c1-170
