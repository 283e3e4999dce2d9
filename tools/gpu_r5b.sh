#!/bin/bash
# Selected GPU tests + bench line + config-5 probe line + graph-replay kernel trace.
# usage: bash tools/gpu_r5b.sh TAG "tests/test_a.py tests/test_b.py"
TAG=$1
TESTS=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/t_$TAG.log 2>&1
  rc=$?; grep -aE "^E  |passed|failed|FAILED|Error" gpurun_out/t_$TAG.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-330 gpurun_out/bench_$TAG.json
if [ -n "$PROBE" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --mode semi_supervised --probe --steps 10 --warmup 3 > gpurun_out/bench_probe_$TAG.json 2> gpurun_out/bench_probe_$TAG.err || { tail -5 gpurun_out/bench_probe_$TAG.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_probe_$TAG.json').readline()); print(d['value'], d['ms_per_step'], d['probe'])"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bprof_$TAG.json 2> gpurun_out/bprof_$TAG.err || exit $?
python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_$TAG.txt
python tools/trace_by_grid.py gpurun_out/prof_$TAG/run_kernel_trace.csv 25 60 > gpurun_out/grid_$TAG.txt
head -12 gpurun_out/ks_$TAG.txt | cut -c1-150; grep -E "sum_rows|all kernels" gpurun_out/grid_$TAG.txt
