#!/bin/bash
# Selected GPU test files, the bench line, then rocprof kernel stats of the graph-replayed bench
# (+ per-stream timeline) and of the eager bench.
#   usage: bash tools/gpu_prof.sh TAG [test files...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -q -m gpu --timeout 120 --timeout-method thread -rf \
      > gpurun_out/sel_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -aE "^E  |passed|failed|FAILED" gpurun_out/sel_$TAG.log | cut -c1-300 | tail -20
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cut -c1-200 gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1 || exit $?
python tools/timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/tl_$TAG.txt
python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 60 > gpurun_out/ks_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eager_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-graph --no-cpu-baseline > gpurun_out/be_$TAG.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_eager_$TAG/run_kernel_stats.csv 60 > gpurun_out/kse_$TAG.txt
head -4 gpurun_out/tl_$TAG.txt
