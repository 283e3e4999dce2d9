#!/bin/bash
# Round-end evidence: full -m gpu suite, smoke(), default bench line (CPU baseline included),
# rocprof kernel stats of the graph-replayed bench and of the same bench eager (whose average
# per launch is what bench.py's roofline events time: eager steps after the timed region).
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/final_tests_$TAG.log 2>&1
rc=$?; grep -aE "^E  |passed|failed|FAILED" gpurun_out/final_tests_$TAG.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final_$TAG.json 2> gpurun_out/bench_final_$TAG.err || { tail -5 gpurun_out/bench_final_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_final_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final_$TAG -o run -- \
    python bench.py --no-cpu-baseline > gpurun_out/bprof_final_$TAG.json 2> gpurun_out/bprof_final_$TAG.err || exit $?
python tools/kstats.py gpurun_out/prof_final_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_final_$TAG.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eager_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-graph --no-cpu-baseline > gpurun_out/bprof_eager_$TAG.json 2> gpurun_out/bprof_eager_$TAG.err || exit $?
python tools/kstats.py gpurun_out/prof_eager_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_eager_$TAG.txt
head -4 gpurun_out/ks_final_$TAG.txt | cut -c1-150; head -4 gpurun_out/ks_eager_$TAG.txt | cut -c1-150
