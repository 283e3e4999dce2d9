#!/bin/bash
# round-end style check: full -m gpu suite, smoke(), default bench line, rocprof kernel stats
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/final_tests_$TAG.log 2>&1
rc=$?; grep -E "^E  |passed|failed|FAILED" gpurun_out/final_tests_$TAG.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final_$TAG.json 2> gpurun_out/bench_final_$TAG.err || { tail -5 gpurun_out/bench_final_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_final_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final_$TAG -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bprof_final_$TAG.json 2> gpurun_out/bprof_final_$TAG.err || exit $?
python tools/prof_summary.py $(find gpurun_out/prof_final_$TAG -name "*kernel_stats.csv" | head -1) 25 40 > gpurun_out/kstats_final_$TAG.txt 2>&1; head -12 gpurun_out/kstats_final_$TAG.txt | cut -c1-160
