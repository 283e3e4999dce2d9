#!/bin/bash
# full check: all GPU tests, smoke, profiled bench (kernel trace + stats), default bench with
# CPU baseline.  usage: bash tools/gpu_round.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -rf > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^E  |passed|failed|FAILED" gpurun_out/t_$TAG.log | cut -c1-300 | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric gpurun_out/b_$TAG.log | cut -c1-250
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench rc=$?"; cut -c1-300 gpurun_out/bench_$TAG.json
