#!/bin/bash
# Round-6 evidence: smoke(), the default bench line (CPU baseline included), rocprof kernel
# stats of the graph-replayed bench.   usage: bash tools/gpu_evid6.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/bench_$TAG.json; grep "in-graph candidates" gpurun_out/bench_$TAG.err | cut -c1-600
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 30 > $GRAFT_REPO_ROOT/gpurun_out/bprof_$TAG.json 2> $GRAFT_REPO_ROOT/gpurun_out/bprof_$TAG.err || exit $?
cd $GRAFT_REPO_ROOT && python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_$TAG.txt
head -6 gpurun_out/ks_$TAG.txt | cut -c1-160
