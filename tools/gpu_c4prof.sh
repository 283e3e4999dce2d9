#!/bin/bash
# Config 4 (SimCLR) evidence: PMC traffic of its dominant launch, then rocprof kernel stats of the
# graph-replayed bench.  usage: bash tools/gpu_c4prof.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc_key.sh c4$TAG "cl_conv_fwd[2048x56x56x32->64 k3p1 torch.bfloat16]" --workload simclr || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4$TAG -o run -- \
    python bench.py --workload simclr --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_c4$TAG.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_c4$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_c4$TAG.txt
head -30 gpurun_out/ks_c4$TAG.txt | cut -c1-200
