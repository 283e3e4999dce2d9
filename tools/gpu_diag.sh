#!/bin/bash
# kernel diagnosis: per-op replay timings, then SQ counters over a short bench run
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/opbench.py > gpurun_out/opbench_$TAG.txt 2>&1
echo "opbench rc=$?"; head -40 gpurun_out/opbench_$TAG.txt
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES \
    --kernel-trace --output-format csv -d gpurun_out/pmcSQ_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcSQ_$TAG.log 2>&1
echo "pmc rc=$?"
python tools/pmc_kernels.py gpurun_out/pmcSQ_$TAG > gpurun_out/pmcSQ_$TAG.txt 2>&1; head -30 gpurun_out/pmcSQ_$TAG.txt | cut -c1-330
