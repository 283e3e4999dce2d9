#!/bin/bash
# SQ counter passes over one bench step (kernel time breakdown: wait / issue-stall / active,
# VALU vs MFMA vs LDS instruction counts).  usage: bash tools/gpu_sqpmc.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d gpurun_out/sq1_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sq1_$TAG.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sq1_$TAG.log; exit $rc; }
python tools/pmc_kernels.py gpurun_out/sq1_$TAG > gpurun_out/sq_$TAG.txt
head -40 gpurun_out/sq_$TAG.txt | cut -c1-260
