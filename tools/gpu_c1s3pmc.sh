#!/bin/bash
# SQ counters of config 4's 3x3 first-layer passes alone (tools/c1s3bench.py, 112^2 + 28^2):
# two passes (LDS / wait cycles; issue / instruction mix).  usage: bash tools/gpu_c1s3pmc.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d gpurun_out/c1s3pmc1_$TAG -o run -- python tools/c1s3bench.py > gpurun_out/c1s3pmc1_$TAG.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c1s3pmc1_$TAG.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-trace --output-format csv -d gpurun_out/c1s3pmc2_$TAG -o run -- python tools/c1s3bench.py > gpurun_out/c1s3pmc2_$TAG.log 2>&1
rc=$?; echo "pass2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c1s3pmc2_$TAG.log; exit $rc; }
python tools/pmc_kernels.py gpurun_out/c1s3pmc1_$TAG > gpurun_out/c1s3pmc_$TAG.txt
python tools/pmc_kernels.py gpurun_out/c1s3pmc2_$TAG >> gpurun_out/c1s3pmc_$TAG.txt
grep -A10 "c1s3\|c1r3" gpurun_out/c1s3pmc_$TAG.txt | cut -c1-220 | head -80
