#!/bin/bash
# SQ counters of the audio conv1 passes alone (tools/c1wbench.py): LDS array / conflict /
# unaligned cycles, LDS issue stalls, wave-parked cycles.  usage: bash tools/gpu_c1pmc.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d gpurun_out/c1pmc_$TAG -o run -- python tools/c1wbench.py > gpurun_out/c1pmc_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c1pmc_$TAG.log; exit $rc; }
python tools/pmc_kernels.py gpurun_out/c1pmc_$TAG > gpurun_out/c1pmc_$TAG.txt
grep -A9 "c1p8" gpurun_out/c1pmc_$TAG.txt | cut -c1-200
