#!/bin/bash
# SQ / TCC counters of the conv launches replayed alone (tools/opbench.py --filter cl_conv),
# one rocprofv3 pass per counter group.  usage: bash tools/gpu_wspmc.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/wspmc_$TAG
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/wspmc_$TAG/p$i -o run -- \
      python tools/opbench.py --filter cl_conv --reps 3 > gpurun_out/wspmc_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/wspmc_$TAG/p$i.log; exit $rc; }
done
python tools/pmc_kernels.py gpurun_out/wspmc_$TAG 170 > gpurun_out/wspmc_$TAG.txt
grep -A16 "conv_ws_kernel\|wgrad_ws_kernel" gpurun_out/wspmc_$TAG.txt | cut -c1-200 | head -150
