#!/bin/bash
# PMC passes over one conv3 op / shape: bash tools/gpu_c3pmc.sh OP SHAPE
export TMPDIR=/tmp
mkdir -p gpurun_out/c3pmc
export C3B_ONLY=$1 C3B_SHAPE=$2
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/c3pmc/p$i -o run -- python tools/c3bench.py > gpurun_out/c3pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/c3pmc/p$i.log; exit 1; }
done
python tools/pmc_kernels.py gpurun_out/c3pmc
