#!/bin/bash
# The fused 56² layer backward under counters: HBM traffic (FETCH x2 + WRITE passes) and two SQ
# passes (LDS / wait / MFMA), the launch replayed alone 20 times after one step.
#   usage: bash tools/gpu_lbpmc.sh TAG
TAG=$1
KEY="${KEY:-cl_layer_bwd[7168x56x56x8->16 k5 apply]}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lbpmc_$TAG
[ -n "$NOTRAFFIC" ] || bash tools/gpu_pmc_key.sh $TAG "$KEY" || exit $?
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/lbpmc_$TAG/p$i -o run -- \
      python bench.py --steps 1 --warmup 2 --no-cpu-baseline --probe-dominant 20 --dominant "$KEY" \
      > gpurun_out/lbpmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/lbpmc_$TAG/p$i.log; exit 1; }
done
python tools/pmc_kernels.py gpurun_out/lbpmc_$TAG 40 | grep -A20 "${GREP:-lbwd}" > gpurun_out/lbpmc_$TAG.txt; cat gpurun_out/lbpmc_$TAG.txt
rm -rf gpurun_out/lbpmc_$TAG/p*/
