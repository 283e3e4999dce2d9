#!/bin/bash
# Whole-step evidence: kernel trace of the graph-replayed bench, whole-step
# HBM traffic from FETCH_SIZE / WRITE_SIZE (separate passes, difference of a 4-step and a
# 1-step run = 3 steps), MFMA counters per kernel.  usage: bash tools/gpu_pmc_step.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g_$TAG -o run -- \
    $B --steps 20 --warmup 5 > gpurun_out/bprof_g_$TAG.json 2> gpurun_out/bprof_g_$TAG.err
echo "trace rc=$?"
for C in FETCH_SIZE WRITE_SIZE; do
  for S in 1 4; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${C}_${S}_$TAG -o run -- \
        $B --no-graph --steps $S --warmup 3 > gpurun_out/pmc_${C}_${S}_$TAG.json 2> gpurun_out/pmc_${C}_${S}_$TAG.err
    rc=$?; echo "$C steps=$S rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/pmc_sq_$TAG -o run -- \
    $B --no-graph --steps 1 --warmup 2 > gpurun_out/pmc_sq_$TAG.json 2> gpurun_out/pmc_sq_$TAG.err
echo "sq rc=$?"
python tools/pmc_step.py gpurun_out $TAG > gpurun_out/pmc_step_$TAG.txt 2>&1; echo "analysis rc=$?"; head -60 gpurun_out/pmc_step_$TAG.txt
