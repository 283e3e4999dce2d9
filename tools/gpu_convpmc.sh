#!/bin/bash
# SQ counter passes over the conv launches of one step (opbench replay).  usage: bash tools/gpu_convpmc.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d gpurun_out/cp1_$TAG -o run -- python tools/opbench.py --filter ${FILT:-cl_conv} --reps 1 > gpurun_out/cp1_$TAG.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/cp1_$TAG.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/cp2_$TAG -o run -- python tools/opbench.py --filter ${FILT:-cl_conv} --reps 1 > gpurun_out/cp2_$TAG.log 2>&1
rc=$?; echo "pass2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/cp2_$TAG.log; exit $rc; }
python tools/pmc_kernels.py gpurun_out/cp1_$TAG gpurun_out/cp2_$TAG > gpurun_out/convpmc_$TAG.txt
cut -c1-400 gpurun_out/convpmc_$TAG.txt | head -40
