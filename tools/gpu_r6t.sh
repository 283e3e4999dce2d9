#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_evid6.sh r6e2 || exit $?
bash tools/gpu_pmc_key.sh r6c1 "c1_apply_codes[7168x112x112x1->8 k5]"
