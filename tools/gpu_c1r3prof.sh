#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0; do
  AVDINO_L1_RECOMPUTE3=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rc3p$v -o run -- python bench.py --workload simclr --no-cpu-baseline --steps 20 > gpurun_out/rc3p$v.json 2> gpurun_out/rc3p$v.err || exit $?
done
