#!/bin/bash
# rocprof kernel stats of the config-5 (semi-supervised, B = 4096) bench step, bf16 and fp8
#   usage: bash tools/gpu_c5prof.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for dt in fp8 bf16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5${dt}_$TAG -o run -- \
      python bench.py --mode semi_supervised --dtype $dt --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/c5prof_${dt}_$TAG.json 2> gpurun_out/c5prof_$TAG.err || { tail -5 gpurun_out/c5prof_$TAG.err; exit 1; }
  python tools/kstats.py gpurun_out/prof_c5${dt}_$TAG/run_kernel_stats.csv 30 > gpurun_out/ks_c5${dt}_$TAG.txt
done
