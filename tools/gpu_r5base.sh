#!/bin/bash
# Bench line + PMC traffic of the launches the bench now reports (the 14^2 and 56^2 weight
# gradients, replayed alone) + whole-step PMC bytes.  usage: bash tools/gpu_r5base.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_$TAG.json
rm -f gpurun_out/traffic_$TAG.json
for DOM in "cl_conv_wgrad[7168x14x14x32->64 k5p2 torch.bfloat16] @side" "cl_conv_wgrad[7168x56x56x8->16 k5p2 torch.bfloat16] @side"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc${C:0:1}_$TAG -o run -- \
        python bench.py --steps 1 --warmup 2 --no-cpu-baseline --probe-dominant 20 --dominant "$DOM" \
        > gpurun_out/probe${C:0:1}_$TAG.json 2> gpurun_out/probe${C:0:1}_$TAG.err
    rc=$?; echo "$DOM $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python tools/pmc_traffic.py gpurun_out/probeF_$TAG.json gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG gpurun_out/traffic_$TAG.json || exit 1
  rm -rf gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG
done
bash tools/gpu_pmc_step.sh $TAG
