#!/bin/bash
# PMC HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate passes) of one bench launch key, replayed
# alone 20 times after a step; merged into gpurun_out/traffic_TAG.json.
#   usage: bash tools/gpu_pmc_key.sh TAG "launch key" [bench.py args, e.g. --workload simclr]
TAG=$1; DOM=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc${C:0:1}_$TAG -o run -- \
      python bench.py --steps 1 --warmup 2 --no-cpu-baseline --probe-dominant 20 --dominant "$DOM" "$@" \
      > gpurun_out/probe${C:0:1}_$TAG.json 2> gpurun_out/probe${C:0:1}_$TAG.err
  rc=$?; echo "$DOM $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py gpurun_out/probeF_$TAG.json gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG gpurun_out/traffic_$TAG.json || exit 1
rm -rf gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG
