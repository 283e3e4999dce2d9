#!/bin/bash
# HBM traffic of the bench's dominant launch: two counter passes (FETCH_SIZE and WRITE_SIZE do
# not fit one TCC pass), each replaying only that launch K times.  usage: bash tools/gpu_pmc.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
K=20
# the roofline kernel of this round's bench line (gpu_round.sh writes it), so the counters
# measure exactly the launch the bench reports
# (or pass it as DOM=... when the bench ran in another call: gpurun_out/ does not travel)
DOM=${DOM:-$(python -c "import json,sys; print(json.loads(open('gpurun_out/bench_$TAG.json').readline())['roofline']['kernel'])")}
echo "dominant: $DOM"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcF_$TAG -o run -- \
    python bench.py --steps 1 --warmup 2 --no-cpu-baseline --probe-dominant $K --dominant "$DOM" > gpurun_out/probeF_$TAG.json 2> gpurun_out/probeF_$TAG.err \
&& timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcW_$TAG -o run -- \
    python bench.py --steps 1 --warmup 2 --no-cpu-baseline --probe-dominant $K --dominant "$DOM" > gpurun_out/probeW_$TAG.json 2> gpurun_out/probeW_$TAG.err \
&& python tools/pmc_traffic.py gpurun_out/probeF_$TAG.json gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG gpurun_out/traffic_$TAG.json
echo "pmc rc=$?"
