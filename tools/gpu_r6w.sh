#!/bin/bash
# round-6 lines of the other BASELINE configs (1 GPU): config 1 (uni), 3 (infonce), 4 (simclr),
# 5 (semi_supervised B=4096, bf16 and fp8)
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r6_workloads.jsonl
for args in "--workload uni" "--mode infonce" "--workload simclr --steps 60" "--mode semi_supervised --steps 20" "--mode semi_supervised --dtype fp8 --steps 20"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/w.json 2> gpurun_out/w.err || { echo "FAILED: $args"; tail -5 gpurun_out/w.err; exit 1; }
  head -1 gpurun_out/w.json >> gpurun_out/r6_workloads.jsonl
  python -c "import json; d=json.loads(open('gpurun_out/w.json').readline()); r=d['roofline']; print('$args', d['value'], d['ms_per_step'], r['kernel'][:50], r['avg_launch_us'], r['frac'])"
done
