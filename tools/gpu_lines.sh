#!/bin/bash
# Bench lines of every BASELINE config (no CPU baseline): config 5 bf16 and fp8 (B=4096), config 4
# SimCLR (all 4 modality graphs captured before timing), config 3 InfoNCE, config 1 UniModal, then the default config 2 line.
#   usage: bash tools/gpu_lines.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/lines_$TAG.jsonl; : > $out
run() {   # label, env, args
  local label=$1 envs=$2; shift 2
  line=$(env $envs timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2> gpurun_out/lines_$TAG.err) || { echo "FAILED $label"; tail -5 gpurun_out/lines_$TAG.err; exit 1; }
  echo "{\"label\": \"$label\", \"line\": $line}" >> $out
  echo "$label: $(echo "$line" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['unit'], d['ms_per_step'], 'ms', 'graph', d.get('graph'), 'host_ms', d.get('host_issue_ms_per_step'))")"
}
run c5_bf16 "" --mode semi_supervised --dtype bf16
run c5_fp8 "" --mode semi_supervised --dtype fp8
run c4_simclr "" --workload simclr
run c3_infonce "" --mode infonce
run c1_uni "" --workload uni
run c2_mse "" --mode mse
