#!/bin/bash
# configs 1 / 4 / 5 shapes: bench lines + rocprof kernel stats.  usage: bash tools/gpu_cfg.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for W in "simclr" "uni" ; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline > gpurun_out/bench_${W}_$TAG.json 2> gpurun_out/bench_${W}_$TAG.err
  echo "bench $W rc=$?"; cut -c1-160 gpurun_out/bench_${W}_$TAG.json; grep -o '"ms_per_step[^,]*' gpurun_out/bench_${W}_$TAG.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${W}_$TAG -o run -- \
      python bench.py --workload $W --no-cpu-baseline --no-graph --steps 10 --warmup 3 > /dev/null 2> gpurun_out/prof_${W}_$TAG.err
  echo "prof $W rc=$?"
  python tools/prof_summary.py gpurun_out/prof_${W}_$TAG/run_kernel_stats.csv 13 25 | cut -c1-170
done
timeout -k 10 300 python bench.py --mode semi_supervised --no-cpu-baseline > gpurun_out/bench_semi_$TAG.json 2> gpurun_out/bench_semi_$TAG.err
echo "bench semi rc=$?"; grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/bench_semi_$TAG.json
