#!/bin/bash
# The default bench line (in-graph span timing of the watched launches) and rocprofv3 kernel
# stats of the same command, for the agreement check of roofline.avg_launch_us.
#   usage: bash tools/gpu_span.sh TAG [bench args...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print(d["value"], d["ms_per_step"])
for k in ("roofline", "roofline_hbm"):
    r = d.get(k) or {}
    print(k, r.get("kernel"), "avg", r.get("avg_launch_us"), "eager", r.get("eager_avg_launch_us"),
          "iso", r.get("isolated_avg_launch_us"), "frac", r.get("frac"), r.get("timing"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --no-cpu-baseline "$@" > gpurun_out/bprof_$TAG.json 2> gpurun_out/bprof_$TAG.err || exit $?
python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 12 > gpurun_out/ks_$TAG.txt
cut -c1-160 gpurun_out/ks_$TAG.txt
