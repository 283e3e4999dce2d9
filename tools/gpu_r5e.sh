#!/bin/bash
# Selected tests (-k filter) + bench line + graph-replay kernel trace + phase marks.
# usage: K="expr" bash tools/gpu_r5e.sh TAG "tests..."   (K optional: a pytest -k expression)
TAG=$1; TESTS=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread -rf -s > gpurun_out/t_$TAG.log 2>&1
  rc=$?; grep -aE "^E  |passed|failed|FAILED|Error|curve|ours bf16" gpurun_out/t_$TAG.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-330 gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bprof_$TAG.json 2> gpurun_out/bprof_$TAG.err || exit $?
python tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 > gpurun_out/ks_$TAG.txt
python tools/trace_by_grid.py gpurun_out/prof_$TAG/run_kernel_trace.csv 25 300 > gpurun_out/grid_$TAG.txt
grep -E "gemm_pair|gemm_mfma_kernel<2, 128, 256|sum_rows|all kernels" gpurun_out/grid_$TAG.txt | head -12
timeout -k 10 300 python tools/phase_marks.py --steps 8 > gpurun_out/marks_$TAG.txt 2>&1
echo "marks rc=$?"; grep -E "bwd.main_heads|heads_joined|end$|# " gpurun_out/marks_$TAG.txt | head
