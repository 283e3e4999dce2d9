#!/bin/bash
# 3x3 conv kernels: bench-size parity, the conv unit tests, then per-shape timings
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_benchsize.py -k "ws_kernels" > gpurun_out/c3w_bench_tests.log 2>&1 || { tail -30 gpurun_out/c3w_bench_tests.log; exit 1; }
tail -3 gpurun_out/c3w_bench_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_cl.py tests/test_gpu_simclr.py tests/test_gpu_uni.py > gpurun_out/c3w_cl_tests.log 2>&1 || { tail -30 gpurun_out/c3w_cl_tests.log; exit 1; }
tail -3 gpurun_out/c3w_cl_tests.log
for cfg in "" "AVDINO_C3_GPW=4"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python tools/c3bench.py || exit $?
done
timeout -k 10 300 python bench.py --workload simclr --no-cpu-baseline > gpurun_out/bench_simclr_glds.json 2>gpurun_out/bench_simclr_glds.err
grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/bench_simclr_glds.json
