#!/bin/bash
# 3x3 weight-gradient kernel: bench-size parity, the conv unit tests, then timings per strip size
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_benchsize.py -k "ws_kernels" > gpurun_out/c3w_bench_tests.log 2>&1 || { tail -30 gpurun_out/c3w_bench_tests.log; exit 1; }
tail -3 gpurun_out/c3w_bench_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_cl.py tests/test_gpu_simclr.py > gpurun_out/c3w_cl_tests.log 2>&1 || { tail -30 gpurun_out/c3w_cl_tests.log; exit 1; }
tail -3 gpurun_out/c3w_cl_tests.log
for cfg in "" "AVDINO_C3_TR=2" "AVDINO_C3_WBLK=512" "AVDINO_C3_WBLK=2048"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python tools/c3bench.py || exit $?
done
