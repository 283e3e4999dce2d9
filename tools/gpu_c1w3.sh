#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cl.py tests/test_gpu_simclr.py tests/test_gpu_uni.py tests/test_gpu_benchsize.py -k "apply_wgrad or simclr or uni or Uni" -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/c1w3_tests.log 2>&1
rc=$?; grep -E "^E  |passed|failed|FAILED" gpurun_out/c1w3_tests.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload simclr --no-cpu-baseline > gpurun_out/bench_simclr_c1w3.json 2>gpurun_out/bench_simclr_c1w3.err || exit $?
grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/bench_simclr_c1w3.json
