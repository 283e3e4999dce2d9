#!/bin/bash
# fp8 conv path: tests, then config-5 bench lines (bf16 and fp8)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -v -s -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/fp8_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^E  |passed|failed|loss err" gpurun_out/fp8_tests.log | cut -c1-250 | tail -30; [ $rc -eq 0 ] || exit $rc
for dt in fp8 bf16; do
  timeout -k 10 300 python bench.py --mode semi_supervised --dtype $dt --no-cpu-baseline > gpurun_out/bench_c5_$dt.json 2> gpurun_out/bench_c5_$dt.err || { tail -5 gpurun_out/bench_c5_$dt.err; exit 1; }
  echo "$dt: $(grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/bench_c5_$dt.json | tr '\n' ' ')"
done
