#!/bin/bash
# augmentation: GPU tests, then the augmentation / real-data step benchmark
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_augment.py -v -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/aug_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^E  |passed|failed" gpurun_out/aug_tests.log | cut -c1-250 | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/aug_bench.py > gpurun_out/aug_bench.txt 2>&1; rc=$?; cat gpurun_out/aug_bench.txt | tail -20; exit $rc
