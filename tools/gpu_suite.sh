#!/bin/bash
# full GPU test suite into gpurun_out/suite_$1.log
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/suite_$1.log 2>&1; rc=$?
grep -E "^E  |passed|failed|FAILED" gpurun_out/suite_$1.log | cut -c1-250 | tail -15; exit $rc
