#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
KEEP_EVENTS_RING=4096 timeout -k 10 900 python -u tools/pytest_keep_events.py tests/test_gpu_step.py tests/test_gpu_graph.py tests/test_gpu_benchsize.py -q -m gpu --timeout 400 --timeout-method thread -rf > gpurun_out/seg2.log 2>&1
rc=$?; echo "keep-events ring 4096 rc=$rc :: $(grep -aE 'passed|failed|Fatal' gpurun_out/seg2.log | tail -1)"; exit $rc
