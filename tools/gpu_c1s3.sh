#!/bin/bash
# config 4's 3x3 first layer on the pixel-major passes: parity tests + timing (tools/c1s3bench.py)
set -o pipefail
mkdir -p gpurun_out
T=${1:-c1s3}
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_c1r3_codes.py "tests/test_gpu_cl.py::test_cl_c1_recompute_passes_match_stored_y_path" \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 120 python -u tools/c1s3bench.py > gpurun_out/${T}_bench.txt 2>&1 && cat gpurun_out/${T}_bench.txt
