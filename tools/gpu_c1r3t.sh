export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cl.py -k "recompute" -q -s -m gpu --timeout 120 --timeout-method thread -rf > gpurun_out/c1r3_tests.log 2>&1; rc=$?
grep -E "^E  |passed|failed|pass-4" gpurun_out/c1r3_tests.log | cut -c1-250; exit $rc
