#!/bin/bash
# c1r3 recompute passes: parity tests, then simclr bench A/B over AVDINO_L1_RECOMPUTE3
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cl.py -k "recompute or apply_wgrad" -q -s -m gpu --timeout 120 --timeout-method thread -rf > gpurun_out/c1r3_tests.log 2>&1
rc=$?; grep -E "^E  |passed|failed|FAILED|pass-4" gpurun_out/c1r3_tests.log | cut -c1-300 | tail -20; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  AVDINO_L1_RECOMPUTE3=$v timeout -k 10 300 python bench.py --workload simclr --no-cpu-baseline --steps 50 > gpurun_out/c1r3_$v.json 2> gpurun_out/c1r3_$v.err || { tail -5 gpurun_out/c1r3_$v.err; exit 1; }
  echo "RC3=$v $(grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/c1r3_$v.json | tr '\n' ' ')"
done
