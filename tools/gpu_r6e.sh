#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dbg_prefetch4.py 8 A B E F > gpurun_out/dbg4.log 2>&1; grep -v amdgpu.ids gpurun_out/dbg4.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_contrastive_size.py -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6_e_xent.log 2>&1
rc=$?; echo "xent tests rc=$rc"; grep -aE "PASSED|FAILED|^E  |passed|failed|xent R|NT-Xent|InfoNCE" gpurun_out/r6_e_xent.log | cut -c1-250 | tail -30
[ $rc -le 1 ] || exit $rc
for w in "--workload simclr" "--mode infonce"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 $w > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err || { tail -5 gpurun_out/bench_e.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_e.json').readline()); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel'][:50], d['roofline']['avg_launch_us'])"
done
