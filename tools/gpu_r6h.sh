#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dbg_prefetch6.py 25 nolds > gpurun_out/dbg6n.log 2>&1 || { tail -20 gpurun_out/dbg6n.log; exit 1; }
grep -v "amdgpu.ids\|(view, sample\|data_ptr" gpurun_out/dbg6n.log | grep -v "run differs False" | tail -25
timeout -k 10 400 python -u tools/dbg_prefetch6.py 25 > gpurun_out/dbg6.log 2>&1 || { tail -20 gpurun_out/dbg6.log; exit 1; }
grep -v "amdgpu.ids\|(view, sample\|data_ptr" gpurun_out/dbg6.log | grep -v "run differs False" | tail -25
