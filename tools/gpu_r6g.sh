#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_contrastive_size.py > gpurun_out/xent_t.log 2>&1 || { tail -30 gpurun_out/xent_t.log; exit 1; }
tail -3 gpurun_out/xent_t.log
timeout -k 10 500 python -u tools/dbg_prefetch5.py 20 C A > gpurun_out/dbg5c.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/dbg5c.log; exit $rc
