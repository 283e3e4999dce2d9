#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dbg_prefetch5.py 20 F A > gpurun_out/dbg5f.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/dbg5f.log | grep -v "^   "; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_augment.py > gpurun_out/aug_t.log 2>&1; rc=$?; tail -4 gpurun_out/aug_t.log; exit $rc
