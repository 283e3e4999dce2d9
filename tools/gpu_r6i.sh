#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/dbg_guard.py 4096 1024 > gpurun_out/guard.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/guard.log | tail -60; exit $rc
