#!/bin/bash
# The -m gpu suite (one pytest process), the default bench line, then the phase timeline of the
# unprofiled replayed step (phase_marks.py).   usage: bash tools/gpu_suite_marks.sh TAG
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_suite.sh $TAG || exit $?
timeout -k 10 300 python tools/phase_marks.py --steps 8 > gpurun_out/marks_$TAG.txt 2>&1
echo "marks rc=$?"; tail -3 gpurun_out/marks_$TAG.txt
