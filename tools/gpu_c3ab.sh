#!/bin/bash
export TMPDIR=/tmp
for cfg in "" "AVDINO_C3_NT=2" "AVDINO_C3_GPW=4" "AVDINO_C3_NT=2 AVDINO_C3_GPW=4" "AVDINO_C3_OFF=1"; do
  env $cfg timeout -k 10 300 python tools/c3bench.py || exit $?
done
