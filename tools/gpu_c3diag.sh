#!/bin/bash
# conv3 diagnostics builds (wrong results): timings with staging / epilogue removed
export TMPDIR=/tmp C3B_ONLY=fwd
for d in 0 16; do
  echo "== diag $d"
  AVDINO_C3_DIAG=$d timeout -k 10 120 python tools/c3bench.py || exit $?
done
