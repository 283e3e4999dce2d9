#!/bin/bash
# interleaved same-box A/B of env settings, 3 rounds.  usage: bash tools/gpu_ab3.sh TAG "A" "B" ...
TAG=$1; shift
for r in 1 2 3; do bash tools/gpu_abenv.sh $TAG "$@" || exit 1; done
