#!/bin/bash
# Builds libavdino variants that differ only in one source's layer table (-D<MACRO>=n) into
# multimodal-ssl-avmnist_amd/avdino/variants/ (select one with AVDINO_LIB=...).
#   usage: SRC=conv_ws MACRO=WS_VARIANT bash tools/build_ws_variants.sh 0 1 2 3
set -e
cd "$(dirname "$0")/../multimodal-ssl-avmnist_amd/csrc"
make -j8 ARCH=gfx950 > /dev/null
mkdir -p ../avdino/variants
SRC=${SRC:-conv_ws}; MACRO=${MACRO:-WS_VARIANT}
OBJS=$(ls build/*.o | grep -v "build/$SRC.o")
for v in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -D$MACRO=$v -I../../include -c $SRC.hip -o build/${SRC}_v$v.o &
done
wait
for v in "$@"; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../avdino/variants/libavdino_v$v.so $OBJS build/${SRC}_v$v.o
  rm -f build/${SRC}_v$v.o
done
