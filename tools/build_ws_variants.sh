#!/bin/bash
# Builds libavdino variants that differ only in conv_ws.hip's layer table (-DWS_VARIANT=n) into
# multimodal-ssl-avmnist_amd/avdino/variants/ (select one with AVDINO_LIB=...).
set -e
cd "$(dirname "$0")/../multimodal-ssl-avmnist_amd/csrc"
make -j8 ARCH=gfx950 > /dev/null
mkdir -p ../avdino/variants
OBJS=$(ls build/*.o | grep -v conv_ws)
for v in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DWS_VARIANT=$v -I../../include -c conv_ws.hip -o build/conv_ws_v$v.o &
done
wait
for v in "$@"; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../avdino/variants/libavdino_v$v.so $OBJS build/conv_ws_v$v.o
  mv build/conv_ws_v$v.o build/v$v.o.keep
done
