#!/bin/bash
# Builds libavdino variants that differ in one compile-time macro of one source file into
# multimodal-ssl-avmnist_amd/avdino/variants/libavdino_<name>.so (select with AVDINO_LIB=...).
#   usage: bash tools/build_variants.sh SRC name1=MACRO=val name2=MACRO=val ...
#   e.g.   bash tools/build_variants.sh conv_c1p pf1=RC_PF=1 pf2=RC_PF=2   (several macros: A=1+B=2)
set -e
SRC=$1; shift
CS=multimodal-ssl-avmnist_amd/csrc
OUT=multimodal-ssl-avmnist_amd/avdino/variants
mkdir -p $OUT $CS/build/var
make -C $CS -j8 > /dev/null
for v in "$@"; do
  name=${v%%=*}; def=${v#*=}
  defs=""; IFS='+' read -ra parts <<< "$def"; for d in "${parts[@]}"; do defs="$defs -D$d"; done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I include \
      $defs -c $CS/$SRC.hip -o $CS/build/var/${SRC}_$name.o
  objs=$(ls $CS/build/*.o | grep -v "/$SRC.o$")
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libavdino_$name.so $objs $CS/build/var/${SRC}_$name.o
  echo "built $OUT/libavdino_$name.so ($def)"
done
