#!/bin/bash
# A/B library variant: libflr.so with one source compiled under extra flags,
# into abl/<name>/libflr.so (select with FLR_LIB=... at run time).
# usage: tools/ab_build.sh <name> "<extra hipcc flags>" [source.hip (default train_conv_t.hip)]
set -eu
cd "$(dirname "$0")/../multimodal-fl-security_amd/csrc"
name=$1; flags=$2; src=${3:-train_conv_t.hip}
stem=${src%.hip}
mkdir -p ../../abl/$name/obj
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $flags \
  -c $src -o ../../abl/$name/obj/$stem.o
objs=$(ls ../build/*.o | grep -v "/$stem")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../abl/$name/libflr.so $objs ../../abl/$name/obj/$stem.o
rm -rf ../../abl/$name/obj
echo built abl/$name/libflr.so
