#!/bin/bash
# A/B library variant: libflr.so with train_conv_t.hip compiled under extra
# flags, into abl/<name>/libflr.so (select with FLR_LIB=... at run time).
# usage: tools/ab_build.sh <name> "<extra hipcc flags>"
set -eu
cd "$(dirname "$0")/../multimodal-fl-security_amd/csrc"
name=$1; flags=$2
mkdir -p ../../abl/$name/obj
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $flags \
  -c train_conv_t.hip -o ../../abl/$name/obj/train_conv_t.o
objs=$(ls ../build/*.o | grep -v "train_conv_t")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../abl/$name/libflr.so $objs ../../abl/$name/obj/train_conv_t.o
rm -rf ../../abl/$name/obj
echo built abl/$name/libflr.so
