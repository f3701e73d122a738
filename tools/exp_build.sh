#!/bin/bash
# Experiment build: exp/<name>/libgi_amd.so = the product objects with <file>.hip recompiled
# under extra flags; select it at run time with GI_AMD_LIB=exp/<name>/libgi_amd.so.
# usage: tools/exp_build.sh <name> <csrc file stem, e.g. gi_knn_chunk> "<extra hipcc flags>"
set -e
cd "$(dirname "$0")/../global-illumination_amd"
make -s -j8 libgi_amd.so
D=../exp/$1
mkdir -p $D
OBJS=""
for o in build/*.o; do
  if [ "$(basename $o .o)" = "$2" ]; then
    SRC=csrc/$2.hip; [ -f $SRC ] || SRC="-x hip csrc/$2.cpp"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc $3 -c $SRC -o $D/$2.o
    OBJS="$OBJS $D/$2.o"
  else
    OBJS="$OBJS $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libgi_amd.so $OBJS -lz -lpthread
echo "built $D/libgi_amd.so"
