#!/bin/bash
# Experiment build over several sources: exp/<name>/libgi_amd.so = the product objects with the
# listed csrc stems recompiled under the extra flags (GI_AMD_LIB=exp/<name>/libgi_amd.so).
# usage: tools/exp_build2.sh <name> "<extra hipcc flags>" <stem> [<stem> ...]
set -e
cd "$(dirname "$0")/../global-illumination_amd"
make -s -j8 libgi_amd.so
D=../exp/$1
FL=$2
shift 2
mkdir -p $D
OBJS=""
for o in build/*.o; do
  st=$(basename $o .o)
  if [[ " $* " == *" $st "* ]]; then
    SRC=csrc/$st.hip; [ -f $SRC ] || SRC="-x hip csrc/$st.cpp"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc $FL -c $SRC -o $D/$st.o 2>/dev/null
    OBJS="$OBJS $D/$st.o"
  else
    OBJS="$OBJS $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libgi_amd.so $OBJS -lz -lpthread
echo "built $D/libgi_amd.so"
