#!/bin/bash
# tools/buildvar.sh NAME "-DFOO=1 ..." [SRC...]: lib/var_NAME.so = the Makefile's libbic.so objects with the
# given sources (default: bic_fused.hip and bic_kernels.hip) recompiled under extra defines, for same-box
# A/B timing (tools/ab.sh). The other objects are the Makefile's own list.
set -e
cd "$(dirname "$0")/../binary-image-compression_amd"
N=$1; D=$2; shift 2
SRCS=${@:-csrc/bic_fused.hip csrc/bic_kernels.hip}
make -s lib/libbic.so
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I../include -Icsrc $D"
mkdir -p build/var lib
OBJS=$(sed -n 's/^lib\/libbic.so:\(.*\)$/\1/p' Makefile | tr ' ' '\n' | grep '\.o$')
OUT=""
for o in $OBJS; do
  b=$(basename $o .o)
  if echo "$SRCS" | grep -q "$b.hip\|$b.cpp"; then
    src=$(echo $SRCS | tr ' ' '\n' | grep "$b\.")
    x=""; [[ $src == *.cpp ]] && x="-x hip"
    /opt/rocm/bin/hipcc $FL $x -c -o build/var/${N}_$b.o $src &
    OUT="$OUT build/var/${N}_$b.o"
  else
    OUT="$OUT $o"
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/var_$N.so $OUT
echo lib/var_$N.so
