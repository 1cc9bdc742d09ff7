#!/bin/bash
# tools/variant.sh NAME FUSED_SRC [KERNELS_SRC]: build binary-image-compression_amd/lib/var_NAME.so from
# alternative sources of bic_fused.hip (and bic_kernels.hip) for same-box A/B timing (tools/ab.sh).
# The other objects are the Makefile's own libbic.so list (read from its rule, so the two cannot drift).
set -e
cd "$(dirname "$0")/../binary-image-compression_amd"
N=$1; F=$2; K=${3:-csrc/bic_kernels.hip}
make -s lib/libbic.so
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I../include -Icsrc"
mkdir -p build/var lib
/opt/rocm/bin/hipcc $FL -c -o build/var/${N}_fused.o $F &
/opt/rocm/bin/hipcc $FL -c -o build/var/${N}_kern.o $K &
wait
OTHERS=$(sed -n 's/^lib\/libbic.so:\(.*\)$/\1/p' Makefile | tr ' ' '\n' | grep '\.o$' | grep -v -e bic_fused.o -e bic_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/var_$N.so build/var/${N}_fused.o build/var/${N}_kern.o $OTHERS
echo lib/var_$N.so
