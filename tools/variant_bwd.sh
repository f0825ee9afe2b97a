#!/bin/bash
# Build a variant of the library with only fa_bwd.hip recompiled (dev tool, A/B and ablations):
#   tools/variant_bwd.sh NAME [EXTRA_HIPCC_FLAGS...]  ->  variants/libfa_NAME.so
# Links the variant's fa_bwd object with the other objects of the in-tree build (csrc/build).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/xhy-flash-attention_amd/csrc
mkdir -p "$ROOT/variants" /tmp/fa_vb
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -x hip -c "$CS/fa_bwd.hip" \
  -o /tmp/fa_vb/fa_bwd_$NAME.o
OBJS=$(ls $CS/build/*.o | grep -v fa_bwd)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libfa_$NAME.so" /tmp/fa_vb/fa_bwd_$NAME.o $OBJS
echo "$ROOT/variants/libfa_$NAME.so"
