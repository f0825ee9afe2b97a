#!/bin/bash
# Build a variant of the library with some sources recompiled (dev tool, A/B and ablations):
#   [FILES="fa_fwd.hip fa_bwd.hip"] tools/variant_bwd.sh NAME [EXTRA_HIPCC_FLAGS...]  ->  variants/libfa_NAME.so
# FILES defaults to fa_bwd.hip; the other objects come from the in-tree build (csrc/build).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/xhy-flash-attention_amd/csrc
FILES=${FILES:-fa_bwd.hip}
mkdir -p "$ROOT/variants" /tmp/fa_vb/$NAME
OBJS=""
for f in $FILES; do
  EXTRA=""
  case $f in fa_fwd.hip|fa_bwd.hip) EXTRA="-fno-slp-vectorize";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $EXTRA "$@" -x hip -c "$CS/$f" \
    -o /tmp/fa_vb/$NAME/$f.o &
  OBJS="$OBJS /tmp/fa_vb/$NAME/$f.o"
done
wait
for o in $CS/build/*.o; do
  b=$(basename $o .o)
  case " $FILES " in *" $b "*) ;; *) OBJS="$OBJS $o";; esac
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libfa_$NAME.so" $OBJS
echo "$ROOT/variants/libfa_$NAME.so"
