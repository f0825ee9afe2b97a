#!/bin/bash
# Build a variant of the library with some sources recompiled (dev tool, A/B and ablations):
#   [FILES="fa_fwd.hip fa_bwd.hip"] tools/variant_bwd.sh NAME [EXTRA_HIPCC_FLAGS...]  ->  variants/libfa_NAME.so
# FILES defaults to fa_bwd.hip; the other objects come from the in-tree build (csrc/build).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/xhy-flash-attention_amd/csrc
FILES=${FILES:-fa_bwd.hip}
rm -rf /tmp/fa_vb/$NAME   # no stale object of an earlier run is ever linked
mkdir -p "$ROOT/variants" /tmp/fa_vb/$NAME
make -s -C "$CS" >/dev/null   # the in-tree objects the variant reuses are current
OBJS=""
PIDS=""
for f in $FILES; do
  # the per-file flags of the Makefile (FLAGS_<file>)
  EXTRA=$(make -s -C "$CS" --no-print-directory -f Makefile -f - print-flags <<<"print-flags: ; @echo \$(FLAGS_$f)")
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $EXTRA "$@" -x hip -c "$CS/$f" \
    -o /tmp/fa_vb/$NAME/$f.o &
  PIDS="$PIDS $!"
  OBJS="$OBJS /tmp/fa_vb/$NAME/$f.o"
done
for p in $PIDS; do wait $p || { echo "variant_bwd.sh: compile failed" >&2; exit 1; }; done
for o in $CS/build/*.o; do
  b=$(basename $o .o)
  [ "$b" = fa_fwd_asm ] && continue   # the gfx950 assembly object (embedded via fa_fwd_asm_blob)
  case " $FILES " in *" $b "*) ;; *) OBJS="$OBJS $o";; esac
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libfa_$NAME.so" $OBJS
echo "$ROOT/variants/libfa_$NAME.so"
