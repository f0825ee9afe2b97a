#!/bin/bash
# Build a library variant whose assembly kernels (forward and dK/dV) are generated with dev switches
# (A/B):   FA_GEN_X=1 FA_GBW_Y=2 ... tools/asm_variant.sh NAME  ->  variants/libfa_NAME.so
# Every other object comes from the in-tree build (csrc/build), except the CXX_FILES (e.g.
# "fa_fwd.hip"), recompiled with CXX_FLAGS (e.g. -DFA_NO_QFOLD) when given.
set -e
NAME=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/xhy-flash-attention_amd/csrc
W=/tmp/fa_asmv/$NAME
rm -rf "$W"; mkdir -p "$W" "$ROOT/variants"
# (the in-tree build must not see the dev switches)
env $(env | grep -o '^FA_G[A-Z_]*' | sed 's/^/-u /') make -s -C "$CS" >/dev/null
for k in fwd bwd dq bwd2 bwd64 dq64 fwdnf; do
  python3 "$CS/asm/gen_$k.py" > "$W/fa_${k}_asm.s"
  /opt/rocm/lib/llvm/bin/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c "$W/fa_${k}_asm.s" -o "$W/fa_${k}_asm.o"
  /opt/rocm/lib/llvm/bin/ld.lld -shared "$W/fa_${k}_asm.o" -o "$W/fa_${k}_asm.co"
  python3 "$CS/asm/embed.py" "$W/fa_${k}_asm.co" fa_${k}_asm_co > "$W/blob_$k.cpp"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -x hip -c "$W/blob_$k.cpp" -o "$W/blob_$k.o"
done
OBJS=""
for f in $CXX_FILES; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize $CXX_FLAGS -x hip -c "$CS/$f" -o "$W/$f.o"
  OBJS="$OBJS $W/$f.o"
done
for o in $CS/build/*.o; do
  b=$(basename $o .o)
  case $b in fa_fwd_asm|fa_fwd_asm_blob.cpp|fa_bwd_asm|fa_bwd_asm_blob.cpp|fa_dq_asm|fa_dq_asm_blob.cpp|fa_bwd2_asm|fa_bwd2_asm_blob.cpp|fa_bwd64_asm|fa_bwd64_asm_blob.cpp|fa_dq64_asm|fa_dq64_asm_blob.cpp|fa_fwdnf_asm|fa_fwdnf_asm_blob.cpp) continue;; esac
  case " $CXX_FILES " in *" $b "*) continue;; esac
  OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libfa_$NAME.so" $OBJS "$W/blob_fwd.o" "$W/blob_bwd.o" "$W/blob_dq.o" "$W/blob_bwd2.o" "$W/blob_bwd64.o" "$W/blob_dq64.o" "$W/blob_fwdnf.o"
echo "$ROOT/variants/libfa_$NAME.so"
