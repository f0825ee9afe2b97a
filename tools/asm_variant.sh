#!/bin/bash
# Build a library variant whose assembly forward is generated with dev switches (A/B):
#   FA_GEN_X=1 ... tools/asm_variant.sh NAME  ->  variants/libfa_NAME.so
# Every other object comes from the in-tree build (csrc/build).
set -e
NAME=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/xhy-flash-attention_amd/csrc
W=/tmp/fa_asmv/$NAME
rm -rf "$W"; mkdir -p "$W" "$ROOT/variants"
make -s -C "$CS" >/dev/null
python3 "$CS/asm/gen_fwd.py" > "$W/fa_fwd_asm.s"
/opt/rocm/lib/llvm/bin/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c "$W/fa_fwd_asm.s" -o "$W/fa_fwd_asm.o"
/opt/rocm/lib/llvm/bin/ld.lld -shared "$W/fa_fwd_asm.o" -o "$W/fa_fwd_asm.co"
python3 "$CS/asm/embed.py" "$W/fa_fwd_asm.co" fa_fwd_asm_co > "$W/blob.cpp"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -x hip -c "$W/blob.cpp" -o "$W/blob.o"
OBJS=""
for o in $CS/build/*.o; do
  b=$(basename $o .o)
  case $b in fa_fwd_asm|fa_fwd_asm_blob.cpp) continue;; esac
  OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libfa_$NAME.so" $OBJS "$W/blob.o"
echo "$ROOT/variants/libfa_$NAME.so"
