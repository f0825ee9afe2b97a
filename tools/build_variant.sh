#!/bin/bash
# Build a variant of the library for A/B timing (dev tool):
#   tools/build_variant.sh NAME [GIT_REV] [EXTRA_HIPCC_FLAGS...]
# Copies csrc/ (from the working tree, or from GIT_REV when given and not "-") to a scratch dir and
# builds variants/libfa_NAME.so; extra flags (e.g. -DFA_FWD_PRIO=1) are appended to CXXFLAGS.
set -e
NAME=$1; REV=${2:--}; shift; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SCR=/tmp/fa_variant_$NAME
rm -rf "$SCR"; mkdir -p "$SCR/pkg/csrc" "$SCR/include" "$ROOT/variants"
if [ "$REV" = "-" ]; then
  cp "$ROOT"/xhy-flash-attention_amd/csrc/*.* "$ROOT"/xhy-flash-attention_amd/csrc/Makefile "$SCR/pkg/csrc/"
  cp -r "$ROOT"/xhy-flash-attention_amd/csrc/asm "$SCR/pkg/csrc/"
  cp "$ROOT"/include/* "$SCR/include/"
else
  (cd "$ROOT" && git archive "$REV" xhy-flash-attention_amd/csrc include) | tar -x -C "$SCR"
  mv "$SCR"/xhy-flash-attention_amd/csrc/* "$SCR/pkg/csrc/"
fi
make -s -C "$SCR/pkg/csrc" -j8 OUTDIR="$ROOT/variants" OBJDIR="$SCR/obj" \
  LIB="$ROOT/variants/libfa_$NAME.so" CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $*" \
  HDRS="" > /dev/null
echo "$ROOT/variants/libfa_$NAME.so"
