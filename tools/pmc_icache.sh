#!/bin/bash
# Instruction-fetch counters of the forward (dev tool; run on the GPU box from the repo root):
#   tools/pmc_icache.sh OUTDIR [WORKLOAD...]
# Lists the counters this rocprofv3 offers, keeps the instruction-cache / fetch ones it finds, and
# runs one --kernel-trace --pmc pass per group of at most 4 over tools/ab.py's forward loop.
OUT=${1:-gpurun_out/icache}; shift
WLS=${*:-c4 c3}
mkdir -p "$OUT"
export TMPDIR=/tmp
LIB=xhy-flash-attention_amd/libflash_attn_mi355x.so
timeout -s KILL 90 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || { echo "counter list failed"; exit 1; }
have() { grep -q -w "$1" "$OUT/avail.txt"; }
G1=""; for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do have $c && G1="$G1 $c"; done
G2=""; for c in SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU; do have $c && G2="$G2 $c"; done
echo "groups: [$G1] [$G2]" | tee "$OUT/groups.txt"
for WL in $WLS; do
  i=0; mkdir -p "$OUT/$WL"
  for G in "$G1" "$G2"; do
    i=$((i+1)); [ -z "$G" ] && continue
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d "$OUT/$WL/g$i" -o run --output-format csv -- \
      python3 tools/ab.py "$LIB" --workload "$WL" --rounds 2 --iters 5 > "$OUT/$WL/g$i.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "pass $WL g$i ended with $rc"; exit $rc; }
  done
done
echo "icache passes done: $OUT"
