#!/bin/bash
# HBM / L2 traffic counters per kernel for each variant library (dev tool; run on the GPU box):
#   tools/pmc_mem.sh OUTDIR "AB_ARGS" LIB...
OUT=$1; ARGS=$2; shift 2
export TMPDIR=/tmp
for LIB in "$@"; do
  N=$(basename "$LIB" .so); mkdir -p "$OUT/$N"
  i=0
  for G in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $G -d "$OUT/$N/m$i" -o run --output-format csv -- \
      python3 tools/ab.py "$LIB" $ARGS > "$OUT/$N/m$i.log" 2>&1 || { echo "rocprof failed for $N m$i"; tail -5 "$OUT/$N/m$i.log"; }
  done
done
python3 tools/pmc_summary.py "$OUT"
