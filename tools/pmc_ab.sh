#!/bin/bash
# PMC counters per kernel for each variant library (dev tool; run on the GPU box from the repo root):
#   tools/pmc_ab.sh OUTDIR "AB_ARGS" LIB...
# One rocprofv3 pass per counter group and library (kernel-trace only, no sys/runtime tracing).
# PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" replaces the two SQ groups (';' between passes).
OUT=$1; ARGS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS"
G2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
for LIB in "$@"; do
  N=$(basename "$LIB" .so)
  i=0; mkdir -p "$OUT/$N"
  IFS=';' read -ra GS <<< "${PMC_GROUPS:-$G1;$G2}"
  for G in "${GS[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $G -d "$OUT/$N/g$i" -o run --output-format csv -- \
      python3 tools/ab.py "$LIB" $ARGS > "$OUT/$N/g$i.log" 2>&1 || { echo "rocprof failed for $N g$i"; exit 1; }
  done
done
python3 tools/pmc_summary.py "$OUT"
