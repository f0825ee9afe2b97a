#!/bin/bash
# PMC passes for the dominant kernels (run on the GPU box from the repo root).
# One counter group per rocprofv3 pass; kernel-trace only, no sys/runtime tracing.
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/l2" -o run --output-format csv -- $ARGS > "$OUT/l2.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES -d "$OUT/sq" -o run --output-format csv -- $ARGS > "$OUT/sq.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/lds" -o run --output-format csv -- $ARGS > "$OUT/lds.log" 2>&1
echo done
