#!/bin/bash
# rocprofv3 PMC passes over the bench command of one workload (run on the GPU box from the repo
# root): one counter group per pass, --kernel-trace only (no sys/runtime tracing), each pass under
# its own time limit.  Then: python3 profiles/pmc.py OUT WORKLOAD  ->  profiles/pmc.json
#   profiles/pmc_run.sh gpurun_out/pmc_c3 c3
set -e
OUT=${1:-gpurun_out/pmc}
WL=${2:-c3}
mkdir -p "$OUT"
export TMPDIR=/tmp
# the build these counters describe (bench.py reports them only for a library with this hash)
python3 -c "import hashlib,sys; print(hashlib.sha256(open(sys.argv[1],'rb').read()).hexdigest()[:16])" \
  xhy-flash-attention_amd/libflash_attn_mi355x.so > "$OUT/lib_sha.txt"
CMD="python3 bench.py --workload $WL --steps 3 --warmup 1 --ramp-s 0 --no-cpu-baseline"
pass() {   # name counters...
  local name=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- $CMD \
    > "$OUT/$name.log" 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
echo "pmc passes done: $OUT"
