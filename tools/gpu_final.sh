#!/bin/bash
# Round-end evidence on one GPU box (run from the repo root by gpurun), in two calls that each fit
# gpurun's 20-minute limit:
#   tools/gpu_final.sh TAG a   the GPU suite, smoke(), the bench lines (C3, C4, C2, C5, d64, C3 dropout)
#   tools/gpu_final.sh TAG b   the PMC passes of the C3 / C2 / C4 bench commands (profiles/pmc_run.sh)
#                              and the rocprofv3 kernel statistics of the C3 bench
#   tools/gpu_final.sh TAG pmc2  the PMC passes of the d64 and C5 bench commands
# Each GPU step has its own time limit; a timeout, abort or crash ends the script there.
export TMPDIR=/tmp
TAG=${1:-final}
PART=${2:-a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
stop() { case $1 in 124|137|134|139) echo "step $2 ended with $1: stopping"; exit $1;; esac; }
if [ "$PART" = a ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/gputests.txt" 2>&1
  rc=$?; tail -3 "$OUT/gputests.txt"; stop $rc pytest
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
  rc=$?; tail -1 "$OUT/smoke.txt"; stop $rc smoke
  timeout -k 10 300 python3 bench.py > "$OUT/bench_c3.log" 2>&1; rc=$?; stop $rc bench_c3
  for w in c4 c2 c5 d64; do
    timeout -k 10 300 python3 bench.py --workload $w > "$OUT/bench_$w.log" 2>&1; rc=$?; stop $rc bench_$w
  done
  timeout -k 10 300 python3 bench.py --dropout 0.1 > "$OUT/bench_c3_drop.log" 2>&1; rc=$?; stop $rc bench_drop
elif [ "$PART" = pmc2 ]; then
  bash profiles/pmc_run.sh "$OUT/pmc_d64" d64; rc=$?; stop $rc pmc_d64
  bash profiles/pmc_run.sh "$OUT/pmc_c5" c5; rc=$?; stop $rc pmc_c5
else
  bash profiles/pmc_run.sh "$OUT/pmc_c3" c3; rc=$?; stop $rc pmc_c3
  bash profiles/pmc_run.sh "$OUT/pmc_c2" c2; rc=$?; stop $rc pmc_c2
  bash profiles/pmc_run.sh "$OUT/pmc_c4" c4; rc=$?; stop $rc pmc_c4
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench_c3_prof.log" 2>&1
  rc=$?; stop $rc rocprof
fi
echo "part $PART done"
