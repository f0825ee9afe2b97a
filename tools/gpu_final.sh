#!/bin/bash
# Round-end evidence on one GPU box (run from the repo root by gpurun): the GPU suite, smoke(), the
# C3 / C4 / C2 bench lines, the PMC passes of the C3 and C2 bench commands and its rocprofv3 kernel statistics.
# Each GPU step has its own time limit; a timeout, abort or crash ends the script there.
export TMPDIR=/tmp
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
stop() { case $1 in 124|137|134|139) echo "step $2 ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/gputests.txt" 2>&1
rc=$?; tail -3 "$OUT/gputests.txt"; stop $rc pytest
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
rc=$?; tail -1 "$OUT/smoke.txt"; stop $rc smoke
timeout -k 10 400 python3 bench.py > "$OUT/bench_c3.log" 2>&1; rc=$?; stop $rc bench_c3
timeout -k 10 400 python3 bench.py --workload c4 > "$OUT/bench_c4.log" 2>&1; rc=$?; stop $rc bench_c4
timeout -k 10 400 python3 bench.py --workload c2 > "$OUT/bench_c2.log" 2>&1; rc=$?; stop $rc bench_c2
bash profiles/pmc_run.sh "$OUT/pmc_c3" c3; rc=$?; stop $rc pmc
bash profiles/pmc_run.sh "$OUT/pmc_c2" c2; rc=$?; stop $rc pmc_c2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench_c3_prof.log" 2>&1
rc=$?; stop $rc rocprof
echo "all steps done"
