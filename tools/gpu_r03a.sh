# round-3 profiling pass (run on the GPU box from the repo root): bench line, kernel-trace stats of
# the same command, PMC passes for c3 (and c2 when asked)
#   bash tools/gpu_r03a.sh TAG [c2]
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1
echo prof done
bash profiles/pmc_run.sh $O/pmc_c3 c3
if [ "$2" = "c2" ]; then bash profiles/pmc_run.sh $O/pmc_c2 c2; fi
