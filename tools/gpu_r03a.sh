set -e
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1
echo prof done
bash profiles/pmc_run.sh $O/pmc_c3 c3
bash profiles/pmc_run.sh $O/pmc_c2 c2
