# bench lines of every BASELINE workload (run on the GPU box from the repo root):  bash tools/gpu_workloads.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
for w in c3 c4 c5 c2; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err
  echo "$w done"
done
