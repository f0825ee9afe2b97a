set -e
export TMPDIR=/tmp
O=gpurun_out/pmc2
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/list.txt 2>&1 || true
CMD="python3 bench.py --workload c3 --steps 3 --warmup 1 --ramp-s 0 --no-cpu-baseline"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- $CMD > $O/a.log 2>&1
echo done
