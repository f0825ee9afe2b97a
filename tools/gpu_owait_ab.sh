# A/B of the dQ kernel's wait before the fused-D O loads (FA_GDQ_OWAIT variants), knob 8 on
mkdir -p gpurun_out
set -o pipefail
export FLASH_ATTN_MI355X_FUSE_PRE=1
timeout -k 10 300 python -u tools/ab.py variants/libfa_base.so variants/libfa_ow63.so variants/libfa_ow39.so --bwd > gpurun_out/ab_owait_c3.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py variants/libfa_base.so variants/libfa_ow63.so variants/libfa_ow39.so --bwd --workload c4 > gpurun_out/ab_owait_c4.txt 2>&1
