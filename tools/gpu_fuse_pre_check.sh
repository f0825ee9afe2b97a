# GPU validation of knob 8 (fused bwd_pre): its tests, the backward suites with the knob on, A/B at C3 / C4
mkdir -p gpurun_out
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fuse_pre_gpu.py > gpurun_out/fuse_tests.txt 2>&1 &&
FLASH_ATTN_MI355X_FUSE_PRE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_attn_gpu.py tests/test_configs_gpu.py tests/test_launch_gpu.py > gpurun_out/fuse_suite.txt 2>&1 &&
timeout -k 10 200 python -u tools/knob_ab.py --knob 8 --values 0,1 --bwd > gpurun_out/fuse_ab_c3.txt 2>&1 &&
timeout -k 10 200 python -u tools/knob_ab.py --knob 8 --values 0,1 --bwd --c4 > gpurun_out/fuse_ab_c4.txt 2>&1
