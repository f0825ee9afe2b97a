import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "xhy-flash-attention_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
# the CPU emulator's kernels start from NaN registers and 0xff LDS bytes (tools/asm_emu.py): a read
# of state the kernel never wrote shows up as NaN, as it would on the GPU
os.environ.setdefault("FA_EMU_POISON", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
