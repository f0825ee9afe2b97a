#!/usr/bin/env python3
"""Phase timeline of the dK/dV kernel from an FA_STAMPS build (dev tool):

    tools/variant_bwd.sh stamps -DFA_STAMPS
    python tools/stamps.py variants/libfa_stamps.so

Runs the C3 backward a few times through the variant library, reads the s_memtime stamps of
workgroups 0-3 (8 waves, 64 slices, 8 points each) and prints, per role, the mean cycles between
consecutive points: 0 loop top | 1 after DMA issue | 2 after dS step | 3 after phase 1 |
4 after P step | 5 after phase 2 | 6 after the barrier.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from ab import load  # noqa: E402

WG, IT, PTS = 4, 64, 8
NAMES = ["issue", "dS step", "init+phase1", "P step", "phase2", "barrier"]


def main():
    lib = load(sys.argv[1])
    lib.flash_attn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    m._lib = lib
    b, s, h, d = 4, 8192, 16, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v, dout = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4))
    res = m.fwd(q, k, v, None, 0.0, d ** -0.5, True, False, None)
    for _ in range(3):
        m.bwd(dout, q, k, v, res[0], res[5], None, None, None, 0.0, d ** -0.5, True, None, res[7])
    torch.cuda.synchronize()
    buf = np.zeros(WG * 8 * IT * PTS, dtype=np.uint64)
    rc = lib.flash_attn_debug_stamps(buf.ctypes.data, buf.nbytes)
    assert rc == 0, rc
    st = buf.reshape(WG, 8, IT, PTS).astype(np.int64)
    for role, waves in (("P waves", range(4)), ("dS waves", range(4, 8))):
        d = np.diff(st[:, list(waves), 2:IT - 2, :7], axis=-1)   # steady-state slices
        means = d.mean(axis=(0, 1, 2))
        print(f"{role}: " + " | ".join(f"{n} {x:.0f}" for n, x in zip(NAMES, means)) + f" | total {means.sum():.0f}")
    step = np.diff(st[:, :, 2:IT - 2, 6], axis=-1).mean()
    print(f"cycles per slice (barrier to barrier): {step:.0f}")
    # skew: when does each wave arrive at the barrier relative to the first arrival
    arr = st[:, :, 2:IT - 2, 5]
    print("mean barrier-arrival lag vs first wave, per wave:",
          np.round((arr - arr.min(axis=1, keepdims=True)).mean(axis=(0, 2))).astype(int).tolist())


if __name__ == "__main__":
    main()
