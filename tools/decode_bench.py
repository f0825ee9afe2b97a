#!/usr/bin/env python3
"""Decode-shaped forward timing, split-KV on and off (dev tool, GPU box).

    python tools/decode_bench.py

One query row per sequence against a long K/V cache (non-causal, bf16, d = 128); reports the
kernel time and the K/V streaming rate (2 * b * sk * hk * d * 2 bytes per call) against the
~8 TB/s HBM roofline.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
from flash_attn.flash_attn_interface import _flash_attn_forward  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
from knobs import no_splitkv  # noqa: E402


def time_fwd(q, k, v, iters=20):
    _flash_attn_forward(q, k, v, 0.0, q.shape[-1] ** -0.5, False, False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        _flash_attn_forward(q, k, v, 0.0, q.shape[-1] ** -0.5, False, False)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    for b, sq, sk, h, hk in ((8, 1, 8192, 32, 8), (4, 1, 32768, 32, 8), (1, 1, 131072, 32, 8),
                             (8, 16, 8192, 32, 8)):
        d = 128
        q = torch.randn(b, sq, h, d, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(b, sk, hk, d, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(b, sk, hk, d, device="cuda", dtype=torch.bfloat16)
        gb = 2 * b * sk * hk * d * 2 / 1e9
        with no_splitkv():
            t0 = time_fwd(q, k, v)
        t1 = time_fwd(q, k, v)
        print(f"b={b} sq={sq} sk={sk} h={h} hk={hk}: unsplit {t0:.3f} ms ({gb / t0 * 1e3:.0f} GB/s), "
              f"split {t1:.3f} ms ({gb / t1 * 1e3:.0f} GB/s), speedup {t0 / t1:.2f}x")


if __name__ == "__main__":
    main()
