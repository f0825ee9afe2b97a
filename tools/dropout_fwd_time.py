#!/usr/bin/env python3
"""Forward kernel time with dropout at head dims 64 and 128 (dev tool):
    python tools/dropout_fwd_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import KernelTimer, flops_fwd  # noqa: E402
from flash_attn import flash_attn_func  # noqa: E402


def main():
    timer = KernelTimer()
    for b, s, h, d, causal in ((4, 4096, 32, 64, True), (4, 4096, 32, 64, False), (4, 8192, 16, 128, True)):
        q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        with torch.no_grad():
            for _ in range(3):
                flash_attn_func(q, k, v, dropout_p=0.1, causal=causal)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(4):
                timer.start()
                for _ in range(10):
                    flash_attn_func(q, k, v, dropout_p=0.1, causal=causal)
                torch.cuda.synchronize()
                best = min(best, timer.stop()["fwd_kernel"]["avg_ms"])
        f = flops_fwd(b, s, h, d, causal)
        print(f"dropout fwd b{b} s{s} h{h} d{d} causal={causal}: {best:.4f} ms ({f / best / 1e9:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
