#!/usr/bin/env python3
"""Forward / backward kernel times per head dim (dev tool): shows what the dedicated d = 160 / 224
instantiations recover against the next power-of-two tile (192 / 256): with them the time scales
with d instead of with the padded tile width.

    python tools/hdim_bench.py [--b 2 --s 4096 --h 16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import KernelTimer, flops_fwd  # noqa: E402
from flash_attn import flash_attn_func  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=2)
    ap.add_argument("--s", type=int, default=4096)
    ap.add_argument("--h", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    timer = KernelTimer()
    for d in (128, 160, 192, 224, 256):
        g = torch.Generator(device="cuda").manual_seed(0)
        q, k, v = (torch.randn(a.b, a.s, a.h, d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
                   for _ in range(3))
        do = torch.randn(a.b, a.s, a.h, d, device="cuda", dtype=torch.bfloat16, generator=g)
        for _ in range(3):
            out = flash_attn_func(q, k, v, causal=True)
            torch.autograd.grad(out, (q, k, v), do)
        torch.cuda.synchronize()
        timer.start()
        for _ in range(a.iters):
            out = flash_attn_func(q, k, v, causal=True)
            torch.autograd.grad(out, (q, k, v), do)
        torch.cuda.synchronize()
        kt = timer.stop()
        f = flops_fwd(a.b, a.s, a.h, d, True)
        fw = kt["fwd_kernel"]["avg_ms"]
        bw = sum(kt[n]["avg_ms"] for n in kt if n.startswith("bwd") and n != "bwd_dkdv_dq_window")
        print(f"d {d:3d}: fwd {fw:.3f} ms ({f / fw / 1e9:.0f} TF)  bwd kernels {bw:.3f} ms "
              f"({2.5 * f / bw / 1e9:.0f} TF, reference convention)", flush=True)


if __name__ == "__main__":
    main()
