#!/usr/bin/env python3
"""Forward / backward kernel times over a set of shapes (dev tool; live HIP-event kernel timers).

    python tools/fwd_shapes.py [--bwd] [--iters 20]
Shapes: C3 causal / non-causal, the guide's reference shape (B16 H64 HKV8 N2048 D128), C2, C5 slice.
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

SHAPES = [
    # b, s, h, hk, d, causal, dtype
    (4, 8192, 16, 16, 128, True, torch.bfloat16),
    (4, 8192, 16, 16, 128, False, torch.bfloat16),
    (16, 2048, 64, 8, 128, False, torch.bfloat16),
    (16, 2048, 64, 8, 128, True, torch.bfloat16),
    (4, 2048, 16, 16, 64, True, torch.bfloat16),
    (2, 32768, 32, 8, 128, True, torch.float16),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    timer = KernelTimer()
    for b, s, h, hk, d, causal, dt in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(b, s, h, d, device="cuda", dtype=dt, generator=g).requires_grad_()
        k = torch.randn(b, s, hk, d, device="cuda", dtype=dt, generator=g).requires_grad_()
        v = torch.randn(b, s, hk, d, device="cuda", dtype=dt, generator=g).requires_grad_()
        dout = torch.randn(b, s, h, d, device="cuda", dtype=dt, generator=g)

        def step():
            if args.bwd:
                out = flash_attn_func(q, k, v, causal=causal)
                torch.autograd.grad(out, (q, k, v), dout)
            else:
                with torch.no_grad():
                    flash_attn_func(q, k, v, causal=causal)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        timer.start()
        for _ in range(args.iters):
            step()
        torch.cuda.synchronize()
        kt = timer.stop()
        f = flops_fwd(b, s, h, d, causal)
        parts = []
        for name, fac in (("fwd_kernel", 1.0), ("bwd_dkdv_kernel", 2.0), ("bwd_dq_kernel", 1.5)):
            if name in kt:
                ms = kt[name]["avg_ms"]
                parts.append(f"{name} {ms:.4f} ms {fac * f / ms / 1e9:.0f} TF")
        print(f"b{b} s{s} h{h}/{hk} d{d} causal={causal} {str(dt)[6:]}: " + " | ".join(parts), flush=True)
        del q, k, v, dout


if __name__ == "__main__":
    main()
