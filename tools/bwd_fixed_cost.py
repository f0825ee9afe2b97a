#!/usr/bin/env python3
"""Per-workgroup fixed cost of the dK/dV kernel (dev tool): exactly one workgroup per CU (2 x 16
heads x 8 key blocks of 128 = 256 workgroups, non-causal), so the dK/dV kernel time (live HIP-event
timer) is one workgroup's latency; a straight-line fit over seqlen_q gives
t = fixed + per_step * steps (a step = 64 query rows).

    python tools/bwd_fixed_cost.py [--hip]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import KernelTimer  # noqa: E402
from flash_attn import flash_attn_func  # noqa: E402
from knobs import knob  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    b, h, sk, d = 2, 16, 1024, 128
    timer = KernelTimer()
    for on in (1, 0):
        xs, ys = [], []
        with knob(3, on):
            for sq in (256, 512, 1024, 2048, 4096):
                g = torch.Generator(device="cuda").manual_seed(0)
                q = torch.randn(b, sq, h, d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
                k = torch.randn(b, sk, h, d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
                v = torch.randn(b, sk, h, d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
                do = torch.randn(b, sq, h, d, device="cuda", dtype=torch.bfloat16, generator=g)
                out = flash_attn_func(q, k, v)
                for _ in range(3):
                    torch.autograd.grad(out, (q, k, v), do, retain_graph=True)
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(3):
                    timer.start()
                    for _ in range(a.iters):
                        torch.autograd.grad(out, (q, k, v), do, retain_graph=True)
                    torch.cuda.synchronize()
                    best = min(best, timer.stop()["bwd_dkdv_kernel"]["avg_ms"])
                steps = sq // 64
                xs.append(steps)
                ys.append(best * 1e3)
                print(f"{'asm' if on else 'HIP'} sq {sq:5d} steps {steps:3d}  {best * 1e3:8.2f} us  ({best * 1e3 / steps:.3f} us/step)",
                      flush=True)
        sl, c0 = np.polyfit(xs, ys, 1)
        print(f"{'asm' if on else 'HIP'} fit: fixed {c0:.2f} us + {sl:.3f} us per 64-row step "
              f"(64 MFMAs per wave: ideal {2048 / 2.4e3:.3f} us at 2.4 GHz)", flush=True)


if __name__ == "__main__":
    main()
