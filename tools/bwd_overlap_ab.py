#!/usr/bin/env python3
"""A/B of the backward's dQ / dK-dV stream overlap modes (fa_bwd.hip run_bwd) at C3 (dev tool): interleaved rounds, backward
time per step from CUDA events, gradients compared between the two modes (must be bitwise equal)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from flash_attn import flash_attn_func  # noqa: E402


def main(b=4, s=8192, h=16, d=128, rounds=4, iters=10):
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    out = flash_attn_func(q, k, v, causal=True)
    g = torch.randn_like(out)
    modes = (0, 1, 2, 3)
    res = {mode: [] for mode in modes}
    grads = {}
    for r in range(rounds):
        for on in modes:
            m._lib.flash_attn_bwd_overlap(on)
            for _ in range(3):
                torch.autograd.grad(out, (q, k, v), g, retain_graph=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                gr = torch.autograd.grad(out, (q, k, v), g, retain_graph=True)
            e1.record()
            torch.cuda.synchronize()
            res[on].append(e0.elapsed_time(e1) / iters)
            grads[on] = gr
    m._lib.flash_attn_bwd_overlap(0)
    same = all(torch.equal(a, c) for mode in modes for a, c in zip(grads[0], grads[mode]))
    f_bwd = 2.5 * 4 * b * s * s * h * d / 2
    for on in modes:
        ms = min(res[on])
        print(f"bwd overlap={on}: min {ms:.4f} ms  median {sorted(res[on])[len(res[on]) // 2]:.4f} ms "
              f"({f_bwd / ms / 1e9:.0f} TF)", flush=True)
    print("gradients bitwise equal:", same, flush=True)


if __name__ == "__main__":
    main()
