#!/usr/bin/env python3
"""GPU check of the assembly dK / dV kernel against the HIP one (dev tool): the same backward with
knob 3 (FLASH_ATTN_MI355X_BWD_ASM) on and off, over a set of shapes; dK / dV differences relative to
max |dK|, |dV|; then C3 kernel times of both.

    python tools/bwd_asm_check.py [--time]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import KernelTimer  # noqa: E402
from flash_attn import flash_attn_func, flash_attn_varlen_func  # noqa: E402
from knobs import knob  # noqa: E402

BWD_ASM, DQ_ASM = 3, 4


class both:
    """both assembly backward kernels on (1) or off (0)"""

    def __init__(self, on):
        self.k = [knob(BWD_ASM, on), knob(DQ_ASM, on)]

    def __enter__(self):
        for k in self.k:
            k.__enter__()

    def __exit__(self, *a):
        for k in reversed(self.k):
            k.__exit__(*a)
SHAPES = [  # b, sq, sk, h, hk, causal, dtype
    (1, 64, 128, 1, 1, True, torch.bfloat16),
    (2, 300, 300, 2, 2, True, torch.bfloat16),
    (1, 200, 330, 4, 2, True, torch.float16),
    (1, 330, 200, 2, 1, True, torch.bfloat16),
    (2, 257, 129, 2, 2, False, torch.bfloat16),
    (1, 1024, 1024, 8, 8, True, torch.bfloat16),
    (2, 1000, 1500, 6, 2, False, torch.float16),
    (1, 4096, 4096, 4, 4, True, torch.bfloat16),
]


def grads(q, k, v, do, causal):
    out = flash_attn_func(q, k, v, causal=causal)
    return torch.autograd.grad(out, (q, k, v), do)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--c5", action="store_true", help="C5-derived GQA / fp16 shapes only")
    a = ap.parse_args()
    bad = 0
    shapes = SHAPES
    if a.c5:
        shapes = [(1, 4096, 4096, 8, 2, True, torch.float16), (2, 4096, 4096, 8, 2, True, torch.float16),
                  (1, 16384, 16384, 4, 1, True, torch.float16), (1, 8192, 8192, 4, 1, True, torch.bfloat16),
                  (1, 8192, 8192, 4, 4, True, torch.float16), (1, 32768, 32768, 4, 1, True, torch.float16)]
    for b, sq, sk, h, hk, causal, dt in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(b, sq, h, 128, device="cuda", dtype=dt, generator=g).requires_grad_()
        k = torch.randn(b, sk, hk, 128, device="cuda", dtype=dt, generator=g).requires_grad_()
        v = torch.randn(b, sk, hk, 128, device="cuda", dtype=dt, generator=g).requires_grad_()
        do = torch.randn(b, sq, h, 128, device="cuda", dtype=dt, generator=g)
        with both(0):
            ref = grads(q, k, v, do, causal)
        with both(1):
            got = grads(q, k, v, do, causal)
        torch.cuda.synchronize()
        msg = []
        for name, x, y in zip(("dq", "dk", "dv"), got, ref):
            fin = bool(torch.isfinite(x).all())
            e = ((x.float() - y.float()).abs().max() / y.float().abs().max().clamp_min(1e-6)).item()
            msg.append(f"{name} {e:.2e}{'' if fin else ' NONFINITE'}")
            if not fin or e > 2e-2:
                bad += 1
        print(f"b{b} sq{sq} sk{sk} h{h}/{hk} causal={causal} {str(dt)[6:]}: " + " ".join(msg), flush=True)
    if a.c5:
        print("mismatches:", bad, flush=True)
        return
    # varlen
    cu = torch.tensor([0, 100, 357, 900], device="cuda", dtype=torch.int32)
    for causal in (True, False):
        g = torch.Generator(device="cuda").manual_seed(1)
        q = torch.randn(900, 4, 128, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
        k = torch.randn(900, 2, 128, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
        v = torch.randn(900, 2, 128, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
        do = torch.randn(900, 4, 128, device="cuda", dtype=torch.bfloat16, generator=g)
        res = {}
        for on in (0, 1):
            with both(on):
                out = flash_attn_varlen_func(q, k, v, cu, cu, 543, 543, causal=causal)
                res[on] = torch.autograd.grad(out, (q, k, v), do)
        msg = []
        for name, x, y in zip(("dq", "dk", "dv"), res[1], res[0]):
            e = ((x.float() - y.float()).abs().max() / y.float().abs().max()).item()
            msg.append(f"{name} {e:.2e}")
            if not torch.isfinite(x).all() or e > 2e-2:
                bad += 1
        print(f"varlen causal={causal}: " + " ".join(msg), flush=True)
    print("mismatches:", bad, flush=True)
    if a.time:
        timer = KernelTimer()
        q = torch.randn(4, 8192, 16, 128, device="cuda", dtype=torch.bfloat16).requires_grad_()
        k = torch.randn(4, 8192, 16, 128, device="cuda", dtype=torch.bfloat16).requires_grad_()
        v = torch.randn(4, 8192, 16, 128, device="cuda", dtype=torch.bfloat16).requires_grad_()
        do = torch.randn(4, 8192, 16, 128, device="cuda", dtype=torch.bfloat16)
        out = flash_attn_func(q, k, v, causal=True)
        f = 4.0 * 4 * 8192 * 8192 * 16 * 128 / 2
        res = {0: [], 1: []}
        for _ in range(4):
            for on in (1, 0):
                with both(on):
                    for _ in range(2):
                        torch.autograd.grad(out, (q, k, v), do, retain_graph=True)
                    torch.cuda.synchronize()
                    timer.start()
                    for _ in range(10):
                        torch.autograd.grad(out, (q, k, v), do, retain_graph=True)
                    torch.cuda.synchronize()
                    t = timer.stop()
                    res[on].append((t["bwd_dkdv_kernel"]["avg_ms"], t["bwd_dq_kernel"]["avg_ms"]))
        for on in (1, 0):
            ms = min(x[0] for x in res[on])
            mq = min(x[1] for x in res[on])
            print(f"C3 {'asm' if on else 'HIP'}: dK/dV {ms:.4f} ms ({2 * f / ms / 1e9:.0f} TF), "
                  f"dQ {mq:.4f} ms ({1.5 * f / mq / 1e9:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
