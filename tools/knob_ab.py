#!/usr/bin/env python3
"""A/B of a launcher switch (include/flash_attn.h flash_attn_set_knob) at one shape (dev tool):
interleaved rounds, per-kernel device times from the live HIP-event timers, min over rounds.

    python tools/knob_ab.py --knob 2 --values 256,0 [--b 4 --s 8192 --h 16 --d 128 --causal 1 --bwd]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import KernelTimer, c4_seqlens, flops_fwd, varlen_flops_fwd  # noqa: E402
from flash_attn import flash_attn_func, flash_attn_varlen_qkvpacked_func  # noqa: E402
from knobs import knob  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", type=int, required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--b", type=int, default=4)
    ap.add_argument("--s", type=int, default=8192)
    ap.add_argument("--h", type=int, default=16)
    ap.add_argument("--hk", type=int, default=0)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--causal", type=int, default=1)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--c4", action="store_true", help="the C4 varlen qkvpacked workload (--h / --d apply)")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    hk = a.hk or a.h
    values = [int(x) for x in a.values.split(",")]
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
    k = torch.randn(a.b, a.s, hk, a.d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
    v = torch.randn(a.b, a.s, hk, a.d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
    dout = torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=torch.bfloat16, generator=g)
    timer = KernelTimer()
    res = {x: {} for x in values}
    if a.c4:
        lens = c4_seqlens()
        cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")
        qkv = torch.randn(sum(lens), 3, a.h, a.d, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_()
        dout = torch.randn(sum(lens), a.h, a.d, device="cuda", dtype=torch.bfloat16, generator=g)

    def step():
        if a.c4:
            with torch.set_grad_enabled(a.bwd):
                out = flash_attn_varlen_qkvpacked_func(qkv, cu, max(lens), causal=bool(a.causal))
                if a.bwd:
                    torch.autograd.grad(out, (qkv,), dout)
            return
        if a.bwd:
            out = flash_attn_func(q, k, v, causal=bool(a.causal))
            torch.autograd.grad(out, (q, k, v), dout)
        else:
            with torch.no_grad():
                flash_attn_func(q, k, v, causal=bool(a.causal))

    for _ in range(a.rounds):
        for x in values:
            with knob(a.knob, x):
                for _ in range(2):
                    step()
                torch.cuda.synchronize()
                timer.start()
                for _ in range(a.iters):
                    step()
                torch.cuda.synchronize()
                for name, r in timer.stop().items():
                    res[x].setdefault(name, []).append(r["avg_ms"])
    f = varlen_flops_fwd(lens, a.h, a.d, bool(a.causal)) if a.c4 else flops_fwd(a.b, a.s, a.h, a.d, bool(a.causal))
    fac = {"fwd_kernel": 1.0, "bwd_dkdv_kernel": 2.0, "bwd_dq_kernel": 1.5}
    for x in values:
        parts = []
        for name, ts in sorted(res[x].items()):
            ms = min(ts)
            tf = f" {fac[name] * f / ms / 1e9:.0f} TF" if name in fac else ""
            parts.append(f"{name} {ms:.4f} ms{tf}")
        print(f"knob {a.knob} = {x}: " + " | ".join(parts), flush=True)


if __name__ == "__main__":
    main()
