#!/usr/bin/env python3
"""GPU check of the assembly forward against fwd_kernel (HIP) and an fp64 reference, plus a C3
forward timing of both paths (dev tool).

    python tools/asm_check.py [--time] [--shapes all|small]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from flash_attn import flash_attn_func, flash_attn_varlen_func  # noqa: E402


def use_asm(on):
    m._lib.flash_attn_fwd_use_asm(int(on))


def ref64(q, k, v, causal):
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    g = h // hk
    qd, kd, vd = (x.double().transpose(1, 2) for x in (q, k, v))
    kd = kd.repeat_interleave(g, 1)
    vd = vd.repeat_interleave(g, 1)
    s = qd @ kd.transpose(-1, -2) * d ** -0.5
    if causal:
        mask = torch.ones(sq, sk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ vd
    return o.transpose(1, 2), lse


def check(b, sq, sk, h, hk, causal, dtype, seed=0, big=None):
    torch.manual_seed(seed)
    dev = "cuda"
    q = torch.randn(b, sq, h, 128, device=dev, dtype=dtype)
    k = torch.randn(b, sk, hk, 128, device=dev, dtype=dtype)
    v = torch.randn(b, sk, hk, 128, device=dev, dtype=dtype)
    if big is not None:
        q *= 0.3
        k[:, big:big + 3] *= 12
    use_asm(1)
    o1, lse1, _ = flash_attn_func(q, k, v, causal=causal, return_attn_probs=True)
    use_asm(0)
    o0, lse0, _ = flash_attn_func(q, k, v, causal=causal, return_attn_probs=True)
    use_asm(1)
    torch.cuda.synchronize()
    line = (f"b={b} sq={sq} sk={sk} h={h} hk={hk} causal={causal} {str(dtype)[6:]}: "
            f"asm-hip |dO| {(o1.float() - o0.float()).abs().max().item():.3e} |dLSE| {(lse1 - lse0).abs().max().item():.3e}")
    if b * sq * sk * h <= 4 * 2048 * 2048 * 4:
        orf, lrf = ref64(q, k, v, causal)
        e1 = (o1.double() - orf).abs().max().item()
        e0 = (o0.double() - orf).abs().max().item()
        l1 = (lse1.double() - lrf).abs().max().item()
        line += f" | vs fp64: asm {e1:.3e} hip {e0:.3e}  lse asm {l1:.2e}"
    print(line, flush=True)
    bad = not torch.isfinite(o1).all().item()
    return bad


def check_varlen(lens, h, causal, dtype):
    torch.manual_seed(1)
    tot = sum(lens)
    qkv = torch.randn(tot, 3, h, 128, device="cuda", dtype=dtype)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    mx = max(lens)
    q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
    use_asm(1)
    o1 = flash_attn_varlen_func(q, k, v, cu, cu, mx, mx, causal=causal)
    use_asm(0)
    o0 = flash_attn_varlen_func(q, k, v, cu, cu, mx, mx, causal=causal)
    use_asm(1)
    torch.cuda.synchronize()
    print(f"varlen {lens} causal={causal}: asm-hip |dO| {(o1.float() - o0.float()).abs().max().item():.3e}", flush=True)


def time_fwd(b, s, h, d, causal, dtype, iters=30):
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=dtype) for _ in range(3))
    flops = 4 * b * s * s * h * d / (2 if causal else 1)
    res = {}
    for on in (1, 0, 1, 0):
        use_asm(on)
        for _ in range(5):
            flash_attn_func(q, k, v, causal=causal)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            flash_attn_func(q, k, v, causal=causal)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        res.setdefault(on, []).append(ms)
    use_asm(1)
    for on in (1, 0):
        ms = min(res[on])
        print(f"fwd b={b} s={s} h={h} d={d} causal={causal} {'asm' if on else 'hip'}: {ms:.4f} ms "
              f"{flops / ms / 1e9:.1f} TF ({flops / ms / 1e9 / 2516.6 * 100:.1f}% of peak)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--shapes", default="all")
    a = ap.parse_args()
    t0 = time.time()
    bad = False
    cases = [(1, 64, 64, 1, 1, True), (1, 600, 600, 2, 1, True), (2, 300, 700, 4, 2, True),
             (1, 700, 260, 2, 2, True), (2, 130, 77, 2, 1, False), (1, 1000, 1000, 4, 4, False),
             (2, 2048, 2048, 4, 4, True)]
    for c in cases:
        for dt in (torch.bfloat16, torch.float16):
            bad |= check(*c, dt)
    bad |= check(1, 520, 520, 2, 2, True, torch.bfloat16, big=400)
    bad |= check(1, 1030, 1030, 2, 1, False, torch.float16, big=700)
    check_varlen([100, 513, 64, 1000, 257], 4, True, torch.bfloat16)
    check_varlen([100, 513, 64, 1000, 257], 4, False, torch.float16)
    if a.shapes == "all":
        bad |= check(4, 8192, 8192, 16, 16, True, torch.bfloat16)
    print(f"checks done in {time.time() - t0:.1f}s, nonfinite={bad}", flush=True)
    if a.time:
        time_fwd(4, 8192, 16, 128, True, torch.bfloat16)
        time_fwd(4, 8192, 16, 128, False, torch.bfloat16, iters=15)
        time_fwd(8, 32768 // 4, 32, 128, True, torch.float16, iters=10)
