#!/usr/bin/env python3
"""Per-32-row error map of the assembly forward on small shapes (dev tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from flash_attn import flash_attn_func  # noqa: E402
from asm_check import ref64  # noqa: E402


def case(sq, sk, causal, h=1, dtype=torch.bfloat16):
    torch.manual_seed(0)
    q = torch.randn(1, sq, h, 128, device="cuda", dtype=dtype)
    k = torch.randn(1, sk, h, 128, device="cuda", dtype=dtype)
    v = torch.randn(1, sk, h, 128, device="cuda", dtype=dtype)
    m._lib.flash_attn_fwd_use_asm(1)
    o, lse, _ = flash_attn_func(q, k, v, causal=causal, return_attn_probs=True)
    orf, lrf = ref64(q, k, v, causal)
    eo = (o.double() - orf).abs()[0, :, 0, :]
    el = (lse.double() - lrf).abs()[0, 0]
    print(f"sq={sq} sk={sk} causal={causal}", flush=True)
    for r0 in range(0, sq, 32):
        print(f"   rows {r0:4d}: O {eo[r0:r0 + 32].max().item():.2e}  LSE {el[r0:r0 + 32].max().item():.2e}"
              f"  lse[r0]={lse[0, 0, r0].item():.4f} ref={lrf[0, 0, r0].item():.4f}", flush=True)


if __name__ == "__main__":
    for sq, sk, causal in ((64, 64, False), (64, 64, True), (128, 128, False), (192, 192, False),
                           (256, 256, True), (64, 77, False), (300, 300, True)):
        case(sq, sk, causal)
