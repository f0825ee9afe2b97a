#!/usr/bin/env python3
"""Per-workgroup fixed cost of the forward (dev tool): exactly one workgroup per CU (2 x 16 heads x
8 query blocks of 256 rows = 256 workgroups, non-causal; the 8 blocks of a head share one XCD and
its K/V stream), so the kernel time (live HIP-event timer) is one workgroup's latency; a straight-
line fit over seqlen_k gives  t = fixed + per_tile * tiles.

    python tools/fwd_fixed_cost.py [--d 128]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import KernelTimer  # noqa: E402
from flash_attn import flash_attn_func  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    b, h, sq, d = 2, 16, 2048, args.d
    timer = KernelTimer()
    xs, ys = [], []
    for sk in (256, 512, 1024, 2048, 4096):
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(b, sq, h, d, device="cuda", dtype=torch.bfloat16, generator=g)
        k = torch.randn(b, sk, h, d, device="cuda", dtype=torch.bfloat16, generator=g)
        v = torch.randn(b, sk, h, d, device="cuda", dtype=torch.bfloat16, generator=g)
        for _ in range(5):
            flash_attn_func(q, k, v)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            timer.start()
            for _ in range(args.iters):
                flash_attn_func(q, k, v)
            torch.cuda.synchronize()
            best = min(best, timer.stop()["fwd_kernel"]["avg_ms"])
        tiles = sk // 64
        xs.append(tiles)
        ys.append(best * 1e3)
        print(f"sk {sk:5d}  tiles {tiles:3d}  {best * 1e3:8.2f} us  ({best * 1e3 / tiles:.3f} us/tile)", flush=True)
    a, c0 = np.polyfit(xs, ys, 1)
    print(f"fit: fixed {c0:.2f} us + {a:.3f} us per 64-key tile "
          f"(ideal MFMA-bound tile at 2.4 GHz: {2048 / 2.4e3:.3f} us)", flush=True)


if __name__ == "__main__":
    main()
