#!/usr/bin/env python3
"""FlashMask forward / backward timing through the C ABI (dev tool, GPU box).

    python tools/fm_bench.py [--docs 8] [--seqlen 8192] [--batch 4] [--heads 16]

Causal document mask with `docs` equal documents, bf16, d = 128.  Prints the kernel-event times and
the throughput over the kept (row, key) pairs next to the plain causal launch of the same shape.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
import flash_attn_2_cuda as m  # noqa: E402


def run(q, k, v, dout, causal, fm, iters):
    b, s, h, d = q.shape
    P = m._ptr
    out = torch.empty_like(q)
    lse = torch.empty(b, h, s, device="cuda")
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    sd = torch.empty(b, h, s, device="cuda")
    st = (q.stride(1),) * 3 + (q.stride(2),) * 3 + (out.stride(1), out.stride(2)) + (q.stride(0),) * 4
    bst = st + (q.stride(1),) * 3 + (q.stride(2),) * 3 + (q.stride(1), q.stride(2)) + (q.stride(0),) * 4
    fmargs = fm if fm is not None else (None,) * 6

    def fwd():
        assert m._lib.flash_attn_fwd(P(q), P(k), P(v), None, P(out), None, P(lse), b, s, s, s, s, h, h, d, d,
                                     0.0, d ** -0.5, 1.0, causal, False, True, m._stream(q), 0, 0,
                                     None, None, *fmargs, *st), m._lib.flash_attn_error()

    def bwd():
        assert m._lib.flash_attn_bwd(P(dout), P(q), P(k), P(v), P(out), P(sd), P(lse), None, P(dq), P(dk),
                                     P(dv), None, b, s, s, s, s, h, h, d, d, 0.0, d ** -0.5, 1.0, causal,
                                     True, 1, m._stream(q), 0, 0, None, None, *fmargs,
                                     *bst), m._lib.flash_attn_error()

    res = {}
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / iters
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=8)
    ap.add_argument("--seqlen", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    b, s, h, d = a.batch, a.seqlen, a.heads, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v, dout = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4))
    ends = np.repeat(np.arange(1, a.docs + 1) * (s // a.docs), s // a.docs).astype(np.int32)
    ends[-1:] = s
    lts = torch.from_numpy(np.broadcast_to(ends, (b, 1, s)).copy()).cuda()
    dims = torch.tensor([b, 1, s, 1], dtype=torch.int64)
    fm = (m._ptr(lts), dims.numpy().ctypes.data, None, None, None, None)
    flops_causal = 4 * b * h * d * s * (s + 1) / 2
    doc = s // a.docs
    flops_doc = 4 * b * h * d * a.docs * doc * (doc + 1) / 2
    base = run(q, k, v, dout, True, None, a.iters)
    fmr = run(q, k, v, dout, True, fm, a.iters)
    for name, r, fl in (("causal", base, flops_causal), (f"doc{a.docs}", fmr, flops_doc)):
        print(f"{name:8s} fwd {r['fwd']:.3f} ms ({fl / r['fwd'] / 1e9:.0f} TF on kept pairs)  "
              f"bwd {r['bwd']:.3f} ms ({2.5 * fl / r['bwd'] / 1e9:.0f} TF)")


if __name__ == "__main__":
    main()
