#!/usr/bin/env python3
"""Workgroup timeline of the assembly dK/dV kernel (dev tool): with a library whose kernel was
generated with FA_GBW_STAMP=1 (tools/asm_variant.sh), every workgroup stores its start / end
s_memtime and CU; per CU the workgroups are sorted by start and the gaps between them, the busy
share and the tail are reported.

    FA_GBW_STAMP=1 bash tools/asm_variant.sh stamp && python tools/bwd_stamps.py variants/libfa_stamp.so
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from ab import load  # noqa: E402


def main(path, b=4, s=8192, h=16, c4=False):
    """c4: the C4 varlen workload (bench.c4_seqlens, 32 heads; one workgroup per item)"""
    lib = load(path)
    lib.flash_attn_debug_bwd_stamps.argtypes = [ctypes.c_void_p]
    m._lib = lib
    scale = 128 ** -0.5
    if c4:
        from bench import c4_seqlens
        lens = c4_seqlens()
        h, b, s = 32, len(lens), max(lens)
        cu_t = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")
        q, k, v, do = (torch.randn(sum(lens), h, 128, device="cuda", dtype=torch.bfloat16) for _ in range(4))
        res = m.varlen_fwd(q, k, v, None, cu_t, cu_t, s, s, 0.0, scale, False, True, False, None)
    else:
        q, k, v, do = (torch.randn(b, s, h, 128, device="cuda", dtype=torch.bfloat16) for _ in range(4))
        res = m.fwd(q, k, v, None, 0.0, scale, True, False, None)
    nwg = b * h * ((s + 127) // 128)
    steps = "--steps" in sys.argv[2:]
    buf = torch.zeros(nwg * 16 * (4 if steps else 1), dtype=torch.int32, device="cuda")
    for it in range(3):
        lib.flash_attn_debug_bwd_stamps(ctypes.c_void_p(buf.data_ptr() if it == 2 else 0))
        if c4:
            m.varlen_bwd(do, q, k, v, res[0], res[5], None, None, None, cu_t, cu_t, s, s, 0.0, scale, False, True,
                         None, res[7])
        else:
            m.bwd(do, q, k, v, res[0], res[5], None, None, None, 0.0, scale, True, None, res[7])
        torch.cuda.synchronize()
    lib.flash_attn_debug_bwd_stamps(ctypes.c_void_p(0))
    if steps:   # FA_GBW_STAMP=2: per wave {compute, wait, barrier, steps, -, prologue, epilogue, items}
        a = buf.cpu().numpy().view(np.uint32).reshape(nwg * 4, 16).astype(np.int64)
        a = a[a[:, 7] > 0]
        st = np.maximum(a[:, 3], 1)
        it = np.maximum(a[:, 7], 1)
        cont = "cont" in sys.argv[2:]   # a pipelined-loop build: 10, 11 = item switch parts, 12 = the last steps' compute
        if cont:
            a[:, 0] += a[:, 12]
            print(f"  (pipelined loop) last step compute per item med {np.median(a[:, 12] / np.maximum(a[:, 7], 1)):.0f}; "
                  f"switch: record {np.median(a[:, 10] / np.maximum(a[:, 7], 1)):.0f}, DMA drain {np.median(a[:, 11] / np.maximum(a[:, 7], 1)):.0f}")
            print(f"  (pipelined loop) the 2 steps before the last: compute per item med {np.median(a[:, 13] / np.maximum(a[:, 7], 1)):.0f}; "
                  f"switch tail (re-issue, C) {np.median(a[:, 14] / np.maximum(a[:, 7], 1)):.0f}, item barrier {np.median(a[:, 15] / np.maximum(a[:, 7], 1)):.0f}")
            a[:, 12] = 0
            a[:, 13] = 0
        tot = a[:, 0] + a[:, 1] + a[:, 2] + a[:, 5] + a[:, 6] + a[:, 10:16].sum(1)
        a[:, 5] += a[:, 10:16].sum(1)   # the prologue: its parts (10..15) and phase -1 (5)
        print(f"waves {len(a)}, items per wave med {np.median(a[:, 7]):.0f}, steps per wave med {np.median(a[:, 3]):.0f}")
        for i, nm in ((0, "compute"), (1, "vmwait"), (2, "barrier")):
            print(f"  {nm}: per step med {np.median(a[:, i] / st):.0f} cycles, share {np.median(a[:, i] / tot):.3f}")
        for i, nm in ((5, "prologue"), (6, "tail+epilogue")):
            print(f"  {nm}: per item med {np.median(a[:, i] / it):.0f} cycles, share {np.median(a[:, i] / tot):.3f}")
        for i, nm in ((10, "head (barrier, item)"), (11, "kernargs + work order"), (12, "geometry"),
                      (13, "K / V loads + lane values"), (14, "DMA issue"), (15, "first wait + barrier")):
            print(f"    prologue part {nm}: per item med {np.median(a[:, i] / it):.0f} cycles")
        print(f"    prologue part phase -1 + wait: per item med {np.median((a[:, 5] - a[:, 10:16].sum(1)) / it):.0f} cycles")
        print(f"  total per wave med {np.median(tot):.0f} cycles; ideal MFMA cycles per step 2048 (64 MFMAs)")
        return
    start = a[:, 0].astype(np.int64) | (a[:, 1].astype(np.int64) << 32)
    end = a[:, 5].astype(np.int64) | (a[:, 6].astype(np.int64) << 32)
    hwid, xcc = a[:, 2], a[:, 3]
    cu = (xcc.astype(np.int64) << 16) | ((hwid >> 8) & 0xFF)
    ran = end > 0                       # (a persistent grid leaves the records of unrun items at 0)
    start, end, hwid, xcc, cu, a = start[ran], end[ran], hwid[ran], xcc[ran], cu[ran], a[ran]
    nwg = int(ran.sum())
    # s_memtime runs per XCD: spans and heads / tails are taken within each XCD
    t0x = {x: start[xcc == x].min() for x in np.unique(xcc)}
    t1x = {x: end[xcc == x].max() for x in np.unique(xcc)}
    t0 = start.min()
    span = float(np.median([t1x[x] - t0x[x] for x in t0x]))
    print(f"{nwg} workgroups, span {span} ticks (s_memtime), mean WG duration {np.mean(end - start):.0f}")
    gaps, busy, tails, heads = [], [], [], []
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        o = idx[np.argsort(start[idx])]
        st, en = start[o], end[o]
        gaps += list(st[1:] - en[:-1])
        x = xcc[o[0]]
        busy.append((en - st).sum() / (t1x[x] - t0x[x]))
        heads.append(st[0] - t0x[x])
        tails.append(t1x[x] - en[-1])
    gaps = np.array(gaps)
    print(f"CUs {len(busy)}; WGs per CU {nwg / len(busy):.1f}; busy share mean {np.mean(busy):.3f} min {np.min(busy):.3f}")
    print(f"gap between consecutive WGs on a CU: median {np.median(gaps):.0f} mean {gaps.mean():.0f} p90 {np.percentile(gaps, 90):.0f}"
          f" ticks ({gaps.sum() / len(busy) / span:.3f} of the span per CU)")
    print(f"first WG start after t0: median {np.median(heads):.0f}; tail after last WG end: median {np.median(tails):.0f} "
          f"mean {np.mean(tails):.0f} ({np.mean(tails) / span:.3f} of the span)")
    # durations of the heaviest / lightest key blocks (kblock from the WG's table order is unknown here:
    # report the distribution)
    d = end - start
    print("WG duration percentiles (ticks): " + ", ".join(f"p{p} {np.percentile(d, p):.0f}" for p in (1, 10, 50, 90, 99)))
    loop = a[:, 8].astype(np.int64) | (a[:, 9].astype(np.int64) << 32)
    epi = a[:, 10].astype(np.int64) | (a[:, 11].astype(np.int64) << 32)
    ok = (loop > 0) & (epi > 0)
    pro_t, epi_t = (loop - start)[ok], (end - epi)[ok]
    print(f"prologue (start -> first step) median {np.median(pro_t):.0f} ticks, epilogue median {np.median(epi_t):.0f};"
          f" per CU {np.sum(pro_t) / len(busy) / span:.3f} / {np.sum(epi_t) / len(busy) / span:.3f} of the span")


if __name__ == "__main__":
    main(sys.argv[1], c4="--c4" in sys.argv[2:])
