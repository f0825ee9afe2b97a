#!/usr/bin/env python3
"""Held clock and cycles per K/V tile of the assembly forward (dev tool; MI355X_MICROARCH.md 'DVFS
give-back' item 6).  With a library whose forward was generated with FA_GEN_STAMP=1, every wave
stores {s_memtime, s_memrealtime} at its start and end plus the tiles / items it ran; after >= 2 s of
back-to-back launches on random data one stamped launch is read back:

    clock  = d(s_memtime) / d(s_memrealtime) x 100 MHz    (median over waves)
    cycles per tile = d(s_memtime) / tiles                  (all of a wave's items, prologues included)
With FA_GEN_STAMP=2 each pipelined step also sums its compute, its end-of-step wait and its barrier
wait (s_memtime around them), reported per step.

    FA_GEN_STAMP=1 bash tools/asm_variant.sh stamp && python tools/fwd_stamps.py variants/libfa_stamp.so
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from ab import load  # noqa: E402
from bench import WORKLOADS, c4_seqlens  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--warm-s", type=float, default=2.0)
    ap.add_argument("--samples", type=int, default=3)
    ap.add_argument("--epi", action="store_true", help="library built with FA_GEN_STAMP=3 (epilogue parts)")
    ap.add_argument("--t0", action="store_true", help="library built with FA_GEN_STAMP=4 (item-start parts)")
    args = ap.parse_args()
    lib = load(args.lib)
    lib.flash_attn_debug_fwd_stamps.argtypes = [ctypes.c_void_p]
    m._lib = lib
    b, s, h, hk, d, dt, causal, _ = WORKLOADS[args.workload]
    dtype = torch.bfloat16 if dt == "bf16" else torch.float16
    scale = d ** -0.5
    if b is None:   # c4: varlen over the SURVEY 8(d) sequence lengths, packed qkv views
        lens = c4_seqlens(total=s)
        cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")
        q, k, v = torch.randn(s, 3, h, d, device="cuda", dtype=dtype).unbind(1)
        ms_ = max(lens)

        def call():
            m.varlen_fwd(q, k, v, None, cu, cu, ms_, ms_, 0.0, scale, False, causal, False, None)
    else:
        q = torch.randn(b, s, h, d, device="cuda", dtype=dtype)
        k = torch.randn(b, s, hk, d, device="cuda", dtype=dtype)
        v = torch.randn(b, s, hk, d, device="cuda", dtype=dtype)

        def call():
            m.fwd(q, k, v, None, 0.0, scale, causal, False, None)
    # one 128-byte record per wave of the grid: the persistent grid has one workgroup per CU, but a
    # varlen launch without the device list runs one workgroup per item -- size for the larger (an
    # item covers >= 32 query rows of one head), or the stamp stores run past the buffer
    rows_q = s if b is None else b * s
    nwave = max(256 * 4 * 4, 4 * h * (rows_q // 32 + (0 if b is None else b) + 256))
    buf = torch.zeros(nwave * 32, dtype=torch.int32, device="cuda")
    rows = []
    for smp in range(args.samples):
        lib.flash_attn_debug_fwd_stamps(ctypes.c_void_p(0))
        t_end = time.time() + args.warm_s
        n = 0
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        while time.time() < t_end:
            for _ in range(10):
                call()
            n += 10
            torch.cuda.synchronize()
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / n
        buf.zero_()
        lib.flash_attn_debug_fwd_stamps(ctypes.c_void_p(buf.data_ptr()))
        call()
        torch.cuda.synchronize()
        lib.flash_attn_debug_fwd_stamps(ctypes.c_void_p(0))
        a = buf.cpu().numpy().view(np.uint32).reshape(nwave, 32).astype(np.int64)
        live = a[:, 0] | a[:, 1] | a[:, 4] | a[:, 5]
        a = a[live != 0]
        t0 = a[:, 0] | (a[:, 1] << 32)
        r0 = a[:, 2] | (a[:, 3] << 32)
        t1 = a[:, 4] | (a[:, 5] << 32)
        r1 = a[:, 6] | (a[:, 7] << 32)
        tiles, items = a[:, 8], a[:, 9]
        clk = (t1 - t0) / np.maximum(r1 - r0, 1) * 0.1       # GHz
        cpt = (t1 - t0) / np.maximum(tiles, 1)
        span_us = (r1.max() - r0.min()) / 100.0
        row = dict(sample=smp, launches=n, launch_ms=ms, waves=len(a), clock_ghz_med=float(np.median(clk)),
                   clock_ghz_p10=float(np.percentile(clk, 10)), clock_ghz_p90=float(np.percentile(clk, 90)),
                   cycles_per_tile_med=float(np.median(cpt)), cycles_per_tile_min=float(cpt.min()),
                   us_per_tile_med=float(np.median((r1 - r0) / 100.0 / np.maximum(tiles, 1))),
                   tiles_med=float(np.median(tiles)), items_med=float(np.median(items)), span_us=float(span_us),
                   ideal_cycles_per_tile=16 * d)
        row["mfma_busy_cycles"] = 16 * d / row["cycles_per_tile_med"]
        steps = a[:, 19]
        if steps.max() > 0:   # FA_GEN_STAMP=2: per-step compute / wait / barrier cycles
            for i, nm in ((16, "compute"), (17, "vmwait"), (18, "barrier")):
                row[f"{nm}_per_step_med"] = float(np.median(a[:, i] / np.maximum(steps, 1)))
            row["steps_med"] = float(np.median(steps))
            items = np.maximum(a[:, 9], 1)
            names = (("epi_lse", "last_step", "epi_o_b", "epi_o_a") if args.epi else
                     ("t0_vmwait", "last_step", "epilogue", "geometry") if args.t0 else
                     ("tile0", "last_step", "epilogue", "item_start"))
            for i, nm in zip((20, 21, 22, 23), names):
                row[f"{nm}_per_item_med"] = float(np.median(a[:, i] / items))
            if args.t0:
                row["t0_barrier_per_item_med"] = float(np.median(a[:, 24] / items))
        rows.append(row)
        print(" ".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}" for k, v in row.items()), flush=True)


if __name__ == "__main__":
    main()
