#!/usr/bin/env python3
"""A/B timing of library variants in ONE process (dev tool, not part of the product).

    python tools/ab.py LIB_A.so LIB_B.so ... [--workload c3] [--rounds 5] [--iters 10] [--bwd]

A variant may carry knob settings, ``LIB.so@9=2,6=0``: flash_attn_set_knob before each of its turns
(the same library may then appear several times; knobs another variant sets return to their
default values for the variants that do not).

Every variant library is loaded side by side (ctypes, RTLD_LOCAL) and driven through the same
``flash_attn_2_cuda`` Python mirror by swapping its ``_lib`` handle; rounds interleave the variants
so clock / thermal drift hits all of them alike (cdna_hip_programming.md §5.4 rule 24).  Each
variant's kernel times come from its own HIP-event timers (``flash_attn_timing_*``).  Outputs of
every variant are compared with the first one's.
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import flash_attn_2_cuda as m  # noqa: E402
from bench import KERNELS, WORKLOADS, c4_seqlens, flops_fwd, varlen_flops_fwd  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    for name, sig in (("flash_attn_fwd", m._FWD), ("flash_attn_varlen_fwd", m._VARLEN_FWD),
                      ("flash_attn_bwd", m._BWD), ("flash_attn_bwd_gqa", m._BWD),
                      ("flash_attn_varlen_bwd", m._VARLEN_BWD), ("flash_attn_varlen_bwd_gqa", m._VARLEN_BWD)):
        fn = getattr(lib, name)
        fn.argtypes = sig
        fn.restype = ctypes.c_bool
    lib.flash_attn_error.restype = ctypes.c_char_p
    lib.flash_attn_timing_enable.argtypes = [ctypes.c_int]
    lib.flash_attn_timing_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_long)]
    return lib


def read_times(lib):
    out = {}
    for kid, name in KERNELS.items():
        ms, n = ctypes.c_double(), ctypes.c_long()
        lib.flash_attn_timing_read(kid, ctypes.byref(ms), ctypes.byref(n))
        if n.value:
            out[name] = ms.value / n.value
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--dropout", type=float, default=0.0)
    args = ap.parse_args()
    pd = args.dropout

    b, s, h, hk, d, dt, causal, _kind = WORKLOADS[args.workload]
    dtype = torch.bfloat16 if dt == "bf16" else torch.float16
    g = torch.Generator(device="cuda").manual_seed(1234)
    varlen = b is None       # c4: varlen, the packed qkv's views, SURVEY 8(d) sequence lengths
    if varlen:
        lens = c4_seqlens(total=s)
        cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")
        qkv = torch.randn(s, 3, h, d, device="cuda", dtype=dtype, generator=g)
        q, k, v = qkv.unbind(1)
        dout = torch.randn(s, h, d, device="cuda", dtype=dtype, generator=g)
        ms_ = max(lens)
    else:
        q = torch.randn(b, s, h, d, device="cuda", dtype=dtype, generator=g)
        k = torch.randn(b, s, hk, d, device="cuda", dtype=dtype, generator=g)
        v = torch.randn(b, s, hk, d, device="cuda", dtype=dtype, generator=g)
        dout = torch.randn(b, s, h, d, device="cuda", dtype=dtype, generator=g)
    scale = d ** -0.5

    def fwd(gen):
        if varlen:
            return m.varlen_fwd(q, k, v, None, cu, cu, ms_, ms_, pd, scale, False, causal, False, gen)
        return m.fwd(q, k, v, None, pd, scale, causal, False, gen)

    def bwd(res):
        if varlen:
            return m.varlen_bwd(dout, q, k, v, res[0], res[5], None, None, None, cu, cu, ms_, ms_, pd, scale, False,
                                causal, None, res[7])
        return m.bwd(dout, q, k, v, res[0], res[5], None, None, None, pd, scale, causal, None, res[7])
    specs = [(p.split("@")[0], dict(tuple(int(x) for x in kv.split("=")) for kv in p.split("@")[1].split(",")) if "@" in p else {})
             for p in args.libs]
    cache = {}
    libs = [cache.setdefault(p, load(p)) if p not in cache else cache[p] for p, _ in specs]
    for lib in cache.values():
        lib.flash_attn_get_knob.restype = ctypes.c_int
    touched = sorted({kid for _, kn in specs for kid in kn})
    defaults = {kid: cache[specs[0][0]].flash_attn_get_knob(kid) for kid in touched}
    names = [os.path.basename(p) + ("@" + ",".join(f"{kid}={val}" for kid, val in kn.items()) if kn else "") for p, kn in specs]
    times = {n: {} for n in names}
    ref = None
    for rnd in range(args.rounds):
        for lib, name, (_, kn) in zip(libs, names, specs):
            m._lib = lib
            for kid in touched:
                lib.flash_attn_set_knob(kid, kn.get(kid, defaults[kid]))
            gen = torch.Generator(device="cuda").manual_seed(7) if pd > 0 else None
            res = fwd(gen)
            out, lse = res[0], res[5]
            grads = None
            if args.bwd:
                grads = bwd(res)[:3]
            torch.cuda.synchronize()
            if rnd == 0:
                cur = [out, lse] + (list(grads) if grads else [])
                if ref is None:
                    ref = [x.clone() for x in cur]
                else:
                    diffs = [(a.float() - r.float()).abs().max().item() for a, r in zip(cur, ref)]
                    print(f"{name}: max|diff| vs {names[0]} (out, lse, dq, dk, dv) = "
                          + ", ".join(f"{x:.3e}" for x in diffs), flush=True)
            lib.flash_attn_timing_enable(1)
            for _ in range(args.iters):
                r2 = fwd(None)
                if args.bwd:
                    bwd(r2)
            torch.cuda.synchronize()
            t = read_times(lib)
            lib.flash_attn_timing_enable(0)
            for kname, ms in t.items():
                times[name].setdefault(kname, []).append(ms)
    f = varlen_flops_fwd(lens, h, d, causal) if varlen else flops_fwd(b, s, h, d, causal)
    alg = {"fwd_kernel": f, "bwd_dkdv_kernel": 2 * f, "bwd_dq_kernel": 1.5 * f, "bwd_pre_kernel": 0}
    for name in names:
        parts = []
        for kname, xs in sorted(times[name].items()):
            med, mn = statistics.median(xs), min(xs)
            tf = alg.get(kname, 0) / (med / 1e3) / 1e12 if alg.get(kname) else 0
            parts.append(f"{kname} med {med:.4f} ms min {mn:.4f} ({tf:.0f} TF)")
        print(f"{name}: " + " | ".join(parts), flush=True)


if __name__ == "__main__":
    main()
