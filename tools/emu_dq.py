#!/usr/bin/env python3
"""Runs the generated assembly dQ kernel (csrc/asm/gen_dq.py) in the CPU emulator (tools/asm_emu.py)
on small inputs and compares dQ with a float64 reference (dev / test tool).

    python tools/emu_dq.py [--b 1 --sq 300 --sk 300 --h 2 --hk 1 --full --fp16]
"""
import argparse
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from asm_emu import Emu, Heap, bf16_to_f32, f16_to_f32, f32_to_bf16, f32_to_f16  # noqa: E402
from emu_bwd import reference as bwd_reference  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm"))
from isa import fwd_item_decode  # noqa: E402

GEN = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_dq.py")
GEN64 = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_dq64.py")
BM = 256


def asm_text(d=128):
    return subprocess.run([sys.executable, GEN64 if d == 64 else GEN], check=True, capture_output=True, text=True).stdout


def pack_args(**kw):
    out = struct.pack("<10Q", kw["q"], kw["k"], kw["v"], kw["do"], kw["dq"], kw["lse"], kw["dsum"], kw["sched"],
                      kw["cuq"], kw["cuk"])
    out += struct.pack("<4q", kw["q_batch"], kw["kv_batch"], kw["do_batch"], kw["dq_batch"])
    out += struct.pack("<4i", kw["q_row"], kw["kv_row"], kw["do_row"], kw["dq_row"])
    out += struct.pack("<5i", kw["q_head"], kw["k_head"], kw["v_head"], kw["do_head"], kw["dq_head"])
    out += struct.pack("<7i", kw["sq"], kw["sk"], kw["lse_pitch"], kw["dsum_pitch"], kw["h"], kw["hk"], kw["flags"])
    out += struct.pack("<ff", kw["c"], kw["scale"])
    out += struct.pack("<10I", *kw["dec"])
    out += struct.pack("<ii", kw["n_items"], kw["grid"])
    # fused bwd_pre (flags bit 1): o, o_batch, o_row, o_head, lsed, lsed_ng, -1 / scale
    out += struct.pack("<Qqii", kw.get("o", 0), kw.get("o_batch", 0), kw.get("o_row", 0), kw.get("o_head", 0))
    out += struct.pack("<Qif", kw.get("lsed", 0), kw.get("lsed_ng", 0), kw.get("nrscale", 0.0))
    # the Q fold (flags bit 2): qf, qf_batch, qf_row, qf_head, qc
    out += struct.pack("<Qqiifi", kw.get("qf", 0), kw.get("qf_batch", 0), kw.get("qf_row", 0), kw.get("qf_head", 0),
                       kw.get("qc", 0.0), 0)
    assert len(out) == 304, len(out)
    return out


def reference_dq(q, k, v, do, causal, scale, o=None):
    """o: D = rowsum(dO o O) from this O instead of the forward's (the fused-D test)"""
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    g = h // hk
    lse, dsum, _, _ = bwd_reference(q, k, v, do, causal, scale)
    if o is not None:
        dsum = np.einsum("bshd,bshd->bhs", do, o)
    dq = np.zeros_like(q)
    for bi in range(b):
        for hi in range(h):
            s = q[bi, :, hi] @ k[bi, :, hi // g].T * scale
            if causal:
                s = np.where(np.arange(sk)[None, :] > np.arange(sq)[:, None], -np.inf, s)
            with np.errstate(all="ignore"):
                p = np.where(np.isfinite(lse[bi, hi])[:, None], np.exp(s - lse[bi, hi][:, None]), 0)
            dp = do[bi, :, hi] @ v[bi, :, hi // g].T
            ds = p * (dp - dsum[bi, hi][:, None])
            dq[bi, :, hi] = scale * ds @ k[bi, :, hi // g]
    return lse, dsum, dq


def run(b=1, sq=300, sk=300, h=2, hk=1, causal=True, bf16=True, seed=0, text=None, verbose=True, hp=0, grid=None,
        fused=False, wgs=None, qfold=False, d=128, qmul=1.0, kmul=1.0):
    """hp: heads per XCD group of the work order (0: head-fastest); grid: workgroups of the
    persistent item loop (default: one per item); fused: the kernel computes D = rowsum(dO o O) itself
    (flags bit 1, bwd_pre fused): the D input is garbage, softmax_d and the dK/dV scratch
    [-LSE / scale | -D] are checked against float64 (the error returned is the max of the three);
    qfold (with fused): the Q fold (flags bit 2) -- the kernel rewrites Q as bf16/f16(c Q), stores it
    (checked bitwise against the forward's rounding) and runs with c = 1, scale ln 2 on the chain
    starts, dQ scaled by the softmax scale, against a float64 reference on that Q'; d: head dim
    (128: gen_dq.py, 64: gen_dq64.py); qmul / kmul scale Q and K / V (large |LSE|: the fp16 overflow
    cases)"""
    D = d
    rng = np.random.default_rng(seed)
    q = rng.standard_normal((b, sq, h, D)).astype(np.float32) * np.float32(qmul)
    k = rng.standard_normal((b, sk, hk, D)).astype(np.float32) * np.float32(kmul)
    v = rng.standard_normal((b, sk, hk, D)).astype(np.float32) * np.float32(kmul)
    do = rng.standard_normal((b, sq, h, D)).astype(np.float32)
    enc, dec = (f32_to_bf16, bf16_to_f32) if bf16 else (f32_to_f16, f16_to_f32)
    q16, k16, v16, do16 = (enc(x).astype(np.uint16) for x in (q, k, v, do))
    qf, kf, vf, dof = (dec(x).astype(np.float64) for x in (q16, k16, v16, do16))
    scale = D ** -0.5
    of = None
    if fused:
        o16 = enc(rng.standard_normal((b, sq, h, D)).astype(np.float32)).astype(np.uint16)
        of = dec(o16).astype(np.float64)
    qc32 = np.float32(scale * 1.4426950408889634)
    q_s = qf      # the Q the scores are made of
    if qfold:
        qfold16 = enc(qf.astype(np.float32) * qc32).astype(np.uint16)
        q_s = dec(qfold16).astype(np.float64) * (np.log(2.0) / scale)
    lse, dsum, dq_ref = reference_dq(q_s, kf, vf, dof, causal, scale, o=of)
    if fused:
        dsum = np.einsum("bshd,bshd->bhs", dof, of)
    sqr = (sq + 127) // 128 * 128
    lse32 = lse.astype(np.float32)
    ds32 = np.zeros((b, h, sqr), np.float32)
    ds32[:, :, :sq] = np.nan if fused else dsum
    heap = Heap(64 << 20)
    aq, ak, av, ado = heap.put(q16), heap.put(k16), heap.put(v16), heap.put(do16)
    adq = heap.alloc(b * sq * h * D * 2)
    heap.get(adq, b * sq * h * D * 2)[:] = 0xAB
    alse, ads = heap.put(lse32), heap.put(ds32)
    nmb = (sq + BM - 1) // BM
    n_items = b * h * nmb
    kw = dict(q=aq, k=ak, v=av, do=ado, dq=adq, lse=alse, dsum=ads, sched=0, cuq=0, cuk=0,
              dec=fwd_item_decode(b * h, h, h // hk, nmb, hp), n_items=n_items, grid=grid or n_items,
              q_batch=sq * h * D * 2, kv_batch=sk * hk * D * 2, do_batch=sq * h * D * 2, dq_batch=sq * h * D * 2,
              q_row=h * D * 2, kv_row=hk * D * 2, do_row=h * D * 2, dq_row=h * D * 2,
              q_head=D * 2, k_head=D * 2, v_head=D * 2, do_head=D * 2, dq_head=D * 2,
              sq=sq, sk=sk, lse_pitch=sq, dsum_pitch=sqr, h=h, hk=hk, flags=0,
              c=float(np.float32(scale * 1.4426950408889634)), scale=float(np.float32(scale)))
    ng = (sq + 31) // 32
    sc_l = np.log(2.0) if qfold else scale      # the chain starts' scale (launch_bwd: ln 2 with the fold)
    if fused:
        ao = heap.put(o16)
        alsed = heap.alloc(b * h * ng * 256)
        heap.get(alsed, b * h * ng * 256).view(np.float32)[:] = np.nan
        kw.update(o=ao, o_batch=sq * h * D * 2, o_row=h * D * 2, o_head=D * 2, lsed=alsed, lsed_ng=ng,
                  nrscale=float(np.float32(-1.0 / sc_l)), flags=2)
    if qfold:
        assert fused
        aqf = heap.alloc(b * sq * h * D * 2)
        heap.get(aqf, b * sq * h * D * 2)[:] = 0xAB
        kw.update(qf=aqf, qf_batch=sq * h * D * 2, qf_row=h * D * 2, qf_head=D * 2, qc=float(qc32), c=1.0,
                  flags=2 | 4)
    akarg = heap.put(np.frombuffer(pack_args(**kw), dtype=np.uint8))
    text = text or asm_text(D)
    name = (f"fa_bwd_dq_asm_d{D}_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}"
            f"{'_c1' if D == 64 and kw['c'] == 1.0 else ''}")     # (d = 64: the c = 1 kernels, fa_bwd_asm.cpp)
    emu = Emu(text, name, heap)
    for L in range(grid or n_items) if wgs is None else wgs:
        emu.run_wg(L, akarg)
    dq = dec(heap.get(adq, b * sq * h * D * 2).view(np.uint16)).reshape(b, sq, h, D).astype(np.float64)
    e = np.abs(dq - dq_ref).max() / max(np.abs(dq_ref).max(), 1e-9)
    if fused:
        got = heap.get(ads, b * h * sqr * 4).view(np.float32).reshape(b, h, sqr)[:, :, :sq]
        if wgs is not None:     # a subset of the items: the rows they wrote
            ok = np.isfinite(got)
            ed = np.abs(got[ok] - dsum[ok]).max() / max(np.abs(dsum).max(), 1e-9)
            print(f"softmax_d: {ok.sum()} rows written, rel max err {ed:.3e}")
            return ed, got, dsum
        e = max(e, np.abs(got - dsum).max() / max(np.abs(dsum).max(), 1e-9))
        sc = heap.get(alsed, b * h * ng * 256).view(np.float32).reshape(b, h, ng, 2, 32)
        want = np.zeros((b, h, ng * 32, 2))
        with np.errstate(all="ignore"):
            want[:, :, :sq, 0] = -lse / sc_l
        want[:, :, :sq, 1] = -dsum
        want = want.reshape(b, h, ng, 32, 2).transpose(0, 1, 2, 4, 3)
        fin = np.isfinite(want)
        assert np.array_equal(fin, np.isfinite(sc)), "scratch: non-finite entries differ"
        assert np.array_equal(want[~fin], sc[~fin].astype(np.float64)), "scratch: infinite entries differ"
        e = max(e, np.abs(sc[fin] - want[fin]).max() / max(np.abs(want[fin]).max(), 1e-9))
    if qfold:
        got_qf = heap.get(aqf, b * sq * h * D * 2).view(np.uint16).reshape(b, sq, h, D)
        assert np.array_equal(got_qf, qfold16.reshape(b, sq, h, D)), "Q': not the forward's bf16/f16(c Q)"
    if verbose:
        print(f"b={b} sq={sq} sk={sk} h={h} hk={hk} causal={causal} bf16={bf16}: rel max|ddQ| {e:.3e} "
              f"({emu.count} instructions, {emu.mfma_count} MFMAs)")
    return e, dq, dq_ref


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=1)
    ap.add_argument("--sq", type=int, default=300)
    ap.add_argument("--sk", type=int, default=300)
    ap.add_argument("--h", type=int, default=2)
    ap.add_argument("--hk", type=int, default=1)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--fp16", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fused", action="store_true", help="the kernel computes D (bwd_pre fused)")
    ap.add_argument("--qfold", action="store_true", help="with --fused: the Q fold")
    ap.add_argument("--d", type=int, default=128)
    a = ap.parse_args()
    run(a.b, a.sq, a.sk, a.h, a.hk, not a.full, not a.fp16, a.seed, fused=a.fused or a.qfold, qfold=a.qfold, d=a.d)
