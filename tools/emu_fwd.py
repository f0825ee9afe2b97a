#!/usr/bin/env python3
"""Runs the generated assembly forward (csrc/asm/gen_fwd.py) in the CPU emulator (tools/asm_emu.py)
on small inputs and compares O / LSE with a float64 reference (dev / test tool).

    python tools/emu_fwd.py [--b 1 --sq 300 --sk 300 --h 2 --hk 1 --full --fp16 --grid G --hp HP]
"""
import argparse
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm"))
from asm_emu import Emu, Heap, bf16_to_f32, f16_to_f32, f32_to_bf16, f32_to_f16  # noqa: E402
from isa import fwd_item_decode  # noqa: E402

GEN = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_fwd.py")
D = 128
BM = 256


def asm_text():
    return subprocess.run([sys.executable, GEN], check=True, capture_output=True, text=True).stdout


def pack_args(**kw):
    head = struct.pack("<11Q4q", kw["q"], kw["k"], kw["v"], kw["o"], kw["lse"], kw["sched"], kw["cuq"], kw["cuk"],
                       kw["rng"], kw["seed"], kw["off"], kw["q_batch"], kw["k_batch"], kw["v_batch"], kw["o_batch"])
    assert len(head) == 120
    tail = struct.pack("<11i", kw["q_row"], kw["kv_row"], kw["o_row"], kw["q_head"], kw["k_head"], kw["v_head"],
                       kw["o_head"], kw["sq"], kw["sk"], kw["lse_pitch"], kw["h"])
    tail += struct.pack("<fiiii", kw["c"], kw["flags"], kw["n_items"], kw["grid"], 0)
    out = head + tail + struct.pack("<10I", *kw["dec"])
    assert len(out) == 224, len(out)
    return out


def reference(q, k, v, causal, scale, seqs_q=None, seqs_k=None):
    """float64 attention; q (b, sq, h, d), k/v (b, sk, hk, d); returns o, lse (b, h, sq)"""
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    g = h // hk
    o = np.zeros((b, sq, h, d))
    lse = np.full((b, h, sq), np.inf)
    for bi in range(b):
        lq = seqs_q[bi] if seqs_q is not None else sq
        lk = seqs_k[bi] if seqs_k is not None else sk
        for hi in range(h):
            s = q[bi, :lq, hi].astype(np.float64) @ k[bi, :lk, hi // g].astype(np.float64).T * scale
            if causal:
                s = np.where(np.arange(lk)[None, :] > np.arange(lq)[:, None], -np.inf, s)
            m = s.max(axis=1, keepdims=True)
            p = np.exp(s - m)
            l = p.sum(axis=1, keepdims=True)
            o[bi, :lq, hi] = (p / l) @ v[bi, :lk, hi // g]
            lse[bi, hi, :lq] = (m + np.log(l))[:, 0]
    return o, lse


def run(b=1, sq=300, sk=300, h=2, hk=1, causal=True, bf16=True, seed=0, big=None, text=None, verbose=True,
        grid=None, d=128, hp=0, fold=None, prefix="fa_fwd_asm"):
    """grid: workgroups of the persistent item loop (default: one per item); d: head dim (128, 64);
    hp: heads per XCD group of the work order (0: head-fastest); fold: compare with the folded-scale
    arithmetic (gen_fwd.py FA_GEN_FOLD, default as the generator's environment); prefix: the kernel
    name prefix ("fa_fwdnf_asm": gen_fwdnf.py's unfolded kernels, with fold=False)"""
    if fold is None:
        fold = os.environ.get("FA_GEN_FOLD", "1") == "1"
    D = d
    rng = np.random.default_rng(seed)
    q = rng.standard_normal((b, sq, h, D)).astype(np.float32)
    k = rng.standard_normal((b, sk, hk, D)).astype(np.float32)
    v = rng.standard_normal((b, sk, hk, D)).astype(np.float32)
    if big is not None:   # a late score jump: forces the refit path
        q[:, :, :, :] *= 0.3
        k[:, big:big + 3] *= 12.0
    enc, dec = (f32_to_bf16, bf16_to_f32) if bf16 else (f32_to_f16, f16_to_f32)
    q16, k16, v16 = (enc(x).astype(np.uint16) for x in (q, k, v))
    qf, kf, vf = (dec(x).astype(np.float64) for x in (q16, k16, v16))
    scale = D ** -0.5
    heap = Heap(64 << 20)
    aq, ak, av = heap.put(q16), heap.put(k16), heap.put(v16)
    ao = heap.alloc(b * sq * h * D * 2)
    heap.get(ao, b * sq * h * D * 2)[:] = 0xAB   # poison
    alse = heap.alloc(b * h * sq * 4)
    nmb = (sq + BM - 1) // BM
    n_items = b * h * nmb
    kw = dict(q=aq, k=ak, v=av, o=ao, lse=alse, sched=0, cuq=0, cuk=0, rng=0, seed=0, off=0,
              q_batch=sq * h * D * 2, k_batch=sk * hk * D * 2, v_batch=sk * hk * D * 2, o_batch=sq * h * D * 2,
              q_row=h * D * 2, kv_row=hk * D * 2, o_row=h * D * 2, q_head=D * 2, k_head=D * 2, v_head=D * 2,
              o_head=D * 2, sq=sq, sk=sk, lse_pitch=sq, h=h, c=float(np.float32(scale * 1.4426950408889634)), flags=0,
              n_items=n_items, grid=grid or n_items, dec=fwd_item_decode(b * h, h, h // hk, nmb, hp))
    akarg = heap.put(np.frombuffer(pack_args(**kw), dtype=np.uint8))
    text = text or asm_text()
    name = f"{prefix}_d{D}_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}"
    emu = Emu(text, name, heap)
    for L in range(grid or n_items):
        emu.run_wg(L, akarg)
    o = dec(heap.get(ao, b * sq * h * D * 2).view(np.uint16)).reshape(b, sq, h, D).astype(np.float64)
    lse = heap.get(alse, b * h * sq * 4).view(np.float32).reshape(b, h, sq).astype(np.float64)
    o_ref, lse_ref = reference(qf, kf, vf, causal, scale)
    if fold:
        # the kernel's own arithmetic: Q held as bf16/f16(c Q), scores c S in the log2 domain
        c = np.float32(scale * 1.4426950408889634)
        qc = dec(enc(qf.astype(np.float32) * c).astype(np.uint16)).astype(np.float64)
        o_ref, lse_ref = reference(qc * (np.log(2.0) / scale), kf, vf, causal, scale)
    eo = np.abs(o - o_ref).max()
    el = np.abs(lse - lse_ref).max()
    if verbose:
        print(f"b={b} sq={sq} sk={sk} h={h} hk={hk} causal={causal} bf16={bf16}: max|dO| {eo:.3e} max|dLSE| {el:.3e}"
              f"  ({emu.count} instructions, {emu.mfma_count} MFMAs)")
    return eo, el, o, o_ref, lse, lse_ref


def run_varlen(seqs_q, seqs_k=None, h=2, hk=1, causal=True, bf16=True, seed=0, text=None, verbose=True, d=128):
    """varlen: packed (total, h, d) Q / K / V and cu_seqlens (one workgroup per item, as the
    launcher runs varlen calls whose K/V stream is grouped per XCD); compares every sequence with
    the float64 reference on the kernel's folded scores"""
    seqs_k = seqs_k or seqs_q
    D, b = d, len(seqs_q)
    rng = np.random.default_rng(seed)
    tq, tk = sum(seqs_q), sum(seqs_k)
    q = rng.standard_normal((tq, h, D)).astype(np.float32)
    k = rng.standard_normal((tk, hk, D)).astype(np.float32)
    v = rng.standard_normal((tk, hk, D)).astype(np.float32)
    enc, dec = (f32_to_bf16, bf16_to_f32) if bf16 else (f32_to_f16, f16_to_f32)
    q16, k16, v16 = (enc(x).astype(np.uint16) for x in (q, k, v))
    qf, kf, vf = (dec(x).astype(np.float64) for x in (q16, k16, v16))
    scale = D ** -0.5
    msq, msk = max(seqs_q), max(seqs_k)
    heap = Heap(64 << 20)
    aq, ak, av = heap.put(q16), heap.put(k16), heap.put(v16)
    ao = heap.alloc(tq * h * D * 2)
    heap.get(ao, tq * h * D * 2)[:] = 0xAB   # poison
    alse = heap.alloc(b * h * msq * 4)
    cuq = np.array([0] + list(np.cumsum(seqs_q)), dtype=np.int32)
    cuk = np.array([0] + list(np.cumsum(seqs_k)), dtype=np.int32)
    acq, ack = heap.put(cuq), heap.put(cuk)
    nmb = (msq + BM - 1) // BM
    n_items = b * h * nmb
    kw = dict(q=aq, k=ak, v=av, o=ao, lse=alse, sched=0, cuq=acq, cuk=ack, rng=0, seed=0, off=0,
              q_batch=0, k_batch=0, v_batch=0, o_batch=0,
              q_row=h * D * 2, kv_row=hk * D * 2, o_row=h * D * 2, q_head=D * 2, k_head=D * 2, v_head=D * 2,
              o_head=D * 2, sq=msq, sk=msk, lse_pitch=msq, h=h, c=float(np.float32(scale * 1.4426950408889634)),
              flags=0, n_items=n_items, grid=n_items, dec=fwd_item_decode(b * h, h, h // hk, nmb, 0))
    akarg = heap.put(np.frombuffer(pack_args(**kw), dtype=np.uint8))
    text = text or asm_text()
    name = f"fa_fwd_asm_d{D}_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}"
    emu = Emu(text, name, heap)
    for L in range(n_items):
        emu.run_wg(L, akarg)
    o = dec(heap.get(ao, tq * h * D * 2).view(np.uint16)).reshape(tq, h, D).astype(np.float64)
    lse = heap.get(alse, b * h * msq * 4).view(np.float32).reshape(b, h, msq).astype(np.float64)
    c = np.float32(scale * 1.4426950408889634)
    qc = dec(enc(qf.astype(np.float32) * c).astype(np.uint16)).astype(np.float64) * (np.log(2.0) / scale)
    eo = el = 0.0
    for i in range(b):
        lq, lk = seqs_q[i], seqs_k[i]
        if lq and not lk:   # rows without keys: O = 0, LSE = +inf (flash_fwd_kernel.h:509-518)
            eo = max(eo, float(np.nan_to_num(np.abs(o[cuq[i]:cuq[i + 1]]), nan=np.inf).max()))
            el = max(el, 0.0 if np.all(lse[i, :, :lq] == np.inf) else np.inf)
            continue
        if lq == 0 or lk == 0:
            continue
        o_ref, lse_ref = reference(qc[None, cuq[i]:cuq[i + 1]], kf[None, cuk[i]:cuk[i + 1]],
                                   vf[None, cuk[i]:cuk[i + 1]], causal, scale)
        eo = max(eo, np.abs(o[cuq[i]:cuq[i + 1]] - o_ref[0]).max())
        el = max(el, np.abs(lse[i, :, :lq] - lse_ref[0]).max())
    if verbose:
        print(f"varlen seqs_q={seqs_q} seqs_k={seqs_k} h={h} hk={hk} causal={causal} bf16={bf16} d={D}: "
              f"max|dO| {eo:.3e} max|dLSE| {el:.3e}  ({emu.count} instructions)")
    return eo, el


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=1)
    ap.add_argument("--sq", type=int, default=300)
    ap.add_argument("--sk", type=int, default=300)
    ap.add_argument("--h", type=int, default=2)
    ap.add_argument("--hk", type=int, default=1)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--fp16", action="store_true")
    ap.add_argument("--big", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--hp", type=int, default=0)
    ap.add_argument("--varlen", type=str, default=None, help="comma-separated sequence lengths")
    a = ap.parse_args()
    if a.varlen:
        run_varlen([int(x) for x in a.varlen.split(",")], h=a.h, hk=a.hk, causal=not a.full, bf16=not a.fp16, d=a.d)
        sys.exit(0)
    run(a.b, a.sq, a.sk, a.h, a.hk, not a.full, not a.fp16, a.seed, a.big, grid=a.grid, d=a.d, hp=a.hp)
