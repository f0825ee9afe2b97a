#!/usr/bin/env python3
"""Runs the generated assembly dK / dV kernel (csrc/asm/gen_bwd.py) in the CPU emulator
(tools/asm_emu.py) on small inputs and compares dK / dV with a float64 reference (dev / test tool).

    python tools/emu_bwd.py [--b 1 --sq 200 --sk 200 --h 2 --hk 1 --full --fp16 --noreduce]
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
from isa import dkdv_item_decode  # noqa: E402
from asm_emu import Emu, Heap, bf16_to_f32, f16_to_f32, f32_to_bf16, f32_to_f16  # noqa: E402

GEN = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_bwd.py")
GEN2 = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_bwd2.py")
GEN64 = os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_bwd64.py")
D = 128
BKN = 128
# (v2: the two-waves-per-SIMD kernel of gen_bwd2.py, 8 waves per workgroup; same arguments)
KINDS = {1: (GEN, "fa_bwd_dkdv_asm", 4), 2: (GEN2, "fa_bwd2_dkdv_asm", 8), 64: (GEN64, "fa_bwd_dkdv_asm", 4)}
DIMS = {1: (128, 128), 2: (128, 128), 64: (64, 256)}     # (head dim, keys per workgroup)
# the -LSE / -D ring, which every wave DMAs with the same bytes (benign for the race checker)
_NS = int(os.environ.get("FA_GBW_NS", "9"))      # (gen_bwd.py's Q / dO ring slots)
LRING = {1: (_NS * 16384, _NS * 16384 + 4096), 2: (114688, 114688 + 4096), 64: (_NS * 8192, _NS * 8192 + 4096)}
RACES = []          # cross-wave LDS races the last run found (race checker on)


def asm_text(v=1):
    return subprocess.run([sys.executable, KINDS[v][0]], check=True, capture_output=True, text=True).stdout


def pack_args(**kw):
    out = struct.pack("<10Q", kw["q"], kw["k"], kw["v"], kw["do"], kw["dk"], kw["dv"], kw["lsed"], kw["sched"],
                      kw["cuq"], kw["cuk"])
    out += struct.pack("<6q", kw["q_batch"], kw["k_batch"], kw["v_batch"], kw["do_batch"], kw["dk_batch"], kw["dv_batch"])
    out += struct.pack("<6i", kw["q_row"], kw["k_row"], kw["v_row"], kw["do_row"], kw["dk_row"], kw["dv_row"])
    out += struct.pack("<6i", kw["q_head"], kw["k_head"], kw["v_head"], kw["do_head"], kw["dk_head"], kw["dv_head"])
    out += struct.pack("<6i", kw["sq"], kw["sk"], kw["h"], kw["ng"], kw["nh"], kw["group"])
    out += struct.pack("<ffiiQ", kw["c"], kw["scale"], kw["flags"], 0, 0)
    out += struct.pack("<10I", *kw["dec"])
    out += struct.pack("<ii", kw["n_items"], kw["grid"])
    assert len(out) == 272, len(out)
    return out


def reference(q, k, v, do, causal, scale):
    """float64 forward + backward; q, do (b, sq, h, d), k, v (b, sk, hk, d) -> lse (b, h, sq),
    D (b, h, sq), dk, dv (b, sk, h, d) per query head (not yet reduced over the group)"""
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    g = h // hk
    lse = np.full((b, h, sq), np.inf)
    dsum = np.zeros((b, h, sq))
    dk = np.zeros((b, sk, h, d))
    dv = np.zeros((b, sk, h, d))
    for bi in range(b):
        for hi in range(h):
            s = q[bi, :, hi] @ k[bi, :, hi // g].T * scale
            if causal:
                s = np.where(np.arange(sk)[None, :] > np.arange(sq)[:, None], -np.inf, s)
            m = np.max(s, axis=1, keepdims=True)
            m = np.where(np.isfinite(m), m, 0)
            p = np.exp(s - m)
            l = p.sum(axis=1, keepdims=True)
            with np.errstate(all="ignore"):
                lse[bi, hi] = np.where(l[:, 0] > 0, (m + np.log(l))[:, 0], np.inf)
                pn = np.where(l > 0, p / l, 0)
            o = pn @ v[bi, :, hi // g]
            dsum[bi, hi] = (do[bi, :, hi] * o).sum(axis=1)
            dp = do[bi, :, hi] @ v[bi, :, hi // g].T
            ds = pn * (dp - dsum[bi, hi][:, None])
            dv[bi, :, hi] = pn.T @ do[bi, :, hi]
            dk[bi, :, hi] = scale * ds.T @ q[bi, :, hi]
    return lse, dsum, dk, dv


def run(b=1, sq=200, sk=200, h=2, hk=1, causal=True, bf16=True, reduce=True, seed=0, text=None, verbose=True,
        grid=None, unit_c=False, lens=None, table=False, ver=1, order=None):
    """grid: workgroups of the persistent item loop (default: one per item); unit_c: the _c1 kernel
    (c = 1: scale = ln 2, the launch of a backward on the prescaled Q'); lens: varlen (unpadded,
    cu_seqlens_q = cu_seqlens_k from these lengths; b, sq, sk follow from them)"""
    if lens is not None:
        return run_varlen(lens, h, hk, causal, bf16, reduce, seed, text, verbose, grid, table, ver, order)
    D, BKN = DIMS[ver]
    rng = np.random.default_rng(seed)
    q = rng.standard_normal((b, sq, h, D)).astype(np.float32)
    k = rng.standard_normal((b, sk, hk, D)).astype(np.float32)
    v = rng.standard_normal((b, sk, hk, D)).astype(np.float32)
    do = rng.standard_normal((b, sq, h, D)).astype(np.float32)
    enc, dec = (f32_to_bf16, bf16_to_f32) if bf16 else (f32_to_f16, f16_to_f32)
    q16, k16, v16, do16 = (enc(x).astype(np.uint16) for x in (q, k, v, do))
    qf, kf, vf, dof = (dec(x).astype(np.float64) for x in (q16, k16, v16, do16))
    scale = np.log(2.0) if unit_c else D ** -0.5
    lse, dsum, dk_ref, dv_ref = reference(qf, kf, vf, dof, causal, scale)
    g = h // hk
    if reduce and g > 1:
        dk_ref = dk_ref.reshape(b, sk, hk, g, D).sum(axis=3)
        dv_ref = dv_ref.reshape(b, sk, hk, g, D).sum(axis=3)
    nh_out = hk if (reduce and g > 1) else h
    ng = (sq + 31) // 32 + 1
    lsed = np.zeros((b, h, ng, 64), np.float32)
    for bi in range(b):
        for hi in range(h):
            for r in range(sq):
                lsed[bi, hi, r // 32, r % 32] = np.float32(-lse[bi, hi, r] / np.float32(scale))
                lsed[bi, hi, r // 32, 32 + r % 32] = np.float32(-dsum[bi, hi, r])
    heap = Heap(64 << 20)
    aq, ak, av, ado = heap.put(q16), heap.put(k16), heap.put(v16), heap.put(do16)
    adk = heap.alloc(b * sk * nh_out * D * 2)
    adv = heap.alloc(b * sk * nh_out * D * 2)
    heap.get(adk, b * sk * nh_out * D * 2)[:] = 0xAB
    heap.get(adv, b * sk * nh_out * D * 2)[:] = 0xAB
    alsed = heap.put(lsed)
    nblk = (sk + BKN - 1) // BKN
    red = reduce and g > 1
    n_items = b * nh_out * nblk
    kw = dict(q=aq, k=ak, v=av, do=ado, dk=adk, dv=adv, lsed=alsed, sched=0, cuq=0, cuk=0,
              dec=dkdv_item_decode(b * nh_out, nh_out, 1 if red else g, nblk), n_items=n_items,
              grid=grid or n_items,
              q_batch=sq * h * D * 2, k_batch=sk * hk * D * 2, v_batch=sk * hk * D * 2, do_batch=sq * h * D * 2,
              dk_batch=sk * nh_out * D * 2, dv_batch=sk * nh_out * D * 2,
              q_row=h * D * 2, k_row=hk * D * 2, v_row=hk * D * 2, do_row=h * D * 2, dk_row=nh_out * D * 2,
              dv_row=nh_out * D * 2, q_head=D * 2, k_head=D * 2, v_head=D * 2, do_head=D * 2, dk_head=D * 2,
              dv_head=D * 2, sq=sq, sk=sk, h=h, ng=ng, nh=g if red else 1, group=g,
              c=1.0 if unit_c else float(np.float32(scale * 1.4426950408889634)), scale=float(np.float32(scale)), flags=2 if red else 0)
    akarg = heap.put(np.frombuffer(pack_args(**kw), dtype=np.uint8))
    text = text or asm_text(ver)
    name = f"{KINDS[ver][1]}_d{D}_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}{'_c1' if unit_c else ''}"
    emu = Emu(text, name, heap)
    emu.check_races(benign=[LRING[ver]])
    for L in range(grid or n_items):
        emu.run_wg(L, akarg, nwaves=KINDS[ver][2], order=order)
    RACES[:] = emu.races
    if verbose and emu.races:
        print("LDS races:", *emu.races[:10], sep="\n  ")
    dk = dec(heap.get(adk, b * sk * nh_out * D * 2).view(np.uint16)).reshape(b, sk, nh_out, D).astype(np.float64)
    dv = dec(heap.get(adv, b * sk * nh_out * D * 2).view(np.uint16)).reshape(b, sk, nh_out, D).astype(np.float64)
    ek = np.abs(dk - dk_ref).max() / max(np.abs(dk_ref).max(), 1e-9)
    ev = np.abs(dv - dv_ref).max() / max(np.abs(dv_ref).max(), 1e-9)
    if verbose:
        print(f"b={b} sq={sq} sk={sk} h={h} hk={hk} causal={causal} bf16={bf16} reduce={red}: "
              f"rel max|ddK| {ek:.3e} rel max|ddV| {ev:.3e} ({emu.count} instructions, {emu.mfma_count} MFMAs)")
    return ek, ev, dk, dk_ref, dv, dv_ref


def varlen_items(lens, nh, gdiv, rows, nlev, reverse):
    """the device-built work list (fa_fwd_asm.cpp varlen_items_kernel), restated: levels from the
    highest down, within a level the sequences with more blocks first, then heads; entries
    (bidb | head << 16, kvh | block << 16) after [count, 0]"""
    nb = [min((L + rows - 1) // rows, nlev) if L > 0 else 0 for L in lens]
    order = sorted(range(len(lens)), key=lambda s_: -nb[s_])
    out = []
    for lv in range(nlev - 1, -1, -1):
        for s_ in order:
            if nb[s_] > lv:
                for hd in range(nh):
                    blk = nb[s_] - 1 - lv if reverse else lv
                    out += [s_ | (hd << 16), (hd // gdiv) | (blk << 16)]
    return np.array([len(out) // 2, 0] + out, dtype=np.uint32)


def run_varlen(lens, h, hk, causal, bf16, reduce, seed, text, verbose, grid, table=False, ver=1, order=None):
    """varlen launch (flags bit 0 clear: row offsets from cu_seqlens): packed (total, heads, D);
    table: the items from the device-built list (flags bit 2, the persistent varlen launch)"""
    D, BKN = DIMS[ver]
    rng = np.random.default_rng(seed)
    b, total, mx = len(lens), sum(lens), max(lens)
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    q = rng.standard_normal((total, h, D)).astype(np.float32)
    k = rng.standard_normal((total, hk, D)).astype(np.float32)
    v = rng.standard_normal((total, hk, D)).astype(np.float32)
    do = rng.standard_normal((total, h, D)).astype(np.float32)
    enc, dec = (f32_to_bf16, bf16_to_f32) if bf16 else (f32_to_f16, f16_to_f32)
    q16, k16, v16, do16 = (enc(x).astype(np.uint16) for x in (q, k, v, do))
    qf, kf, vf, dof = (dec(x).astype(np.float64) for x in (q16, k16, v16, do16))
    scale = D ** -0.5
    g = h // hk
    red = reduce and g > 1
    nh_out = hk if red else h
    ng = (mx + 31) // 32 + 1
    lsed = np.zeros((b, h, ng, 64), np.float32)
    dk_ref = np.zeros((total, nh_out, D))
    dv_ref = np.zeros((total, nh_out, D))
    for bi, L in enumerate(lens):
        if L == 0:
            continue
        sl = slice(cu[bi], cu[bi + 1])
        lse, dsum, dkr, dvr = reference(qf[None, sl], kf[None, sl], vf[None, sl], dof[None, sl], causal, scale)
        if red:
            dkr = dkr.reshape(1, L, hk, g, D).sum(axis=3)
            dvr = dvr.reshape(1, L, hk, g, D).sum(axis=3)
        dk_ref[sl], dv_ref[sl] = dkr[0], dvr[0]
        for hi in range(h):
            for r in range(L):
                lsed[bi, hi, r // 32, r % 32] = np.float32(-lse[0, hi, r] / np.float32(scale))
                lsed[bi, hi, r // 32, 32 + r % 32] = np.float32(-dsum[0, hi, r])
    heap = Heap(64 << 20)
    aq, ak, av, ado = heap.put(q16), heap.put(k16), heap.put(v16), heap.put(do16)
    nbytes = total * nh_out * D * 2
    adk, adv = heap.alloc(nbytes), heap.alloc(nbytes)
    heap.get(adk, nbytes)[:] = 0xAB
    heap.get(adv, nbytes)[:] = 0xAB
    alsed = heap.put(lsed)
    acu = heap.put(cu)
    nblk = (mx + BKN - 1) // BKN
    n_items = b * nh_out * nblk
    asch = heap.put(varlen_items(lens, nh_out, 1 if red else g, BKN, nblk, True)) if table else 0
    kw = dict(q=aq, k=ak, v=av, do=ado, dk=adk, dv=adv, lsed=alsed, sched=asch, cuq=acu, cuk=acu,
              dec=dkdv_item_decode(b * nh_out, nh_out, 1 if red else g, nblk), n_items=n_items,
              grid=grid or n_items,
              q_batch=0, k_batch=0, v_batch=0, do_batch=0, dk_batch=0, dv_batch=0,
              q_row=h * D * 2, k_row=hk * D * 2, v_row=hk * D * 2, do_row=h * D * 2, dk_row=nh_out * D * 2,
              dv_row=nh_out * D * 2, q_head=D * 2, k_head=D * 2, v_head=D * 2, do_head=D * 2, dk_head=D * 2,
              dv_head=D * 2, sq=mx, sk=mx, h=h, ng=ng, nh=g if red else 1, group=g,
              c=float(np.float32(scale * 1.4426950408889634)), scale=float(np.float32(scale)),
              flags=(2 if red else 0) | (4 if table else 0))
    akarg = heap.put(np.frombuffer(pack_args(**kw), dtype=np.uint8))
    text = text or asm_text(ver)
    name = f"{KINDS[ver][1]}_d{D}_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}"
    emu = Emu(text, name, heap)
    emu.check_races(benign=[LRING[ver]])
    for L in range(grid or n_items):
        emu.run_wg(L, akarg, nwaves=KINDS[ver][2], order=order)
    RACES[:] = emu.races
    if verbose and emu.races:
        print("LDS races:", *emu.races[:10], sep="\n  ")
    dk = dec(heap.get(adk, nbytes).view(np.uint16)).reshape(total, nh_out, D).astype(np.float64)
    dv = dec(heap.get(adv, nbytes).view(np.uint16)).reshape(total, nh_out, D).astype(np.float64)
    ek = np.abs(dk - dk_ref).max() / max(np.abs(dk_ref).max(), 1e-9)
    ev = np.abs(dv - dv_ref).max() / max(np.abs(dv_ref).max(), 1e-9)
    if verbose:
        print(f"varlen {lens} h={h} hk={hk} causal={causal} bf16={bf16} reduce={red} grid={grid}: "
              f"rel max|ddK| {ek:.3e} rel max|ddV| {ev:.3e} ({emu.count} instructions)")
    return ek, ev, dk, dk_ref, dv, dv_ref


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=1)
    ap.add_argument("--sq", type=int, default=200)
    ap.add_argument("--sk", type=int, default=200)
    ap.add_argument("--h", type=int, default=2)
    ap.add_argument("--hk", type=int, default=1)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--fp16", action="store_true")
    ap.add_argument("--noreduce", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--v2", action="store_true", help="the two-waves-per-SIMD kernel (gen_bwd2.py)")
    ap.add_argument("--d64", action="store_true", help="the head-dim-64 kernel (gen_bwd64.py)")
    ap.add_argument("--reverse", action="store_true", help="run the waves last-to-first between barriers")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--c1", action="store_true")
    a = ap.parse_args()
    run(a.b, a.sq, a.sk, a.h, a.hk, not a.full, not a.fp16, not a.noreduce, a.seed, ver=2 if a.v2 else (64 if a.d64 else 1),
        order="reverse" if a.reverse else None, grid=a.grid, unit_c=a.c1)
