#!/usr/bin/env python3
"""Generates fa_dq_asm.s: the gfx950 FlashAttention-2 dQ kernel for head dim 128, written as a
hand-scheduled assembly kernel (one wave per SIMD); gen_dq64.py instantiates it at head dim 64.

    python3 gen_dq.py > fa_dq_asm.s

Algorithm: the dQ half of the reference's backward (csrc/flash_attn/src/flash_bwd_kernel.h:
compute_dq_dk_dv_1colblock, dS :897-906, dQ :948-1008) for one block of query rows, swept over every
key it can see:
    S^T = K Q^T,  P^T = exp2(c S^T - log2e LSE)   (-inf where the causal mask hides the key)
    dP^T = V dO^T,  dS^T = P^T o (dP^T - D)
    dQ^T += K^T dS^T                              (dQ = scale dQ^T^T at the end)
with LSE and D = rowsum(dO o O) per query row -- per lane: the query is the MFMA column.

MI355X structure: gen_bwd.py's (the dK / dV kernel) with the roles of the operands swapped:
  * workgroup = 4 waves x 64 query rows (q-blocks a and b of 32) = a 256-row block; each wave keeps
    its rows' operands and results in its 512 registers for the whole sweep:
      a[0:127] dQ^T (2 q-blocks x 4 d-tiles x 16), a[128:191] Q fragments, a[192:255] dO fragments
      (B operands of S^T = K Q^T and dP^T = V dO^T);
      v[0:127] S^T / dP^T tiles (two buffers x two q-blocks), v[128:159] packed dS^T (two buffers:
      the B operands of dQ^T), v[160:223] a ring of 16 A-operand fragments read from LDS;
  * the keys stream through LDS in 32-key subtiles (K and V, 16 KiB, a 9-slot ring) by LDS-DMA,
    6 subtiles ahead, one s_waitcnt + s_barrier per step of two subtiles;
  * phase p (48 MFMAs):  S^T, dP^T(p+1)  ||  dQ^T += ..(p-1)  and, in the gaps, the VALU of subtile p
    (P, dS and the dS pack of both q-blocks) and the LDS reads (K / V rows with ds_read_b128, K^T with
    ds_read_b64_tr_b16): each A fragment feeds the MFMAs of both q-blocks;
  * causal: the subtiles that reach past the block's first row run a MASKED step variant; keys past
    the causal end or seqlen_k read zero K / V (range-checked descriptors) and contribute nothing.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa import (ACCR, ACCW, BARRIER, BRANCH, DMA, LABEL, LDS, MFMA, PERM, RFL, SALU, SMEM, SOPP,  # noqa: E402
                 TRANS, VALU, VLOAD, VSTORE, WAIT, Inst, add_waits, ar, fix_hazards, item_decode_ops, item_pos_ops, label, nop, rtxt,
                 schedule, sr, vr)

import isa as _isa  # noqa: E402

# scheduling weights (round 4 A/B, profiles/r04/ab_sched_weights_r04.txt): an LDS read weighs 5 (a SALU op 3) issue
# cycles in the gap budget (2 before), spreading the reads over more MFMA gaps
_isa.apply_costs("LDS=5,SALU=3")
_isa.apply_costs(os.environ.get("FA_ISA_COST", ""))
_isa.apply_costs(os.environ.get("FA_GDQ_COST", ""))
D = 128
KS = D // 16            # k-steps of S^T / dP^T
NP = D // 32            # d-tiles of dQ^T
SUB = 32                # keys per subtile
BM = 256                # query rows per workgroup
KT = SUB * D * 2        # bytes of a K (or V) subtile = 8 KiB
SLOT = 2 * KT           # K | V
NS = 9
RING = NS * SLOT        # 147456
LDS_BYTES = RING
KQ = 6                  # K / V subtile s is DMA'd in step (s - KQ) / 2
PIECES = 4              # 1-KiB LDS-DMA pieces a wave issues per subtile (K halves 0 / 1, V halves 0 / 1)
# the end of step n-1 waits for the rows of subtiles <= 2n+3 (step n reads them, its last phase
# prefetching the first fragments of 2n+3); younger than K/V(2n+3) (issued in step n-2): the 8 of step n-1
VMCNT_STEP = 2 * PIECES

OPT_WIN = int(os.environ.get("FA_GDQ_WIN", "16"))
# (a read more than 16 MFMAs ahead would overwrite the ring slot (16 fragments) an earlier MFMA
# still reads: the scheduler orders fillers among themselves, the MFMA sequence only by earliest)
assert 2 <= OPT_WIN <= 16, "FA_GDQ_WIN must be within the 16-slot fragment ring"
OPT_LEAD = int(os.environ.get("FA_GDQ_LEAD", "2"))
OPT_OWAIT = int(os.environ.get("FA_GDQ_OWAIT", "23"))
OPT_DECBURST = os.environ.get("FA_GDQ_DECBURST") == "1"

# ---- AGPRs ----
def DQ(j, dt):
    return 64 * j + 16 * dt


def QF(j, ks):
    return 128 + 32 * j + 4 * ks


def OF(j, ks):
    return 192 + 32 * j + 4 * ks


# ---- VGPRs ----
def SB(par, j):
    return 32 * par + 16 * j


def DPB(par, j):
    return 64 + 32 * par + 16 * j


def DSP(par, j):
    return 128 + 16 * par + 8 * j


RG = 160
# CHAIN_S / CHAIN_D: the S^T / dP^T chains start from per-row constant blocks instead of zero --
# S' = S^T - LSE log2 e / c and dP' = dP^T - D -- so a score needs no v_fma before its exp (P =
# exp2(c S'), exp2(S') on the c = 1 kernels) and no v_sub before its dS multiply (dS = P dP').  d = 64
# (gen_dq64.py): both, the blocks in v[160:223] and the A-fragment ring in the AGPRs d = 64 leaves free
# (a[32:63], a[96:127]); d = 128: CHAIN_D with the ring cut to 8 slots (v[160:191]), -D in v[192:223]
CHAIN_S = False
# (d = 128 A/B, profiles/r06/ab_c{3,5}_dqcd_r06k.txt: dQ -0.9 % at C3, -0.8 % at C5; FA_GDQ_CHAIN_D=0 is the
# 16-slot ring without it)
CHAIN_D = os.environ.get("FA_GDQ_CHAIN_D", "1") == "1"
RING_FILE = "v"
RING_SLOTS = 8 if CHAIN_D else 16


def ring(f):
    if RING_FILE == "a":
        s = f % 16
        return (32 if s < 8 else 96) + 4 * (s % 8)
    return RG + 4 * (f % RING_SLOTS)


def NLCB(j):
    """(CHAIN_S) 16 copies of the q-block's -LSE log2 e / c: the S^T chain start"""
    return 160 + 16 * j


def NDB(j):
    """(CHAIN_D) 16 copies of the q-block's -D: the dP^T chain start"""
    return 192 + 16 * j


V_RB0, V_RB1, V_TB0, V_TB1 = 224, 225, 226, 227
V_KB0, V_KB1, V_VB0, V_VB1 = 228, 229, 230, 231
V_KV0, V_KV1 = 232, 233        # DMA voffsets (K and V share them: k_row == v_row), halves 0 / 1
V_NLC = (234, 235)             # -log2e LSE per q-block
V_D = (236, 237)               # D per q-block
V_LIM = (238, 239)             # mask limit base per q-block: the row's last key - 4 hh
V_LM = 240
V_NINF = 241
V_LANE = 242
V_QOFF = (243, 244)            # Q / dO row offsets (prologue), then dQ row offsets (epilogue)
V_OOFF = (245, 246)
V_TMP = 247                    # 247..255
NVGPR = 256

# ---- SGPRs ----
S_KD, S_VD = 4, 8              # K / V DMA cursors
S_QD, S_OD = 12, 16            # Q / dO (prologue), dQ (epilogue)
S_C = 20                       # scale log2 e
S_SCALE = 21
S_SROW, S_STR, S_SDMA = 22, 23, 24
S_W2K = 25
S_N, S_NLAST = 26, 27
S_MASK0 = 28                   # first masked step (causal), else a large value
S_KV32 = 29                    # 32 rows of K / V (bytes)
S_WAVE = 30
S_TMP = 31                     # 31..39
S_ROUND = 100                  # round r of the persistent item loop
S_ITEM = 101                   # the item index
NSGPR = 102

KARG_SIZE = 304
FUSE_OFF = 232   # DqAsmArgs: o, o_batch, o_row, o_head, lsed, lsed_ng, nrscale (flags bit 1: fused D)
QF_OFF = 272     # DqAsmArgs: qf, qf_batch, qf_row, qf_head, qc (flags bit 2: the Q fold, q_fold)
DEC_OFF = 184    # fa_params.h ItemDecode (40 bytes) after DqAsmArgs' 184
NITEMS_OFF = 224  # n_items, grid (persistent item loop)


class K:
    def __init__(self, bf16, causal, unit_c=False):
        """unit_c (CHAIN_S only): for launches with c = 1 (the folded backward): P = exp2(S') with no
        multiply"""
        self.bf16 = bf16
        self.causal = causal
        self.unit_c = unit_c
        assert CHAIN_S or not unit_c
        self.ty = "bf16" if bf16 else "f16"
        self.name = (f"fa_bwd_dq_asm_d{D}_{self.ty}_{'causal' if causal else 'full'}"   # (D: 128, or 64 via gen_dq64.py)
                     f"{'_c1' if unit_c else ''}")
        self.uid = 0

    def lab(self, s):
        self.uid += 1
        return f".L{self.name}_{s}_{self.uid}"

    # ------------------------------------------------------------------ MFMAs of a phase
    def mf(self, dst, a, b, first=False, c_src=None):
        """c_src: (file, register) of the chain's start block (its first MFMA reads C from there)"""
        dk, dr = dst
        regs = {"v": vr, "a": ar}
        d = regs[dk](dr, 16)
        if c_src is not None:
            c, cr = rtxt(c_src[0], c_src[1], 16), regs[c_src[0]](c_src[1], 16)
        else:
            c, cr = ("0", []) if first else (rtxt(dk, dr, 16), d)
        t = (f"v_mfma_f32_32x32x16_{self.ty} {rtxt(dk, dr, 16)}, {rtxt(a[0], a[1], 4)}, {rtxt(b[0], b[1], 4)}, {c}")
        rd = regs[a[0]](a[1], 4) + regs[b[0]](b[1], 4) + cr
        return Inst(t, MFMA, rd=rd, wr=d, rd_c=cr)

    def phase_frags(self, sdp, dq):
        """the A fragments of a phase in MFMA order: (kind, index) -- KS k-steps of S^T and of dP^T,
        2 NP (d-tile, key half) fragments of dQ^T: 8 each at d = 128, 4 at d = 64"""
        assert KS == 2 * NP
        if sdp and dq:
            return [(t, i) for i in range(KS) for t in ("S", "dQ", "dP")]
        if sdp:
            return [(t, i) for i in range(KS) for t in ("S", "dP")]
        return [("dQ", i) for i in range(KS)]

    def phase_mfmas(self, par, sdp, dq):
        """MFMA list (two per fragment: q-blocks a, b) and the fragment list; par = parity of the VALU
        subtile p: S^T / dP^T(p+1) write buffers 1 - par, dQ(p-1) reads packs 1 - par"""
        nb = 1 - par
        frags = self.phase_frags(sdp, dq)
        out = []
        for f, (t, i) in enumerate(frags):
            for j in range(2):
                if t == "S":
                    out.append(self.mf(("v", SB(nb, j)), (RING_FILE, ring(f)), ("a", QF(j, i)), first=(i == 0),
                                       c_src=("v", NLCB(j)) if CHAIN_S and i == 0 else None))
                elif t == "dP":
                    out.append(self.mf(("v", DPB(nb, j)), (RING_FILE, ring(f)), ("a", OF(j, i)), first=(i == 0),
                                       c_src=("v", NDB(j)) if CHAIN_D and i == 0 else None))
                else:
                    dt, kk = i // 2, i % 2
                    out.append(self.mf(("a", DQ(j, dt)), (RING_FILE, ring(f)), ("v", DSP(nb, j) + 4 * kk)))
        return out, frags

    def frag_reads(self, f, t, i, **kw):
        dst = ring(f)
        if t in ("S", "dP"):
            base = V_KB0 if i % 2 == 0 else V_KB1
            off = (i // 2) * 2048 + (KT if t == "dP" else 0)
            wr = (ar if RING_FILE == "a" else vr)(dst, 4)
            return [Inst(f"ds_read_b128 {rtxt(RING_FILE, dst, 4)}, v{base} offset:{off}", LDS, rd=vr(base), wr=wr, **kw)]
        dt, kk = i // 2, i % 2
        out = []
        for h in range(2):
            base = V_VB0 if h == 0 else V_VB1
            off = dt * 2048 + kk * 1024 + h * 512
            out.append(Inst(f"ds_read_b64_tr_b16 {rtxt(RING_FILE, dst + 2 * h, 2)}, v{base} offset:{off}", LDS,
                            rd=vr(base), wr=(ar if RING_FILE == "a" else vr)(dst + 2 * h, 2), **kw))
        return out

    def cvt(self, dst, s0, s1, **kw):
        return Inst(f"v_cvt_pk_{self.ty}_f32 v{dst}, v{s0}, v{s1}", VALU, rd=vr(s0) + vr(s1), wr=vr(dst), **kw)

    # ------------------------------------------------------------------ VALU of one subtile
    def valu_ops(self, par, masked, n0_add):
        """P^T and dS^T of subtile p (buffers par) for both q-blocks -> dS packs par.  Key base of the
        subtile = S_N * 64 + n0_add"""
        ops = []
        for j in range(2):
            S, DP, PK = SB(par, j), DPB(par, j), DSP(par, j)
            k0 = 200 * j
            if masked:
                # limit = q - 4 hh - key base; element g masked iff (g & 3) + 8 (g >> 2) > limit
                ops.append(Inst(f"s_lshl_b32 s{S_TMP + 8}, s{S_N}, 6", SALU, rd=sr(S_N), wr=sr(S_TMP + 8), key=k0))
                ops.append(Inst(f"v_subrev_u32 v{V_LM}, s{S_TMP + 8}, v{V_LIM[j]}", VALU, rd=sr(S_TMP + 8) + vr(V_LIM[j]),
                                wr=vr(V_LM), key=k0))
                if n0_add:
                    ops.append(Inst(f"v_subrev_u32 v{V_LM}, {n0_add}, v{V_LM}", VALU, rd=vr(V_LM), wr=vr(V_LM), key=k0))
            for g in range(16):
                if not CHAIN_S:
                    ops.append(Inst(f"v_fma_f32 v{S + g}, v{S + g}, s{S_C}, v{V_NLC[j]}", VALU,
                                    rd=vr(S + g) + sr(S_C) + vr(V_NLC[j]), wr=vr(S + g), key=k0 + 4 * g))
                elif not self.unit_c:      # S' = S^T - LSE log2 e / c: c S' is the log2-domain score
                    ops.append(Inst(f"v_mul_f32_e32 v{S + g}, s{S_C}, v{S + g}", VALU, rd=vr(S + g) + sr(S_C),
                                    wr=vr(S + g), key=k0 + 4 * g))
                if masked:
                    const = (g & 3) + 8 * (g >> 2)
                    ops.append(Inst(f"v_cmp_gt_i32_e32 vcc, {const}, v{V_LM}", VALU, rd=vr(V_LM), wr=[("vcc", 0)], key=k0 + 4 * g))
                    ops.append(Inst(f"v_cndmask_b32_e32 v{S + g}, v{S + g}, v{V_NINF}, vcc", VALU,
                                    rd=vr(S + g) + vr(V_NINF) + [("vcc", 0)], wr=vr(S + g), key=k0 + 4 * g))
                ops.append(Inst(f"v_exp_f32_e32 v{S + g}, v{S + g}", TRANS, rd=vr(S + g), wr=vr(S + g), key=k0 + 4 * g + 1))
                if not CHAIN_D:            # (CHAIN_D: dP' = dP^T - D already)
                    ops.append(Inst(f"v_sub_f32_e32 v{DP + g}, v{DP + g}, v{V_D[j]}", VALU, rd=vr(DP + g) + vr(V_D[j]),
                                    wr=vr(DP + g), key=k0 + 4 * g + 2))
                ops.append(Inst(f"v_mul_f32_e32 v{DP + g}, v{S + g}, v{DP + g}", VALU, rd=vr(S + g) + vr(DP + g),
                                wr=vr(DP + g), key=k0 + 4 * g + 3))
                if g % 2 == 1:
                    ops.append(self.cvt(PK + g // 2, DP + g - 1, DP + g, key=k0 + 4 * g + 3))
        return ops

    # ------------------------------------------------------------------ DMA of one subtile
    def dma_subtile(self, key=-50, eg=None):
        t = S_TMP
        I = Inst
        ops = [I(f"s_add_u32 s{t}, s{S_SDMA}, s{S_W2K}", SALU, rd=sr(S_SDMA) + sr(S_W2K), wr=sr(t) + [("scc", 0)], key=key)]
        # d = 128: the wave's 64-byte panel of both 16-row halves of K and of V; d = 64 (two panels):
        # one piece of K and one of V (panel w & 1, rows 16 (w >> 1): S_W2K and V_KV0 say which)
        pieces = (((V_KV0, S_KD, 0), (V_KV1, S_KD, 1024), (V_KV0, S_VD, KT), (V_KV1, S_VD, KT + 1024))
                  if PIECES == 4 else ((V_KV0, S_KD, 0), (V_KV0, S_VD, KT)))
        for jx, (voff, desc, add) in enumerate(pieces):
            e = None if eg is None else eg + 2 * jx
            ops.append(I(f"s_add_u32 m0, s{t}, {add}", SALU, rd=sr(t), wr=[("m0", 0), ("scc", 0)], key=key, earliest=e))
            ops.append(I(f"buffer_load_dwordx4 v{voff}, s[{desc}:{desc + 3}], 0 offen lds", DMA,
                         rd=vr(voff) + sr(desc, 4) + [("m0", 0)], key=key, earliest=e))
        for desc in (S_KD, S_VD):
            ops += [I(f"s_add_u32 s{desc}, s{desc}, s{S_KV32}", SALU, rd=sr(desc) + sr(S_KV32), wr=sr(desc) + [("scc", 0)], key=key + 1),
                    I(f"s_addc_u32 s{desc + 1}, s{desc + 1}, 0", SALU, rd=sr(desc + 1) + [("scc", 0)], wr=sr(desc + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_sub_u32 s{t + 1}, s{desc + 2}, s{S_KV32}", SALU, rd=sr(desc + 2) + sr(S_KV32), wr=sr(t + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_cselect_b32 s{desc + 2}, 0, s{t + 1}", SALU, rd=sr(t + 1) + [("scc", 0)], wr=sr(desc + 2), key=key + 1)]
        ops += self.slot_advance(S_SDMA, key + 1)
        return ops

    def slot_advance(self, reg, key=0):
        """reg = (reg + SLOT) mod RING"""
        t, u = S_TMP + 2, S_TMP + 3
        I = Inst
        return [I(f"s_add_u32 s{u}, s{reg}, {SLOT}", SALU, rd=sr(reg), wr=sr(u) + [("scc", 0)], key=key),
                I(f"s_sub_u32 s{t}, s{reg}, {RING - SLOT}", SALU, rd=sr(reg), wr=sr(t) + [("scc", 0)], key=key),
                I(f"s_cselect_b32 s{reg}, s{u}, s{t}", SALU, rd=sr(u) + sr(t) + [("scc", 0)], wr=sr(reg), key=key)]

    # ------------------------------------------------------------------ one phase
    def phase(self, par, sdp, dq, valu, masked, n0_add, dma, next_kind, tail_ops=None):
        mf, frags = self.phase_mfmas(par, sdp, dq)
        n = len(mf)
        fill = []
        for f, (t, i) in enumerate(frags):
            if f < 3:
                continue        # prefetched by the predecessor
            win = min(OPT_WIN, RING_SLOTS)
            eg = 2 * (f - win) + 1 if f >= win else None
            fill += self.frag_reads(f, t, i, key=-100 + f, earliest=eg, deadline=max(2 * f - OPT_LEAD, 0))
        if valu:
            fill += self.valu_ops(par, masked, n0_add)
        if dma:
            fill += self.dma_subtile(key=-40, eg=2)
        nxt = self.slot_advance(S_SROW, key=400) + self.slot_advance(S_STR, key=400)
        nxt += [Inst(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0), key=401),
                Inst(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1), key=401),
                Inst(f"v_add_u32_e32 v{V_VB0}, s{S_STR}, v{V_TB0}", VALU, rd=sr(S_STR) + vr(V_TB0), wr=vr(V_VB0), key=401),
                Inst(f"v_add_u32_e32 v{V_VB1}, s{S_STR}, v{V_TB1}", VALU, rd=sr(S_STR) + vr(V_TB1), wr=vr(V_VB1), key=401)]
        fill += nxt
        if next_kind is not None:
            nfr = self.phase_frags(next_kind in ("full", "sdp"), next_kind in ("full", "dq"))
            for f in range(3):
                t, i = nfr[f]
                users = [k for k in range(len(frags)) if k % RING_SLOTS == f % RING_SLOTS]
                eg = 2 * max(users) + 1 if users else None
                fill += self.frag_reads(f, t, i, key=600 + f, earliest=eg)
        if tail_ops:
            fill += tail_ops
        return schedule(mf, fill)

    def step(self, first, last, masked):
        a = self.phase(0, sdp=True, dq=not first, valu=True, masked=masked, n0_add=0, dma=True,
                       next_kind="dq" if last else "full")
        tail = [Inst(f"s_add_u32 s{S_N}, s{S_N}, 1", SALU, rd=sr(S_N), wr=sr(S_N) + [("scc", 0)], key=900)]
        b = self.phase(1, sdp=not last, dq=True, valu=True, masked=masked, n0_add=SUB, dma=True,
                       next_kind="dq" if last else "full", tail_ops=tail)
        return a + b

    def step_end(self):
        return [Inst(f"s_waitcnt vmcnt({VMCNT_STEP}) lgkmcnt(0)", WAIT), Inst("s_barrier", BARRIER)]

    def tail(self):
        mf, frags = self.phase_mfmas(0, False, True)     # par 0 -> packs 1 (subtile N-1 is odd)
        fill = []
        for f, (t, i) in enumerate(frags):
            if f < 3:
                continue
            fill += self.frag_reads(f, t, i, key=-100 + f, deadline=max(2 * f - OPT_LEAD, 0),
                                    earliest=2 * (f - RING_SLOTS) + 1 if f >= RING_SLOTS else None)
        return schedule(mf, fill)

    # ------------------------------------------------------------------ prologue
    def prologue(self):
        I = Inst
        ins = []
        # kernargs (DqAsmArgs, fa_bwd_asm.cpp) -> s56..s99
        ka = 56
        ins += [I(f"s_load_dwordx16 s[{ka}:{ka + 15}], s[0:1], 0x0", SMEM, rd=sr(0, 2), wr=sr(ka, 16)),
                I(f"s_load_dwordx16 s[{ka + 16}:{ka + 31}], s[0:1], 0x40", SMEM, rd=sr(0, 2), wr=sr(ka + 16, 16)),
                I(f"s_load_dwordx8 s[{ka + 32}:{ka + 39}], s[0:1], 0x80", SMEM, rd=sr(0, 2), wr=sr(ka + 32, 8)),
                I(f"s_load_dwordx4 s[{ka + 40}:{ka + 43}], s[0:1], 0xa0", SMEM, rd=sr(0, 2), wr=sr(ka + 40, 4)),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        # the c / scale kernargs and the work order (fa_params.h ItemDecode) into s[40:49] (free until
        # the geometry); FA_GDQ_DECBURST=1 (dev switch, off in the shipped build): with the kernargs,
        # one scalar round trip less
        late = [I(f"s_load_dwordx2 s[{S_C}:{S_SCALE}], s[0:1], 0xb0", SMEM, rd=sr(0, 2), wr=sr(S_C, 2)),
                I(f"s_load_dwordx8 s[40:47], s[0:1], {DEC_OFF}", SMEM),
                I(f"s_load_dwordx2 s[48:49], s[0:1], {DEC_OFF + 32}", SMEM)]
        if OPT_DECBURST:
            ins[-1:-1] = late
        P = lambda i: ka + i   # noqa: E731
        # dwords: 0 q, 2 k, 4 v, 6 dout, 8 dq, 10 lse, 12 dsum, 14 sched, 16 cu_q, 18 cu_k,
        # 20 q_batch, 22 kv_batch, 24 do_batch, 26 dq_batch (i64 bytes),
        # 28 q_row, 29 kv_row, 30 do_row, 31 dq_row, 32 q_head, 33 k_head, 34 v_head, 35 do_head, 36 dq_head,
        # 37 sq, 38 sk, 39 lse_pitch, 40 dsum_pitch, 41 h, 42 hk, 43 flags | c, scale follow at 0xb0
        Pq, Pk, Pv, Pdo, Pdq, Pl, Pds, Psch, Pcq, Pck = (P(2 * i) for i in range(10))
        Bq, Bkv, Bdo, Bdq = (P(20 + 2 * i) for i in range(4))
        Rq, Rkv, Rdo, Rdq, Hq, Hk, Hv, Hdo, Hdq = (P(28 + i) for i in range(9))
        SQ, SK, LP, DPt, NH, NHK, FLG = (P(37 + i) for i in range(7))
        T = [S_TMP + i for i in range(9)]
        ins += [I(f"v_mov_b32_e32 v1, s{S_WAVE}", VALU, rd=sr(S_WAVE), wr=vr(1))]     # (v0, v1: S^T tiles in the loop)
        if not OPT_DECBURST:
            ins = ins[:-1] + [late[0], ins[-1]] + late[1:] + [I("s_waitcnt lgkmcnt(0)", WAIT)]
        BIDB, HEAD, KVH, MB = S_N, S_NLAST, S_MASK0, S_KV32     # temporaries until the loop state
        ins += item_decode_ops(L=S_ITEM, M=40, pa=T[1], pb=T[3], t=T[5], u=T[6], o_blk=MB, reverse=True)
        ins += [I(f"s_mov_b32 s{BIDB}, s{T[3]}", SALU), I(f"s_mov_b32 s{HEAD}, s{T[6]}", SALU),
                I(f"s_mov_b32 s{KVH}, s{T[1]}", SALU)]
        # varlen geometry (block_info.h:14-31): byte offsets of row 0 of this sequence (Q-side: Q, dO,
        # dQ; K-side: K and V share it, k_row == v_row and the batch strides are equal)
        QOFF, DOOFF, DQOFF, KOFF = (40, 41), (42, 43), (44, 45), (46, 47)

        def mul64(dst, a32, b32):
            return [I(f"s_mul_i32 s{dst[0]}, s{a32}, s{b32}", SALU, rd=sr(a32) + sr(b32), wr=sr(dst[0])),
                    I(f"s_mul_hi_u32 s{dst[1]}, s{a32}, s{b32}", SALU, rd=sr(a32) + sr(b32), wr=sr(dst[1]))]

        def mul64_i64(dst, a32, b64):
            return [I(f"s_mul_i32 s{dst[0]}, s{a32}, s{b64}", SALU, rd=sr(a32) + sr(b64), wr=sr(dst[0])),
                    I(f"s_mul_hi_u32 s{dst[1]}, s{a32}, s{b64}", SALU, rd=sr(a32) + sr(b64), wr=sr(dst[1])),
                    I(f"s_mul_i32 s{T[0]}, s{a32}, s{b64 + 1}", SALU, rd=sr(a32) + sr(b64 + 1), wr=sr(T[0])),
                    I(f"s_add_u32 s{dst[1]}, s{dst[1]}, s{T[0]}", SALU, rd=sr(dst[1]) + sr(T[0]), wr=sr(dst[1]))]

        # varlen: the cu_seqlens loads of every part are issued together and waited for once (one
        # scalar-memory round trip per item start instead of one per part)
        parts = ((Pcq, Bq, Rq, QOFF, SQ), (Pcq, Bdo, Rdo, DOOFF, None),
                 (Pcq, Bdq, Rdq, DQOFF, None), (Pck, Bkv, Rkv, KOFF, SK))
        ins += [I(f"s_lshl_b32 s{T[1]}, s{BIDB}, 2", SALU, rd=sr(BIDB), wr=sr(T[1]))]
        for cu, bstride, rstride, off, seq in parts:
            lf = self.lab("nold")
            ins += [I(f"s_cmp_eq_u64 s[{cu}:{cu + 1}], 0", SALU, rd=sr(cu, 2), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH),
                    I(f"s_load_dwordx2 s[{off[0]}:{off[1]}], s[{cu}:{cu + 1}], s{T[1]}", SMEM, rd=sr(cu, 2) + sr(T[1]), wr=sr(off[0], 2)),
                    label(lf)]
        ins += [I("s_waitcnt lgkmcnt(0)", WAIT)]
        for cu, bstride, rstride, off, seq in parts:
            lf, ld = self.lab("fixed"), self.lab("done")
            ins += [I(f"s_cmp_eq_u64 s[{cu}:{cu + 1}], 0", SALU, rd=sr(cu, 2), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH)]
            if seq is not None:
                ins += [I(f"s_sub_u32 s{seq}, s{off[1]}, s{off[0]}", SALU, rd=sr(off[0], 2), wr=sr(seq))]
            ins += [I(f"s_bitcmp1_b32 s{FLG}, 0", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH),
                    I(f"s_mov_b32 s{T[1]}, s{off[0]}", SALU, rd=sr(off[0]), wr=sr(T[1]))]
            ins += mul64(off, T[1], rstride)
            ins += [I(f"s_branch {ld}", BRANCH), label(lf)]
            ins += mul64_i64(off, BIDB, bstride)
            ins += [label(ld)]
        # m0 = 256 mb; exit when m0 >= sq
        M0R, NROW = T[4], T[5]
        ins += [I(f"s_lshl_b32 s{M0R}, s{MB}, 8", SALU, rd=sr(MB), wr=sr(M0R)),
                I(f"s_cmp_ge_i32 s{M0R}, s{SQ}", SALU, rd=sr(M0R) + sr(SQ), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {self.lab_next}", BRANCH),
                I(f"s_sub_u32 s{NROW}, s{SQ}, s{M0R}", SALU, rd=sr(SQ) + sr(M0R), wr=sr(NROW)),
                I(f"s_min_u32 s{NROW}, s{NROW}, {BM}", SALU, rd=sr(NROW), wr=sr(NROW))]

        def desc(dst4, ptr, off64, head, hstride, rows, rstride, nrec):
            """dst4 = descriptor of ptr + off64 + head hstride + rows rstride; nrec: list of records ops"""
            o = [I(f"s_mul_i32 s{T[0]}, s{head}, s{hstride}", SALU, rd=sr(head) + sr(hstride), wr=sr(T[0])),
                 I(f"s_mul_hi_u32 s{T[1]}, s{head}, s{hstride}", SALU, rd=sr(head) + sr(hstride), wr=sr(T[1])),
                 I(f"s_add_u32 s{dst4}, s{ptr}, s{T[0]}", SALU, rd=sr(ptr) + sr(T[0]), wr=sr(dst4) + [("scc", 0)]),
                 I(f"s_addc_u32 s{dst4 + 1}, s{ptr + 1}, s{T[1]}", SALU, rd=sr(ptr + 1) + sr(T[1]) + [("scc", 0)], wr=sr(dst4 + 1)),
                 I(f"s_add_u32 s{dst4}, s{dst4}, s{off64[0]}", SALU, rd=sr(dst4) + sr(off64[0]), wr=sr(dst4) + [("scc", 0)]),
                 I(f"s_addc_u32 s{dst4 + 1}, s{dst4 + 1}, s{off64[1]}", SALU, rd=sr(dst4 + 1) + sr(off64[1]) + [("scc", 0)], wr=sr(dst4 + 1))]
            if rows is not None:
                o += [I(f"s_mul_i32 s{T[0]}, s{rows}, s{rstride}", SALU, rd=sr(rows) + sr(rstride), wr=sr(T[0])),
                      I(f"s_mul_hi_u32 s{T[1]}, s{rows}, s{rstride}", SALU, rd=sr(rows) + sr(rstride), wr=sr(T[1])),
                      I(f"s_add_u32 s{dst4}, s{dst4}, s{T[0]}", SALU, rd=sr(dst4) + sr(T[0]), wr=sr(dst4) + [("scc", 0)]),
                      I(f"s_addc_u32 s{dst4 + 1}, s{dst4 + 1}, s{T[1]}", SALU, rd=sr(dst4 + 1) + sr(T[1]) + [("scc", 0)], wr=sr(dst4 + 1))]
            o += [I(f"s_and_b32 s{dst4 + 1}, s{dst4 + 1}, 0xffff", SALU, rd=sr(dst4 + 1), wr=sr(dst4 + 1))]
            o += nrec
            o += [I(f"s_mov_b32 s{dst4 + 3}, 0x20000", SALU, wr=sr(dst4 + 3))]
            return o

        # Q / dO: rows [m0, m0 + nrow) of this sequence and head
        ins += desc(S_QD, Pq, QOFF, HEAD, Hq, M0R, Rq, [I(f"s_mul_i32 s{S_QD + 2}, s{NROW}, s{Rq}", SALU, rd=sr(NROW) + sr(Rq), wr=sr(S_QD + 2))])
        ins += desc(S_OD, Pdo, DOOFF, HEAD, Hdo, M0R, Rdo, [I(f"s_mul_i32 s{S_OD + 2}, s{NROW}, s{Rdo}", SALU, rd=sr(NROW) + sr(Rdo), wr=sr(S_OD + 2))])
        # keys of the sweep: n_end = causal ? min(sk, m0 + 256) : sk (K / V read zero past it)
        NEND = T[6]
        if self.causal:
            ins += [I(f"s_add_u32 s{NEND}, s{M0R}, {BM}", SALU, rd=sr(M0R), wr=sr(NEND)),
                    I(f"s_min_i32 s{NEND}, s{NEND}, s{SK}", SALU, rd=sr(NEND) + sr(SK), wr=sr(NEND))]
        else:
            ins += [I(f"s_mov_b32 s{NEND}, s{SK}", SALU, rd=sr(SK), wr=sr(NEND))]
        ins += [I(f"s_max_i32 s{NEND}, s{NEND}, 0", SALU, rd=sr(NEND), wr=sr(NEND))]
        ZERO = T[7]
        ins += [I(f"s_mov_b32 s{ZERO}, 0", SALU, wr=sr(ZERO))]
        ins += desc(S_KD, Pk, KOFF, KVH, Hk, None, None, [I(f"s_mul_i32 s{S_KD + 2}, s{NEND}, s{Rkv}", SALU, rd=sr(NEND) + sr(Rkv), wr=sr(S_KD + 2))])
        ins += desc(S_VD, Pv, KOFF, KVH, Hv, None, None, [I(f"s_mul_i32 s{S_VD + 2}, s{NEND}, s{Rkv}", SALU, rd=sr(NEND) + sr(Rkv), wr=sr(S_VD + 2))])
        # (flags bit 2, the Q fold) the Q' output of q_fold: descriptor s[56:59] (the q / k / v / dout
        # pointers are consumed), rows [m0, m0 + nrow) of this sequence and head in the compact layout
        # (row 0 at cu_q[bidb] qf_row varlen, bidb qf_batch otherwise); qf_row in s60, qc in s62
        l_noqf, l_qfx, l_qfd = self.lab("noqf"), self.lab("qffixed"), self.lab("qfdone")
        ins += [I(f"s_bitcmp1_b32 s{FLG}, 2", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                I(f"s_cbranch_scc0 {l_noqf}", BRANCH),
                I(f"s_load_dwordx8 s[56:63], s[0:1], {QF_OFF}", SMEM, rd=sr(0, 2), wr=sr(56, 8)),
                I("s_waitcnt lgkmcnt(0)", WAIT),
                I(f"s_cmp_eq_u64 s[{Pcq}:{Pcq + 1}], 0", SALU, rd=sr(Pcq, 2), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_qfx}", BRANCH),
                I(f"s_bitcmp1_b32 s{FLG}, 0", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_qfx}", BRANCH),
                I(f"s_lshl_b32 s{T[2]}, s{BIDB}, 2", SALU, rd=sr(BIDB), wr=sr(T[2])),
                I(f"s_load_dword s{T[2]}, s[{Pcq}:{Pcq + 1}], s{T[2]}", SMEM, rd=sr(Pcq, 2) + sr(T[2]), wr=sr(T[2])),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        ins += mul64((58, 59), T[2], 60)
        ins += [I(f"s_branch {l_qfd}", BRANCH), label(l_qfx)]
        ins += mul64_i64((T[1], T[2]), BIDB, 58)
        ins += [I(f"s_mov_b32 s58, s{T[1]}", SALU), I(f"s_mov_b32 s59, s{T[2]}", SALU), label(l_qfd)]
        ins += desc(56, 56, (58, 59), HEAD, 61, M0R, 60, [I(f"s_mul_i32 s58, s{NROW}, s60", SALU, rd=sr(NROW) + sr(60), wr=sr(58))])
        ins += [label(l_noqf)]
        # steps: subtiles ns = ceil(n_end / 32) rounded up to even; N / 2 steps
        ins += [I(f"s_add_u32 s{T[0]}, s{NEND}, {2 * SUB - 1}", SALU, rd=sr(NEND), wr=sr(T[0])),
                I(f"s_lshr_b32 s{T[0]}, s{T[0]}, 6", SALU, rd=sr(T[0]), wr=sr(T[0])),          # steps
                I(f"s_sub_i32 s{T[8]}, s{T[0]}, 1", SALU, rd=sr(T[0]), wr=sr(T[8]))]           # last step
        # first masked step: causal, the first with keys past the block's first row (m0 / 64); and the
        # step holding key seqlen_k, whose keys past it read zero K / V but would still get P > 0
        # (exp2(-LSE log2 e)): with fp16 dS packs a P dS past 65504 turns into inf and 0 x inf into NaN
        # in dQ^T += K^T dS^T, so the masked step zeroes them (sk / 64 > the last step when sk % 64 == 0)
        if self.causal:
            ins += [I(f"s_lshr_b32 s{T[3]}, s{M0R}, 6", SALU, rd=sr(M0R), wr=sr(T[3]))]
        else:
            ins += [I(f"s_mov_b32 s{T[3]}, 0x7fffffff", SALU, wr=sr(T[3]))]
        ins += [I(f"s_lshr_b32 s{T[2]}, s{SK}, 6", SALU, rd=sr(SK), wr=sr(T[2])),
                I(f"s_min_u32 s{T[3]}, s{T[3]}, s{T[2]}", SALU, rd=sr(T[3]) + sr(T[2]), wr=sr(T[3]))]
        # ---- per-lane values: rows, LSE / D, offsets ----
        r_, hh = V_TMP, V_TMP + 1
        x = V_TMP + 2
        ins += [I(f"v_and_b32_e32 v{r_}, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(r_)),
                I(f"v_lshrrev_b32_e32 v{hh}, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(hh))]
        # LSE / D descriptors: lse + ((bidb h + head) lse_pitch + m0) * 4 (records 4 nrow), the same for D
        LD, DD = 48, 52          # borrowed from the kernarg block (dead by now): q_batch.. / kv_batch..
        for dd, ptr, pitch in ((LD, Pl, LP), (DD, Pds, DPt)):
            ins += [I(f"s_mul_i32 s{T[0]}, s{BIDB}, s{NH}", SALU, rd=sr(BIDB) + sr(NH), wr=sr(T[0])),
                    I(f"s_add_u32 s{T[0]}, s{T[0]}, s{HEAD}", SALU, rd=sr(T[0]) + sr(HEAD), wr=sr(T[0])),
                    I(f"s_mul_i32 s{T[1]}, s{T[0]}, s{pitch}", SALU, rd=sr(T[0]) + sr(pitch), wr=sr(T[1])),
                    I(f"s_mul_hi_u32 s{T[2]}, s{T[0]}, s{pitch}", SALU, rd=sr(T[0]) + sr(pitch), wr=sr(T[2])),
                    I(f"s_add_u32 s{T[1]}, s{T[1]}, s{M0R}", SALU, rd=sr(T[1]) + sr(M0R), wr=sr(T[1]) + [("scc", 0)]),
                    I(f"s_addc_u32 s{T[2]}, s{T[2]}, 0", SALU, rd=sr(T[2]) + [("scc", 0)], wr=sr(T[2])),
                    I(f"s_lshl_b64 s[{T[1]}:{T[2]}], s[{T[1]}:{T[2]}], 2", SALU, rd=sr(T[1], 2), wr=sr(T[1], 2)),
                    I(f"s_add_u32 s{dd}, s{ptr}, s{T[1]}", SALU, rd=sr(ptr) + sr(T[1]), wr=sr(dd) + [("scc", 0)]),
                    I(f"s_addc_u32 s{dd + 1}, s{ptr + 1}, s{T[2]}", SALU, rd=sr(ptr + 1) + sr(T[2]) + [("scc", 0)], wr=sr(dd + 1)),
                    I(f"s_and_b32 s{dd + 1}, s{dd + 1}, 0xffff", SALU, rd=sr(dd + 1), wr=sr(dd + 1)),
                    I(f"s_lshl_b32 s{dd + 2}, s{NROW}, 2", SALU, rd=sr(NROW), wr=sr(dd + 2)),
                    I(f"s_mov_b32 s{dd + 3}, 0x20000", SALU, wr=sr(dd + 3))]
        # rows of the wave: 64 w + 32 j + r
        ins += [I(f"s_sub_i32 s{T[2]}, s{SK}, 1", SALU, rd=sr(SK), wr=sr(T[2]))]        # the last key
        for j in range(2):
            ins += [I(f"v_lshl_add_u32 v{x}, v1, 6, v{r_}", VALU, rd=vr(1) + vr(r_), wr=vr(x)),
                    I(f"v_add_u32_e32 v{x}, {32 * j}, v{x}", VALU, rd=vr(x), wr=vr(x)),
                    I(f"v_lshlrev_b32_e32 v{x + 1}, 2, v{x}", VALU, rd=vr(x), wr=vr(x + 1)),
                    I(f"buffer_load_dword v{V_NLC[j]}, v{x + 1}, s[{LD}:{LD + 3}], 0 offen", VLOAD,
                      rd=vr(x + 1) + sr(LD, 4), wr=vr(V_NLC[j])),
                    I(f"buffer_load_dword v{V_D[j]}, v{x + 1}, s[{DD}:{DD + 3}], 0 offen", VLOAD,
                      rd=vr(x + 1) + sr(DD, 4), wr=vr(V_D[j])),
                    # Q / dO row offsets: row * row_stride + 16 hh
                    I(f"v_mul_lo_u32 v{V_QOFF[j]}, v{x}, s{Rq}", VALU, rd=vr(x) + sr(Rq), wr=vr(V_QOFF[j])),
                    I(f"v_lshl_add_u32 v{V_QOFF[j]}, v{hh}, 4, v{V_QOFF[j]}", VALU, rd=vr(hh) + vr(V_QOFF[j]), wr=vr(V_QOFF[j])),
                    I(f"v_mul_lo_u32 v{V_OOFF[j]}, v{x}, s{Rdo}", VALU, rd=vr(x) + sr(Rdo), wr=vr(V_OOFF[j])),
                    I(f"v_lshl_add_u32 v{V_OOFF[j]}, v{hh}, 4, v{V_OOFF[j]}", VALU, rd=vr(hh) + vr(V_OOFF[j]), wr=vr(V_OOFF[j])),
                    # mask limit base: the row's last key - 4 hh: min(q, sk - 1) causal (q = m0 + row), sk - 1 not
                    (I(f"v_add_u32_e32 v{V_LIM[j]}, s{M0R}, v{x}", VALU, rd=sr(M0R) + vr(x), wr=vr(V_LIM[j])) if self.causal
                     else I(f"v_mov_b32_e32 v{V_LIM[j]}, s{T[2]}", VALU, rd=sr(T[2]), wr=vr(V_LIM[j]))),
                    ] + ([I(f"v_min_i32_e32 v{V_LIM[j]}, s{T[2]}, v{V_LIM[j]}", VALU, rd=sr(T[2]) + vr(V_LIM[j]), wr=vr(V_LIM[j]))]
                         if self.causal else []) + [
                    I(f"v_lshlrev_b32_e32 v{x + 2}, 2, v{hh}", VALU, rd=vr(hh), wr=vr(x + 2)),
                    I(f"v_sub_u32_e32 v{V_LIM[j]}, v{V_LIM[j]}, v{x + 2}", VALU, rd=vr(V_LIM[j]) + vr(x + 2), wr=vr(V_LIM[j]))]
        # Q / dO fragments into AGPRs: lane holds row[16 ks + 8 hh .. +7]
        for j in range(2):
            for ks in range(KS):
                ins.append(I(f"buffer_load_dwordx4 {rtxt('a', QF(j, ks), 4)}, v{V_QOFF[j]}, s[{S_QD}:{S_QD + 3}], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(V_QOFF[j]) + sr(S_QD, 4), wr=ar(QF(j, ks), 4)))
        for j in range(2):
            for ks in range(KS):
                ins.append(I(f"buffer_load_dwordx4 {rtxt('a', OF(j, ks), 4)}, v{V_OOFF[j]}, s[{S_OD}:{S_OD + 3}], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(V_OOFF[j]) + sr(S_OD, 4), wr=ar(OF(j, ks), 4)))
        # dQ row offsets (epilogue) replace the Q / dO ones once those loads are issued
        for j in range(2):
            ins += [I(f"v_lshl_add_u32 v{x}, v1, 6, v{r_}", VALU, rd=vr(1) + vr(r_), wr=vr(x)),
                    I(f"v_add_u32_e32 v{x}, {32 * j}, v{x}", VALU, rd=vr(x), wr=vr(x)),
                    I(f"v_mul_lo_u32 v{x + 3}, v{x}, s{Rdq}", VALU, rd=vr(x) + sr(Rdq), wr=vr(x + 3)),
                    I(f"v_lshl_add_u32 v{V_QOFF[j]}, v{hh}, 4, v{x + 3}", VALU, rd=vr(hh) + vr(x + 3), wr=vr(V_QOFF[j]))]
        # dQ descriptor (S_QD is still read by the loads above: the epilogue builds it in S_OD... kept
        # in SGPRs nothing rewrites: 92..95)
        ins += desc(92, Pdq, DQOFF, HEAD, Hdq, M0R, Rdq, [I(f"s_mul_i32 s94, s{NROW}, s{Rdq}", SALU, rd=sr(NROW) + sr(Rdq), wr=sr(94))])
        # (flags bit 1, knob 8: bwd_pre fused) O fragments for D = rowsum(dO o O).  O descriptor in
        # s[16:19] (the dO loads are issued); the dK/dV scratch descriptor in s[12:15] (the Q loads are
        # issued); kernargs o, o_batch, o_row, o_head, lsed in s[40:47] (the row offsets are consumed),
        # lsed_ng, -1 / scale in s[48:49] (the LSE descriptor's loads are issued; s49 lives to fused_d)
        l_nof = self.lab("nofuse")
        Po, Bo, Ro, Ho, Plsed, NG = 40, 42, 44, 45, 46, 48
        OOFF = (18, 19)
        ins += [I(f"s_bitcmp1_b32 s{FLG}, 1", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                I(f"s_cbranch_scc0 {l_nof}", BRANCH),
                I(f"s_load_dwordx8 s[40:47], s[0:1], {FUSE_OFF}", SMEM, rd=sr(0, 2), wr=sr(40, 8)),
                I(f"s_load_dwordx2 s[48:49], s[0:1], {FUSE_OFF + 32}", SMEM, rd=sr(0, 2), wr=sr(48, 2)),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        lf, ld = self.lab("ofixed"), self.lab("odone")
        ins += [I(f"s_cmp_eq_u64 s[{Pcq}:{Pcq + 1}], 0", SALU, rd=sr(Pcq, 2), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {lf}", BRANCH),
                I(f"s_bitcmp1_b32 s{FLG}, 0", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {lf}", BRANCH),
                I(f"s_lshl_b32 s{T[2]}, s{BIDB}, 2", SALU, rd=sr(BIDB), wr=sr(T[2])),
                I(f"s_load_dword s{T[2]}, s[{Pcq}:{Pcq + 1}], s{T[2]}", SMEM, rd=sr(Pcq, 2) + sr(T[2]), wr=sr(T[2])),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        ins += mul64(OOFF, T[2], Ro)
        ins += [I(f"s_branch {ld}", BRANCH), label(lf)]
        ins += mul64_i64(OOFF, BIDB, Bo)
        ins += [label(ld)]
        ins += desc(16, Po, OOFF, HEAD, Ho, M0R, Ro, [I(f"s_mul_i32 s18, s{NROW}, s{Ro}", SALU, rd=sr(NROW) + sr(Ro), wr=sr(18))])
        # lsed + ((bidb h + head) ng) 256 + m0 8 (the item's first group), records ng 256 - m0 8
        ins += [I(f"s_mul_i32 s{T[0]}, s{BIDB}, s{NH}", SALU, rd=sr(BIDB) + sr(NH), wr=sr(T[0])),
                I(f"s_add_u32 s{T[0]}, s{T[0]}, s{HEAD}", SALU, rd=sr(T[0]) + sr(HEAD), wr=sr(T[0])),
                I(f"s_mul_i32 s{T[0]}, s{T[0]}, s{NG}", SALU, rd=sr(T[0]) + sr(NG), wr=sr(T[0])),
                I(f"s_lshr_b32 s{T[1]}, s{T[0]}, 24", SALU, rd=sr(T[0]), wr=sr(T[1])),
                I(f"s_lshl_b32 s{T[0]}, s{T[0]}, 8", SALU, rd=sr(T[0]), wr=sr(T[0])),
                I(f"s_add_u32 s12, s{Plsed}, s{T[0]}", SALU, rd=sr(Plsed) + sr(T[0]), wr=sr(12) + [("scc", 0)]),
                I(f"s_addc_u32 s13, s{Plsed + 1}, s{T[1]}", SALU, rd=sr(Plsed + 1) + sr(T[1]) + [("scc", 0)], wr=sr(13) + [("scc", 0)]),
                I(f"s_lshl_b32 s{T[0]}, s{M0R}, 3", SALU, rd=sr(M0R), wr=sr(T[0])),
                I(f"s_add_u32 s12, s12, s{T[0]}", SALU, rd=sr(12) + sr(T[0]), wr=sr(12) + [("scc", 0)]),
                I("s_addc_u32 s13, s13, 0", SALU, rd=sr(13) + [("scc", 0)], wr=sr(13)),
                I("s_and_b32 s13, s13, 0xffff", SALU, rd=sr(13), wr=sr(13)),
                I(f"s_lshl_b32 s14, s{NG}, 8", SALU, rd=sr(NG), wr=sr(14)),
                I(f"s_sub_u32 s14, s14, s{T[0]}", SALU, rd=sr(14) + sr(T[0]), wr=sr(14)),
                I("s_mov_b32 s15, 0x20000", SALU, wr=sr(15))]
        # O fragments into v[64 + 32 j + 4 ks ..] (the dP^T tiles, free until phase -1); lane rows as
        # the Q / dO loads', with o_row
        for j in range(2):
            ins += [I(f"v_lshl_add_u32 v{x}, v1, 6, v{r_}", VALU, rd=vr(1) + vr(r_), wr=vr(x)),
                    I(f"v_add_u32_e32 v{x}, {32 * j}, v{x}", VALU, rd=vr(x), wr=vr(x)),
                    I(f"v_mul_lo_u32 v{x + 1 + j}, v{x}, s{Ro}", VALU, rd=vr(x) + sr(Ro), wr=vr(x + 1 + j)),
                    I(f"v_lshl_add_u32 v{x + 1 + j}, v{hh}, 4, v{x + 1 + j}", VALU, rd=vr(hh) + vr(x + 1 + j), wr=vr(x + 1 + j))]
        # the vector memory counter holds 63: LSE / D (4), Q (16), dO (16) are in flight, the O loads (16)
        # and the first 6 K / V subtiles (24) follow -- at most 23 of the first 36 may be outstanding
        ins.append(I(f"s_waitcnt vmcnt({OPT_OWAIT})", WAIT))
        for j in range(2):
            for ks in range(KS):
                ins.append(I(f"buffer_load_dwordx4 {rtxt('v', 64 + 32 * j + 4 * ks, 4)}, v{x + 1 + j}, s[16:19], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(x + 1 + j) + sr(16, 4), wr=vr(64 + 32 * j + 4 * ks, 4)))
        ins += [label(l_nof)]
        # LDS lane bases (as gen_fwd.py)
        ins += [I(f"v_bfe_u32 v{x}, v{r_}, 2, 2", VALU, rd=vr(r_), wr=vr(x)),
                I(f"v_xor_b32_e32 v{x + 1}, v{hh}, v{x}", VALU, rd=vr(hh) + vr(x), wr=vr(x + 1)),
                I(f"v_lshlrev_b32_e32 v{x + 2}, 6, v{r_}", VALU, rd=vr(r_), wr=vr(x + 2)),
                I(f"v_lshl_add_u32 v{V_RB0}, v{x + 1}, 4, v{x + 2}", VALU, rd=vr(x + 1) + vr(x + 2), wr=vr(V_RB0)),
                I(f"v_add_u32_e32 v{x + 1}, 2, v{hh}", VALU, rd=vr(hh), wr=vr(x + 1)),
                I(f"v_xor_b32_e32 v{x + 1}, v{x + 1}, v{x}", VALU, rd=vr(x + 1) + vr(x), wr=vr(x + 1)),
                I(f"v_lshl_add_u32 v{V_RB1}, v{x + 1}, 4, v{x + 2}", VALU, rd=vr(x + 1) + vr(x + 2), wr=vr(V_RB1))]
        ins += [I(f"v_and_b32_e32 v{x}, 15, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x)),             # i
                I(f"v_lshrrev_b32_e32 v{x + 1}, 2, v{x}", VALU, rd=vr(x), wr=vr(x + 1)),            # q
                I(f"v_and_b32_e32 v{x + 2}, 3, v{x}", VALU, rd=vr(x), wr=vr(x + 2)),                # pp
                I(f"v_lshrrev_b32_e32 v{x + 3}, 4, v{r_}", VALU, rd=vr(r_), wr=vr(x + 3)),          # r >> 4
                I(f"v_lshrrev_b32_e32 v{x + 4}, 1, v{x + 2}", VALU, rd=vr(x + 2), wr=vr(x + 4)),    # pp >> 1
                I(f"v_lshl_add_u32 v{x + 3}, v{x + 3}, 1, v{x + 4}", VALU, rd=vr(x + 3) + vr(x + 4), wr=vr(x + 3)),   # trc
                I(f"v_lshl_add_u32 v{x + 4}, v{hh}, 2, v{x + 1}", VALU, rd=vr(hh) + vr(x + 1), wr=vr(x + 4)),      # 4 hh + q
                I(f"v_lshlrev_b32_e32 v{x + 4}, 6, v{x + 4}", VALU, rd=vr(x + 4), wr=vr(x + 4)),
                I(f"v_and_b32_e32 v{x + 5}, 1, v{x + 2}", VALU, rd=vr(x + 2), wr=vr(x + 5)),
                I(f"v_lshl_add_u32 v{x + 4}, v{x + 5}, 3, v{x + 4}", VALU, rd=vr(x + 5) + vr(x + 4), wr=vr(x + 4)),
                I(f"v_xor_b32_e32 v{x + 5}, v{x + 3}, v{hh}", VALU, rd=vr(x + 3) + vr(hh), wr=vr(x + 5)),
                I(f"v_lshl_add_u32 v{V_TB0}, v{x + 5}, 4, v{x + 4}", VALU, rd=vr(x + 5) + vr(x + 4), wr=vr(V_TB0)),
                I(f"v_add_u32_e32 v{x + 5}, 2, v{hh}", VALU, rd=vr(hh), wr=vr(x + 5)),
                I(f"v_xor_b32_e32 v{x + 5}, v{x + 3}, v{x + 5}", VALU, rd=vr(x + 3) + vr(x + 5), wr=vr(x + 5)),
                I(f"v_lshl_add_u32 v{V_TB1}, v{x + 5}, 4, v{x + 4}", VALU, rd=vr(x + 5) + vr(x + 4), wr=vr(V_TB1))]
        # DMA voffsets: wave w, half f: row = 16 f + lane / 4, col = 64 w + 16 ((lane & 3) ^ ((lane >> 4) & 3));
        # d = 64: row = 16 (w >> 1) + lane / 4, col = 64 (w & 1) + 16 (...)
        ins += [I(f"v_lshrrev_b32_e32 v{x}, 2, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x))]
        if PIECES == 2:
            ins += [I(f"s_lshr_b32 s{T[0]}, s{S_WAVE}, 1", SALU, rd=sr(S_WAVE), wr=sr(T[0])),
                    I(f"s_lshl_b32 s{T[0]}, s{T[0]}, 4", SALU, rd=sr(T[0]), wr=sr(T[0])),
                    I(f"v_add_u32_e32 v{x}, s{T[0]}, v{x}", VALU, rd=sr(T[0]) + vr(x), wr=vr(x))]
        ins += [
                I(f"v_bfe_u32 v{x + 1}, v{V_LANE}, 4, 2", VALU, rd=vr(V_LANE), wr=vr(x + 1)),
                I(f"v_and_b32_e32 v{x + 2}, 3, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 2)),
                I(f"v_xor_b32_e32 v{x + 1}, v{x + 1}, v{x + 2}", VALU, rd=vr(x + 1, 2), wr=vr(x + 1)),
                I(f"v_lshlrev_b32_e32 v{x + 1}, 4, v{x + 1}", VALU, rd=vr(x + 1), wr=vr(x + 1)),
                (I(f"s_lshl_b32 s{T[0]}, s{S_WAVE}, 6", SALU, rd=sr(S_WAVE), wr=sr(T[0])) if PIECES == 4 else
                 I(f"s_and_b32 s{T[0]}, s{S_WAVE}, 1", SALU, rd=sr(S_WAVE), wr=sr(T[0]))),
                ] + ([] if PIECES == 4 else [I(f"s_lshl_b32 s{T[0]}, s{T[0]}, 6", SALU, rd=sr(T[0]), wr=sr(T[0]))]) + [
                I(f"v_add_u32_e32 v{x + 1}, s{T[0]}, v{x + 1}", VALU, rd=sr(T[0]) + vr(x + 1), wr=vr(x + 1)),
                I(f"v_mul_lo_u32 v{V_KV0}, v{x}, s{Rkv}", VALU, rd=vr(x) + sr(Rkv), wr=vr(V_KV0)),
                I(f"v_add_u32_e32 v{V_KV0}, v{V_KV0}, v{x + 1}", VALU, rd=vr(V_KV0) + vr(x + 1), wr=vr(V_KV0)),
                I(f"s_lshl_b32 s{T[0]}, s{Rkv}, 4", SALU, rd=sr(Rkv), wr=sr(T[0])),
                I(f"v_add_u32_e32 v{V_KV1}, s{T[0]}, v{V_KV0}", VALU, rd=sr(T[0]) + vr(V_KV0), wr=vr(V_KV1)),
                I(f"v_mov_b32_e32 v{V_NINF}, 0xff800000", VALU, wr=vr(V_NINF))]
        # ---- loop state ----
        if PIECES == 4:     # this wave's LDS panel: 2048 w
            ins += [I(f"s_lshl_b32 s{S_W2K}, s{S_WAVE}, 11", SALU, rd=sr(S_WAVE), wr=sr(S_W2K))]
        else:               # d = 64: panel w & 1, rows 16 (w >> 1) -> 2048 (w & 1) + 1024 (w >> 1)
            ins += [I(f"s_and_b32 s{T[0]}, s{S_WAVE}, 1", SALU, rd=sr(S_WAVE), wr=sr(T[0])),
                    I(f"s_lshl_b32 s{T[0]}, s{T[0]}, 11", SALU, rd=sr(T[0]), wr=sr(T[0])),
                    I(f"s_lshr_b32 s{T[1]}, s{S_WAVE}, 1", SALU, rd=sr(S_WAVE), wr=sr(T[1])),
                    I(f"s_lshl_b32 s{T[1]}, s{T[1]}, 10", SALU, rd=sr(T[1]), wr=sr(T[1])),
                    I(f"s_add_u32 s{S_W2K}, s{T[0]}, s{T[1]}", SALU, rd=sr(T[0]) + sr(T[1]), wr=sr(S_W2K))]
        ins += [
                I(f"s_mov_b32 s{S_SDMA}, 0", SALU, wr=sr(S_SDMA)),
                I(f"s_mov_b32 s{S_NLAST}, s{T[8]}", SALU, rd=sr(T[8]), wr=sr(S_NLAST)),
                I(f"s_mov_b32 s{S_MASK0}, s{T[3]}", SALU, rd=sr(T[3]), wr=sr(S_MASK0)),
                I(f"s_lshl_b32 s{S_KV32}, s{Rkv}, 5", SALU, rd=sr(Rkv), wr=sr(S_KV32)),
                I(f"s_mov_b32 s{S_N}, 0", SALU, wr=sr(S_N))]
        for i in range(128):
            ins.append(I(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i)))
        return ins

    def fused_d(self):
        """(flags bit 1) D = rowsum(dO o O) per row -- bwd_pre_kernel's work (fa_bwd.hip) for the item's
        rows -- from the O fragments (v[64:127], landed with the prologue's wait) and a VGPR copy of the
        dO fragments (v[0:63]); then V_D = D and bwd_pre_kernel's stores: softmax_d (dsum, descriptor
        s[52:55] of the D load: row 4) and the dK/dV scratch [-LSE / scale | -D] of each 32-row group
        (s[12:15] at the item's first group: (2 w + j) 256 + lane 4).  Rows past seqlen_q read zero O,
        dO and LSE: their scratch entries are zero, their softmax_d stores fall outside the records."""
        I = Inst
        l_nof = self.lab("nofused")
        r_, hh, x = V_TMP, V_TMP + 1, V_TMP + 2
        dot = f"v_dot2_f32_{self.ty}"
        ins = [I("s_bitcmp1_b32 s99, 1", SALU, rd=sr(99), wr=[("scc", 0)]), I(f"s_cbranch_scc0 {l_nof}", BRANCH)]
        if os.environ.get("FA_GDQ_FWAIT"):
            ins.append(I("s_waitcnt vmcnt(0)", WAIT))
        for j in range(2):
            for ks in range(KS):
                for k in range(4):
                    ins.append(I(f"v_accvgpr_read_b32 v{32 * j + 4 * ks + k}, a{OF(j, ks) + k}", ACCR,
                                 rd=ar(OF(j, ks) + k), wr=vr(32 * j + 4 * ks + k)))
        ins += [I(f"v_and_b32_e32 v{r_}, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(r_)),
                I(f"v_lshrrev_b32_e32 v{hh}, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(hh)),
                I(f"v_cmp_ne_u32_e32 vcc, 0, v{hh}", VALU, rd=vr(hh), wr=[("vcc", 0)])]
        for j in range(2):
            acc = V_D[j]
            ins.append(I(f"v_mov_b32_e32 v{acc}, 0", VALU, wr=vr(acc)))
            for i in range(4 * KS):
                ins.append(I(f"{dot} v{acc}, v{64 + 32 * j + i}, v{32 * j + i}, v{acc}", VALU,
                             rd=vr(64 + 32 * j + i) + vr(32 * j + i) + vr(acc), wr=vr(acc)))
            # the other lane half holds the row's other 64 columns (a v_dot result read by another
            # VALU op: 3 wait states -- tools/hazard_check.py "dot->valu")
            ins += [nop(2),
                    I(f"v_mov_b32_e32 v{x}, v{acc}", VALU, rd=vr(acc), wr=vr(x)),
                    I(f"v_permlane32_swap_b32_e32 v{acc}, v{x}", PERM, rd=vr(acc) + vr(x), wr=vr(acc) + vr(x)),
                    I(f"v_add_f32_e32 v{acc}, v{acc}, v{x}", VALU, rd=vr(acc) + vr(x), wr=vr(acc))]
            # softmax_d[m0 + 64 w + 32 j + r]
            ins += [I(f"s_lshl_b32 s{S_TMP}, s{S_WAVE}, 6", SALU, rd=sr(S_WAVE), wr=sr(S_TMP)),
                    I(f"v_add_u32_e32 v{x + 1}, s{S_TMP}, v{r_}", VALU, rd=sr(S_TMP) + vr(r_), wr=vr(x + 1)),
                    I(f"v_add_u32_e32 v{x + 1}, {32 * j}, v{x + 1}", VALU, rd=vr(x + 1), wr=vr(x + 1)),
                    I(f"v_lshlrev_b32_e32 v{x + 1}, 2, v{x + 1}", VALU, rd=vr(x + 1), wr=vr(x + 1)),
                    I(f"buffer_store_dword v{acc}, v{x + 1}, s[52:55], 0 offen", VSTORE, rd=vr(acc) + vr(x + 1) + sr(52, 4)),
                    # scratch group 2 w + j, lane: hh ? -D : -LSE / scale (V_NLC holds the raw LSE here)
                    I(f"v_mul_f32_e32 v{x + 2}, s49, v{V_NLC[j]}", VALU, rd=sr(49) + vr(V_NLC[j]), wr=vr(x + 2)),
                    I(f"v_sub_f32_e32 v{x + 3}, 0, v{acc}", VALU, rd=vr(acc), wr=vr(x + 3)),
                    I(f"v_cndmask_b32_e32 v{x + 2}, v{x + 2}, v{x + 3}, vcc", VALU, rd=vr(x + 2, 2) + [("vcc", 0)], wr=vr(x + 2)),
                    I(f"s_lshl_b32 s{S_TMP + 1}, s{S_WAVE}, 9", SALU, rd=sr(S_WAVE), wr=sr(S_TMP + 1)),
                    I(f"v_lshlrev_b32_e32 v{x + 4}, 2, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 4)),
                    I(f"v_add_u32_e32 v{x + 4}, s{S_TMP + 1}, v{x + 4}", VALU, rd=sr(S_TMP + 1) + vr(x + 4), wr=vr(x + 4)),
                    I(f"buffer_store_dword v{x + 2}, v{x + 4}, s[12:15], 0 offen offset:{256 * j}", VSTORE,
                      rd=vr(x + 2) + vr(x + 4) + sr(12, 4))]
        ins += [label(l_nof)]
        return ins

    def q_fold_setup(self):
        """(the Q fold) lane offsets of the Q' stores: (64 w + 32 j + r) qf_row + 16 hh -> v[V_TMP + 2 + j]"""
        I = Inst
        r_, hh, x = V_TMP, V_TMP + 1, V_TMP + 2
        ins = [I(f"v_and_b32_e32 v{r_}, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(r_)),
               I(f"v_lshrrev_b32_e32 v{hh}, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(hh)),
               I(f"s_lshl_b32 s{S_TMP}, s{S_WAVE}, 6", SALU, rd=sr(S_WAVE), wr=sr(S_TMP))]
        for j in range(2):
            off = x + j
            ins += [I(f"v_add_u32_e32 v{off}, s{S_TMP}, v{r_}", VALU, rd=sr(S_TMP) + vr(r_), wr=vr(off)),
                    I(f"v_add_u32_e32 v{off}, {32 * j}, v{off}", VALU, rd=vr(off), wr=vr(off)),
                    I(f"v_mul_lo_u32 v{off}, v{off}, s60", VALU, rd=vr(off) + sr(60), wr=vr(off)),
                    I(f"v_lshl_add_u32 v{off}, v{hh}, 4, v{off}", VALU, rd=vr(hh) + vr(off), wr=vr(off))]
        return ins

    def q_fold_fill(self):
        """(flags bit 2) the backward of a forward that held Q as bf16/f16(c Q) (gen_fwd.py FA_GEN_FOLD,
        launch_bwd): each Q fragment becomes bf16/f16(qc Q) -- v_mul_f32 by qc and a round-to-nearest-
        even pack, the forward's own q_scale_ops, so the scores S^T = K Q'^T (c = 1 on this launch)
        are bitwise the forward's -- before the phase -1 MFMA that reads it (fillers with deadlines:
        the conversion hides in the phase's gaps), and Q' is stored for the dK/dV kernel (descriptor
        s[56:59], qc s62; rows past seqlen_q fall outside the records).  Temporaries: the idle S^T /
        dP^T buffers 1 (v[32:63], v[96:127]), 8 rotating 4-register slots."""
        I = Inst
        x = V_TMP + 2
        ops = []
        for ks in range(KS):
            for j in range(2):
                slot = (2 * ks + j) % 8
                X, LO = 32 + 4 * slot, 96 + 4 * slot
                q = QF(j, ks)
                kw = dict(key=-150 + 8 * ks + 2 * j, deadline=4 * ks + j)
                ops += [I(f"v_accvgpr_read_b32 v{X + i}, a{q + i}", ACCR, rd=ar(q + i), wr=vr(X + i), **kw) for i in range(4)]
                if self.bf16:
                    ops += [I(f"v_lshlrev_b32_e32 v{LO + i}, 16, v{X + i}", VALU, rd=vr(X + i), wr=vr(LO + i), **kw)
                            for i in range(4)]
                    ops += [I(f"v_and_b32_e32 v{X + i}, 0xffff0000, v{X + i}", VALU, rd=vr(X + i), wr=vr(X + i), **kw)
                            for i in range(4)]
                else:
                    ops += [I(f"v_cvt_f32_f16_e32 v{LO + i}, v{X + i}", VALU, rd=vr(X + i), wr=vr(LO + i), **kw)
                            for i in range(4)]
                    ops += [I(f"v_lshrrev_b32_e32 v{X + i}, 16, v{X + i}", VALU, rd=vr(X + i), wr=vr(X + i), **kw)
                            for i in range(4)]
                    ops += [I(f"v_cvt_f32_f16_e32 v{X + i}, v{X + i}", VALU, rd=vr(X + i), wr=vr(X + i), **kw)
                            for i in range(4)]
                for R in (LO, X):
                    ops += [I(f"v_mul_f32_e32 v{R + i}, s62, v{R + i}", VALU, rd=sr(62) + vr(R + i), wr=vr(R + i), **kw)
                            for i in range(4)]
                ops += [self.cvt(LO + i, LO + i, X + i, **kw) for i in range(4)]
                ops += [I(f"v_accvgpr_write_b32 a{q + i}, v{LO + i}", ACCW, rd=vr(LO + i), wr=ar(q + i), **kw)
                        for i in range(4)]
                ops.append(I(f"buffer_store_dwordx4 v[{LO}:{LO + 3}], v{x + j}, s[56:59], 0 offen offset:{32 * ks}",
                             VSTORE, rd=vr(LO, 4) + vr(x + j) + sr(56, 4), key=kw["key"] + 1))
        return ops

    def epilogue(self):
        """dQ = scale dQ^T^T in bf16 / f16, rows < seqlen_q (range-checked; rows on lanes as gen_fwd.py)"""
        I = Inst
        ins = [I("s_waitcnt vmcnt(0)", WAIT)]
        t = 0
        for j in range(2):
            for dt in range(NP):
                for u in (0, 2):
                    w = t + 4 + 4 * ((dt * 2 + u // 2) % 4)
                    o = DQ(j, dt) + 4 * u
                    x = t + 20
                    ins += [I(f"v_accvgpr_read_b32 v{x + k}, a{o + k}", ACCR, rd=ar(o + k), wr=vr(x + k)) for k in range(8)]
                    ins += [I(f"v_mul_f32_e32 v{x + k}, s{S_SCALE}, v{x + k}", VALU, rd=sr(S_SCALE) + vr(x + k), wr=vr(x + k))
                            for k in range(8)]
                    ins += [self.cvt(w + 0, x + 0, x + 1), self.cvt(w + 1, x + 2, x + 3),
                            self.cvt(w + 2, x + 4, x + 5), self.cvt(w + 3, x + 6, x + 7)]
                    ins += [I(f"v_permlane32_swap_b32_e32 v{w}, v{w + 2}", PERM, rd=vr(w) + vr(w + 2), wr=vr(w) + vr(w + 2)),
                            I(f"v_permlane32_swap_b32_e32 v{w + 1}, v{w + 3}", PERM, rd=vr(w + 1) + vr(w + 3), wr=vr(w + 1) + vr(w + 3))]
                    ins.append(I(f"buffer_store_dwordx4 v[{w}:{w + 3}], v{V_QOFF[j]}, s[92:95], 0 offen offset:{64 * dt + 16 * u}",
                                 VSTORE, rd=vr(w, 4) + vr(V_QOFF[j]) + sr(92, 4)))
        return ins

    def phase_m1(self, fold):
        """phase -1: S^T / dP^T(0) -> buffers 0, then the first step's wait and barrier"""
        # -LSE log2 e (LSE = +inf -> -inf: P = 0); the loads landed with the prologue's wait
        ph = [Inst(f"v_mul_f32_e32 v{V_NLC[j]}, 0xbfb8aa3b, v{V_NLC[j]}", VALU, rd=vr(V_NLC[j]), wr=vr(V_NLC[j]), key=-500)
              for j in range(2)]
        if CHAIN_S or CHAIN_D:
            # the chain-start blocks: 16 copies of -LSE log2 e / c and of -D per q-block (a row's 16
            # accumulator elements are 16 keys of that row); c = 1 on the _c1 kernels.  The first MFMAs
            # read them: all in gap -1 (deadline 0; the scheduler orders fillers against MFMAs only so)
            ph = [x for x in ph]
            for x in ph:
                x.dl = 0
            t = V_TMP + 8
            if CHAIN_S and not self.unit_c:
                ph.append(Inst(f"v_rcp_f32_e32 v{t}, s{S_C}", TRANS, rd=sr(S_C), wr=vr(t), key=-500))
            for j in range(2):
                if CHAIN_S:
                    src = V_NLC[j]
                    if not self.unit_c:
                        ph.append(Inst(f"v_mul_f32_e32 v{V_TMP + 6 + j}, v{t}, v{V_NLC[j]}", VALU, rd=vr(t) + vr(V_NLC[j]),
                                       wr=vr(V_TMP + 6 + j), key=-499))
                        src = V_TMP + 6 + j
                    ph += [Inst(f"v_mov_b32_e32 v{NLCB(j) + e}, v{src}", VALU, rd=vr(src), wr=vr(NLCB(j) + e), key=-498)
                           for e in range(16)]
                if CHAIN_D:
                    ph += [Inst(f"v_sub_f32_e32 v{NDB(j) + e}, 0, v{V_D[j]}", VALU, rd=vr(V_D[j]), wr=vr(NDB(j) + e), key=-498)
                           for e in range(16)]
            for x in ph:
                x.dl = 0
        ph += [Inst(f"s_mov_b32 s{S_SROW}, 0", SALU, wr=sr(S_SROW)),
               Inst(f"s_mov_b32 s{S_STR}, {RING - 2 * SLOT}", SALU, wr=sr(S_STR)),
               Inst(f"v_add_u32_e32 v{V_KB0}, 0, v{V_RB0}", VALU, rd=vr(V_RB0), wr=vr(V_KB0)),
               Inst(f"v_add_u32_e32 v{V_KB1}, 0, v{V_RB1}", VALU, rd=vr(V_RB1), wr=vr(V_KB1))]
        mf, frags = self.phase_mfmas(1, True, False)
        fill = []
        for f, (t, i) in enumerate(frags):
            fill += self.frag_reads(f, t, i, key=-100 + f, deadline=max(2 * f - OPT_LEAD, 0),
                                    earliest=2 * (f - RING_SLOTS) + 1 if f >= RING_SLOTS else None)
        if fold:
            fill += self.q_fold_fill()
        fill += self.slot_advance(S_SROW, key=400) + self.slot_advance(S_STR, key=400)
        fill += [Inst(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0), key=401),
                 Inst(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1), key=401),
                 Inst(f"v_add_u32_e32 v{V_VB0}, s{S_STR}, v{V_TB0}", VALU, rd=sr(S_STR) + vr(V_TB0), wr=vr(V_VB0), key=401),
                 Inst(f"v_add_u32_e32 v{V_VB1}, s{S_STR}, v{V_TB1}", VALU, rd=sr(S_STR) + vr(V_TB1), wr=vr(V_VB1), key=401)]
        nfr = self.phase_frags(True, False)
        for f in range(3):
            t, i = nfr[f]
            users = [k for k in range(len(frags)) if k % RING_SLOTS == f % RING_SLOTS]
            fill += self.frag_reads(f, t, i, key=600 + f, earliest=2 * max(users) + 1)
        sch = schedule(mf, ph + fill)
        # (the fold's 16 Q' stores are younger than the K / V DMAs this wait is about)
        sch += [Inst(f"s_waitcnt vmcnt({VMCNT_STEP + (2 * KS if fold else 0)}) lgkmcnt(0)", WAIT), Inst("s_barrier", BARRIER)]
        return sch

    # ------------------------------------------------------------------ whole kernel
    def build(self):
        self.lab_end = self.lab("end")
        self.lab_next = self.lab("next")
        l_epi = self.lab("epi")
        code = []

        def emit(insts, pre=()):
            out, _ = add_waits(insts)
            out, _ = fix_hazards(out, pre=pre)
            code.extend(out)

        # once per workgroup: wave index, lane, round 0
        emit([Inst("v_lshrrev_b32_e32 v1, 6, v0", VALU, rd=vr(0), wr=vr(1)),
              Inst(f"v_readfirstlane_b32 s{S_WAVE}, v1", RFL, rd=vr(1), wr=sr(S_WAVE)),
              Inst(f"v_and_b32_e32 v{V_LANE}, 63, v0", VALU, rd=vr(0), wr=vr(V_LANE)),
              Inst(f"s_mov_b32 s{S_ROUND}, 0", SALU)])
        # persistent item loop (fa_bwd_asm.cpp, knob 6): workgroup w runs items r G + (r odd ? rev(w) :
        # w); G = n_items runs one item per workgroup.  The barrier keeps every wave's LDS reads of
        # the previous item ahead of the DMA of this one.
        l_item = self.lab("item")
        code.append(label(l_item))
        T0, T1, T2, T3 = (S_TMP + i for i in range(4))
        head = [Inst("s_barrier", BARRIER),
                Inst(f"s_load_dwordx2 s[{T0 + 1}:{T0 + 2}], s[0:1], {NITEMS_OFF}", SMEM),
                Inst("s_waitcnt lgkmcnt(0)", WAIT)]
        head += item_pos_ops(S_ITEM, S_ROUND, 2, T0 + 2, T0, T0 + 3)
        head += [Inst(f"s_cmp_ge_u32 s{S_ITEM}, s{T0 + 1}", SALU), Inst(f"s_cbranch_scc1 {self.lab_end}", BRANCH)]
        pro = head + self.prologue()
        for _ in range(KQ):
            pro += self.dma_subtile()
        # K / V(0) and (1) landed (phase -1 reads 0, its tail prefetches 1): 16 younger DMAs (d = 64: 8)
        pro += [Inst(f"s_waitcnt vmcnt({(KQ - 2) * PIECES})", WAIT), Inst("s_barrier", BARRIER)]
        pro += self.fused_d()
        # no keys: epilogue (dQ = 0), after the fused D (softmax_d and the scratch are still written)
        pro += [Inst(f"s_cmp_lt_i32 s{S_NLAST}, 0", SALU, rd=sr(S_NLAST), wr=[("scc", 0)]),
                Inst(f"s_cbranch_scc1 {l_epi}", BRANCH)]
        emit(pro, pre=[nop(15)])
        # phase -1: S^T / dP^T(0) -> buffers 0; with the Q fold (flags bit 2) a variant that converts
        # the Q fragments in its gaps (q_fold_fill)
        l_fold, l_after = self.lab("ph1fold"), self.lab("ph1done")
        code += [Inst("s_bitcmp1_b32 s99, 2", SALU), Inst(f"s_cbranch_scc1 {l_fold}", BRANCH)]
        emit(self.phase_m1(False) + [Inst(f"s_branch {l_after}", BRANCH)], pre=[nop(15)])
        code.append(label(l_fold))
        emit(self.q_fold_setup() + self.phase_m1(True), pre=[nop(15)])
        code.append(label(l_after))
        L = {}
        variants = [(f, l, m) for f in (True, False) for l in (True, False) for m in (True, False)]
        for v in variants:
            L[v] = self.lab("step_" + ("".join(c for c, on in zip("FLM", v) if on) or "R"))
        l_tail = self.lab("tail")
        l_disp = self.lab("dispatch")
        l_notlast = self.lab("notlast")
        l_first = self.lab("first")
        # entry: the first step (masked when causal and m0 == 0)
        code.append(label(l_first))
        code += [Inst(f"s_cmp_eq_u32 s{S_NLAST}, 0", SALU), Inst(f"s_cbranch_scc1 {l_first}_last", BRANCH)]
        code += [Inst(f"s_cmp_eq_u32 s{S_MASK0}, 0", SALU), Inst(f"s_cbranch_scc1 {L[(True, False, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(True, False, False)]}", BRANCH), label(f"{l_first}_last")]
        code += [Inst(f"s_cmp_eq_u32 s{S_MASK0}, 0", SALU), Inst(f"s_cbranch_scc1 {L[(True, True, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(True, True, False)]}", BRANCH)]
        # dispatch: done? last? masked (S_N >= S_MASK0)?
        code += [label(l_disp), Inst(f"s_cmp_gt_u32 s{S_N}, s{S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_tail}", BRANCH),
                 Inst(f"s_cmp_lt_u32 s{S_N}, s{S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_notlast}", BRANCH)]
        code += [Inst(f"s_cmp_ge_u32 s{S_N}, s{S_MASK0}", SALU), Inst(f"s_cbranch_scc1 {L[(False, True, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, True, False)]}", BRANCH), label(l_notlast)]
        code += [Inst(f"s_cmp_ge_u32 s{S_N}, s{S_MASK0}", SALU), Inst(f"s_cbranch_scc1 {L[(False, False, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, False, False)]}", BRANCH)]
        pad = [nop(15)]
        for v in variants:
            f, l, m = v
            code.append(label(L[v]))
            emit(self.step(f, l, m) + self.step_end(), pre=pad)
            code.append(Inst(f"s_branch {l_disp}", BRANCH))
        code.append(label(l_tail))
        emit(self.tail(), pre=pad)
        code.append(label(l_epi))
        emit([nop(15)] + self.epilogue(), pre=pad)
        code.append(label(self.lab_next))
        code += [Inst(f"s_add_u32 s{S_ROUND}, s{S_ROUND}, 1", SALU), Inst(f"s_branch {l_item}", BRANCH)]
        code.append(label(self.lab_end))
        code.append(Inst("s_endpgm", SOPP))
        return code

    def render(self):
        code = self.build()
        out = [f"\t.globl {self.name}", "\t.p2align 8", f"\t.type {self.name},@function", f"{self.name}:"]
        for ins in code:
            out.append(ins.text if ins.kind == LABEL else "\t" + ins.text)
        out.append(f".L{self.name}_fend:")
        out.append(f"\t.size {self.name}, .L{self.name}_fend-{self.name}")
        return "\n".join(out)

    def descriptor(self):
        return f"""
	.rodata
	.p2align 6
	.amdhsa_kernel {self.name}
		.amdhsa_group_segment_fixed_size {LDS_BYTES}
		.amdhsa_private_segment_fixed_size 0
		.amdhsa_kernarg_size {KARG_SIZE}
		.amdhsa_user_sgpr_count 2
		.amdhsa_user_sgpr_kernarg_segment_ptr 1
		.amdhsa_system_sgpr_workgroup_id_x 1
		.amdhsa_system_vgpr_workitem_id 0
		.amdhsa_next_free_vgpr 512
		.amdhsa_next_free_sgpr {NSGPR}
		.amdhsa_accum_offset 256
		.amdhsa_reserve_vcc 1
		.amdhsa_float_denorm_mode_32 3
		.amdhsa_float_denorm_mode_16_64 3
		.amdhsa_dx10_clamp 1
		.amdhsa_ieee_mode 0
	.end_amdhsa_kernel
	.text
"""

    def metadata(self):
        return f"""  - .agpr_count: 256
    .args:
      - .offset: 0
        .size: {KARG_SIZE}
        .value_kind: by_value
    .group_segment_fixed_size: {LDS_BYTES}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {KARG_SIZE}
    .max_flat_workgroup_size: 256
    .name: {self.name}
    .private_segment_fixed_size: 0
    .sgpr_count: {NSGPR + 2}
    .sgpr_spill_count: 0
    .symbol: {self.name}.kd
    .uniform_work_group_size: 1
    .vgpr_count: 512
    .vgpr_spill_count: 0
    .wavefront_size: 64
"""


def main():
    kernels = [K(bf, ca) for bf in (True, False) for ca in (True, False)]
    out = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 5", "\t.text"]
    for k in kernels:
        out.append(k.render())
        out.append(k.descriptor())
    out.append("\t.amdgpu_metadata\n---\namdhsa.kernels:")
    for k in kernels:
        out.append(k.metadata().rstrip("\n"))
    out.append("amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata")
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
