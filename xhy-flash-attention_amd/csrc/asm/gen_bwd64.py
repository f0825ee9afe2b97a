#!/usr/bin/env python3
"""Generates fa_bwd64_asm.s: the gfx950 dK / dV kernel for head dim 64 (round 6), built on
gen_bwd.py's d = 128 kernel (one wave per SIMD, all 512 registers).

    python3 gen_bwd64.py > fa_bwd64_asm.s

Same algorithm, kernel arguments, LSE / D scratch, work order and step structure as gen_bwd.py (the
reference's compute_dq_dk_dv_1colblock dK / dV half, csrc/flash_attn/src/flash_bwd_kernel.h:421-1046,
head-dim-64 instance flash_bwd_launch_template.h:194-235).  What changes at d = 64:

  * a wave owns 64 keys in two groups of 32 (workgroup = 4 waves = 256 keys): with the d = 128 layout
    (32 keys per wave) a d = 64 phase would have 16 MFMAs beside the same softmax VALU, LDS-DMA and
    SALU as at d = 128 -- issue-bound at about 60 % of the matrix pipe.  Two key groups give 32 MFMAs
    a phase again, and every A fragment read from LDS (Q / dO rows, dO^T / Q^T) feeds BOTH groups'
    MFMAs: 24 LDS fragment reads per 32 MFMAs (48 at d = 128).
  * registers: a[0:63] dV^T, a[64:127] dK^T (2 groups x 2 d-tiles x 16), a[128:159] K, a[160:191] V
    fragments (2 groups x 4 k-steps), a[192:255] the 16-slot A-fragment ring (one slot per fragment,
    two MFMAs per slot); v[0:63] S, v[64:127] dP (2 groups x 2 buffers), v[128:159] P packs,
    v[160:191] dS packs; P and dS are formed in place (no temporaries).
  * LDS: Q | dO subtiles of 32 rows x 64 (8 KiB a slot, 9 slots) and the -LSE / -D ring; each wave
    DMAs one 1-KiB piece of Q and one of dO per subtile (panel w & 1, rows 16 (w >> 1)).
  * causal: the diagonal crosses the first 8 subtiles of each head's sweep (a 256-key block).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bwd as G  # noqa: E402
import isa as _isa  # noqa: E402
from isa import (LDS, SALU, TRANS, VALU, VLOAD, Inst, ar, rtxt, schedule, sr, vr)  # noqa: E402

assert not G.OPT_CONT and not G.OPT_STAMP and not G.OPT_STEPSTAMP, "gen_bwd64: the dev builds are gen_bwd.py's"
_isa.apply_costs(os.environ.get("FA_G64_COST", ""))

D = G.D = 64
KS = G.KS = D // 16                 # 4 k-steps of S / dP
NP = G.NP = D // 32                 # 2 d-tiles of dV^T / dK^T
QT = G.QT = G.SUB * D * 2           # 4 KiB: one Q (or dO) subtile
SLOT = G.SLOT = 2 * QT
G.RING = G.NS * SLOT                # 9 slots = 72 KiB
G.LBASE = G.RING
G.LDS_BYTES = G.LBASE + G.NLS * G.LSLOT
assert G.LBASE % 4096 == 0
BKN = 256                           # keys per workgroup
# vmcnt at a step's end: younger than Q / dO(2n + 3) (issued in step n - 2, 2 pieces): L(2n + 5) and the
# 6 ops of step n - 1 (Q / dO 2 + 2, L 1 + 1)
G.VMCNT_STEP = 7
PRO_VMCNT = 13                      # the prologue's wait (gen_bwd.py's 21 with 2-piece subtiles)


# ---- AGPRs ----
def DVg(g):
    return 32 * g


def DKg(g):
    return 64 + 32 * g


def KFg(g):
    return 128 + 16 * g


def VFg(g):
    return 160 + 16 * g


G.DV, G.DK, G.KF, G.VF = DVg(0), DKg(0), KFg(0), VFg(0)
RGB = 192


def ring(slot):
    return RGB + 4 * (slot % 16)


G.ring = ring


# ---- VGPRs ----
def SBg(g, par):
    return 32 * g + 16 * par


def DPBg(g, par):
    return 64 + 32 * g + 16 * par


def PPg(g, par):
    return 128 + 16 * g + 8 * par


def DSPg(g, par):
    return 160 + 16 * g + 8 * par


(G.V_RB0, G.V_RB1, G.V_TB0, G.V_TB1, G.V_KB0, G.V_KB1, G.V_VB0, G.V_VB1) = range(192, 200)
G.V_LB, G.V_LCUR = 200, 201
G.V_QV0, G.V_QV1, G.V_OV0, G.V_OV1 = 202, 203, 204, 205
G.V_L4, G.V_LANEK, G.V_LM, G.V_NINF, G.V_LANE = 206, 207, 208, 209, 210
G.V_TMP = 211                       # 211..219 (prologue)
G.V_ST = 220                        # 220..234 (the epilogue's scalars)
G.V_ROUND = 235
V_LANEK1, V_LM1 = 236, 237          # key group 1's mask lane value and limit
V_KOFF1, V_VOFF1 = 238, 239         # key group 1's K / V fragment offsets (32 rows on)
G.T = 0                             # (unused: P and dS are formed in place)
V_LANEK = (G.V_LANEK, V_LANEK1)
V_LM = (G.V_LM, V_LM1)
WIN = int(os.environ.get("FA_G64_WIN", "16"))   # a fragment read may run WIN MFMAs (WIN / 2 slots) ahead
assert WIN <= 32
LEAD = 2


class K64(G.K):
    """one kernel variant (bf16 / f16, causal or not, c = 1 or not)"""

    def __init__(self, bf16, causal, unit_c=False):
        super().__init__(bf16, causal, unit_c)
        self.name = f"fa_bwd_dkdv_asm_d64_{self.ty}_{'causal' if causal else 'full'}{'_c1' if unit_c else ''}"

    # ------------------------------------------------------------------ MFMAs: pairs sharing an A fragment
    def phase_mfmas(self, par, sdp, dvdk):
        """(mfma, type, i) list; MFMAs 2j and 2j + 1 are the two key groups' and read ring slot j"""
        nb = 1 - par
        kinds = [t for t in ("S", "dV", "dP", "dK") if (sdp if t in ("S", "dP") else dvdk)]
        out = []
        for i in range(4):
            for t in kinds:
                slot = len(out) // 2
                for g in (0, 1):
                    if t == "S":
                        mf = self.mf(("v", SBg(g, nb)), ("a", ring(slot)), ("a", KFg(g) + 4 * i), "v")
                    elif t == "dP":
                        mf = self.mf(("v", DPBg(g, nb)), ("a", ring(slot)), ("a", VFg(g) + 4 * i), "v")
                    elif t == "dV":
                        dt, kk = i // 2, i % 2
                        mf = self.mf(("a", DVg(g) + 16 * dt), ("a", ring(slot)), ("v", PPg(g, nb) + 4 * kk), "a")
                    else:
                        dt, kk = i // 2, i % 2
                        mf = self.mf(("a", DKg(g) + 16 * dt), ("a", ring(slot)), ("v", DSPg(g, nb) + 4 * kk), "a")
                    out.append((mf, t, i))
        return out

    def frag_reads(self, m, t, i, **kw):
        """the shared A fragment of the MFMA pair m // 2 (nothing for the pair's second MFMA)"""
        if m % 2:
            return []
        if kw.get("key", 0) >= 600 and kw.get("earliest") == m:
            # (gen_bwd's phase -1 prefetch passes "slot m is free after MFMA m": here slot m // 2
            # is read by MFMAs m and m + 1)
            kw["earliest"] = m + 1
        dst = ring(m // 2)
        if t in ("S", "dP"):
            base = G.V_KB0 if i % 2 == 0 else G.V_KB1
            off = (i // 2) * 2048 + (QT if t == "dP" else 0)
            return [Inst(f"ds_read_b128 {rtxt('a', dst, 4)}, v{base} offset:{off}", LDS, rd=vr(base), wr=ar(dst, 4), **kw)]
        dt, kk = i // 2, i % 2
        out = []
        for h in range(2):
            base = G.V_VB0 if h == 0 else G.V_VB1
            off = (QT if t == "dV" else 0) + dt * 2048 + kk * 1024 + h * 512
            out.append(Inst(f"ds_read_b64_tr_b16 {rtxt('a', dst + 2 * h, 2)}, v{base} offset:{off}", LDS,
                            rd=vr(base), wr=ar(dst + 2 * h, 2), **kw))
        return out

    # ------------------------------------------------------------------ VALU of one subtile, both groups
    def valu_ops(self, par, masked, q0_add):
        ops = []
        for g in (0, 1):
            S, DP, PK, DSK = SBg(g, par), DPBg(g, par), PPg(g, par), DSPg(g, par)
            lm, lk = V_LM[g], V_LANEK[g]
            k0 = 128 * g
            if masked:
                ops.append(Inst(f"v_subrev_u32 v{lm}, s{G.S_Q0V}, v{lk}", VALU, rd=sr(G.S_Q0V) + vr(lk), wr=vr(lm), key=k0))
                if q0_add:
                    ops.append(Inst(f"v_subrev_u32 v{lm}, {q0_add}, v{lm}", VALU, rd=vr(lm), wr=vr(lm), key=k0))
            for e in range(16):
                x = S + e
                if not self.unit_c:
                    ops.append(Inst(f"v_mul_f32_e32 v{x}, s{G.S_C}, v{x}", VALU, rd=sr(G.S_C) + vr(x), wr=vr(x), key=k0 + 4 * e))
                if masked:
                    const = (e & 3) + 8 * (e >> 2)
                    ops.append(Inst(f"v_cmp_lt_i32_e32 vcc, {const}, v{lm}", VALU, rd=vr(lm), wr=[("vcc", 0)], key=k0 + 4 * e))
                    ops.append(Inst(f"v_cndmask_b32_e32 v{x}, v{x}, v{G.V_NINF}, vcc", VALU,
                                    rd=vr(x) + vr(G.V_NINF) + [("vcc", 0)], wr=vr(x), key=k0 + 4 * e))
                ops.append(Inst(f"v_exp_f32_e32 v{x}, v{x}", TRANS, rd=vr(x), wr=vr(x), key=k0 + 4 * e + 1))
                if e % 2 == 1:
                    ops.append(self.cvt(PK + e // 2, x - 1, x, key=k0 + 4 * e + 2))
            for e in range(16):
                ops.append(Inst(f"v_mul_f32_e32 v{DP + e}, v{S + e}, v{DP + e}", VALU, rd=vr(S + e) + vr(DP + e),
                                wr=vr(DP + e), key=k0 + 64 + 2 * e))
                if e % 2 == 1:
                    ops.append(self.cvt(DSK + e // 2, DP + e - 1, DP + e, key=k0 + 64 + 2 * e + 1))
        return ops

    def init_reads(self, par):
        """chain starts of the subtile two ahead, for both groups (the same rows: read twice, LDS is
        cheaper than 32 v_mov)"""
        ops = []
        for g in (0, 1):
            for u in range(4):
                ops.append(Inst(f"ds_read_b128 v[{SBg(g, par) + 4 * u}:{SBg(g, par) + 4 * u + 3}], v{G.V_LCUR} offset:{32 * u}",
                                LDS, rd=vr(G.V_LCUR), wr=vr(SBg(g, par) + 4 * u, 4), key=200))
            for u in range(4):
                ops.append(Inst(f"ds_read_b128 v[{DPBg(g, par) + 4 * u}:{DPBg(g, par) + 4 * u + 3}], v{G.V_LCUR} offset:{128 + 32 * u}",
                                LDS, rd=vr(G.V_LCUR), wr=vr(DPBg(g, par) + 4 * u, 4), key=300))
        return ops

    # ------------------------------------------------------------------ DMA: one Q and one dO piece a wave
    def dma_subtile(self, with_l, key=-50, eg=None):
        I = Inst
        t = G.S_TMP
        ops = [I(f"s_add_u32 s{t}, s{G.S_SDMA}, s{G.S_W2K}", SALU, rd=sr(G.S_SDMA) + sr(G.S_W2K), wr=sr(t) + [("scc", 0)], key=key)]
        for j, (voff, desc, add) in enumerate(((G.V_QV0, G.S_QD, 0), (G.V_OV0, G.S_OD, QT))):
            e = None if eg is None else eg + 2 * j
            ops.append(I(f"s_add_u32 m0, s{t}, {add}", SALU, rd=sr(t), wr=[("m0", 0)] + [("scc", 0)], key=key, earliest=e))
            ops.append(I(f"buffer_load_dwordx4 v{voff}, s[{desc}:{desc + 3}], 0 offen lds", G.DMA,
                         rd=vr(voff) + sr(desc, 4) + [("m0", 0)], key=key, earliest=e))
        full = super().dma_subtile(with_l, key, eg)
        # (the base version: its t = s_add, 4 x (m0, piece), then the L piece and the cursors)
        rest = full[1 + 8:]
        return ops + rest

    # ------------------------------------------------------------------ one phase (pairs share ring slots)
    def phase(self, par, sdp, dvdk, valu, masked, q0_add, dma, next_kind, first_pref, tail_of_step):
        mf = self.phase_mfmas(par, sdp, dvdk)
        mfmas = [x[0] for x in mf]
        n = len(mfmas)
        fill = []
        for m, (_, t, i) in enumerate(mf):
            if m < 3 and first_pref:
                continue
            fill += self.frag_reads(m, t, i, key=-100 + m, earliest=(m - WIN) if m >= WIN else None,
                                    deadline=max(m - LEAD, 0))
        if valu:
            fill += self.valu_ops(par, masked, q0_add)
            fill += self.init_reads(par)
        if dma:
            fill += self.dma_subtile(True, key=-40, eg=2)
        I = Inst
        nxt = self.slot_advance(G.S_SROW, key=400) + self.slot_advance(G.S_STR, key=400) + self.lslot_advance(G.S_LRD, key=400)
        nxt += [I(f"v_add_u32_e32 v{G.V_KB0}, s{G.S_SROW}, v{G.V_RB0}", VALU, rd=sr(G.S_SROW) + vr(G.V_RB0), wr=vr(G.V_KB0), key=401),
                I(f"v_add_u32_e32 v{G.V_KB1}, s{G.S_SROW}, v{G.V_RB1}", VALU, rd=sr(G.S_SROW) + vr(G.V_RB1), wr=vr(G.V_KB1), key=401),
                I(f"v_add_u32_e32 v{G.V_VB0}, s{G.S_STR}, v{G.V_TB0}", VALU, rd=sr(G.S_STR) + vr(G.V_TB0), wr=vr(G.V_VB0), key=401),
                I(f"v_add_u32_e32 v{G.V_VB1}, s{G.S_STR}, v{G.V_TB1}", VALU, rd=sr(G.S_STR) + vr(G.V_TB1), wr=vr(G.V_VB1), key=401),
                I(f"v_add_u32_e32 v{G.V_LCUR}, s{G.S_LRD}, v{G.V_LB}", VALU, rd=sr(G.S_LRD) + vr(G.V_LB), wr=vr(G.V_LCUR), key=401)]
        fill += nxt
        if next_kind is not None:
            nm = self.phase_mfmas(0, next_kind in ("full", "sdp"), next_kind in ("full", "dvdk"))
            for m in range(3):
                _, t, i = nm[m]
                # slot m // 2 is free once this phase's last MFMA reading it has issued
                last_user = max([k for k in range(n) if (k // 2) % 16 == (m // 2) % 16], default=None)
                fill += self.frag_reads(m, t, i, key=600 + m, earliest=last_user)
        if tail_of_step:
            fill += tail_of_step
        return schedule(mfmas, fill)

    def tail(self):
        mf = self.phase_mfmas(0, False, True)
        fill = []
        for m, (_, t, i) in enumerate(mf):
            if m < 3:
                continue
            fill += self.frag_reads(m, t, i, key=-100 + m, earliest=(m - WIN) if m >= WIN else None,
                                    deadline=max(m - 2, 0))
        return schedule([x[0] for x in mf], fill)

    # ------------------------------------------------------------------ prologue: patches of gen_bwd's
    def prologue(self, l_epi, l_nokeys=None, cont=False):
        ins = super().prologue(l_epi, l_nokeys, cont)
        I = Inst
        T0, T1 = G.S_TMP, G.S_TMP + 1
        ka = 56
        Rq, Rk, Rv, Rdo = ka + 32, ka + 33, ka + 34, ka + 35
        out = []
        n_fix = 0
        for x in ins:
            if x.kind == SALU and x.text.endswith(f", s{G.S_WAVE}, 5"):           # KW0 = n0 + 64 w
                x = I(x.text[:-1] + "6", SALU, rd=x.rd, wr=x.wr)
                n_fix += 1
            if x.kind == SALU and x.text.startswith("s_lshl_b32 ") and x.text.endswith(", 7") and \
                    x.text.split()[2] == f"s{27}," :                                # n0 = 256 key block
                x = I(x.text[:-1] + "8", SALU, rd=x.rd, wr=x.wr)
                n_fix += 1
            if x.kind == SALU and x.text == f"s_lshl_b32 s{G.S_W2K}, s{G.S_WAVE}, 11":
                # this wave's DMA piece: panel w & 1, rows 16 (w >> 1) -> LDS + 2048 (w & 1) + 1024 (w >> 1)
                out += [I(f"s_and_b32 s{T0}, s{G.S_WAVE}, 1", SALU, rd=sr(G.S_WAVE), wr=sr(T0)),
                        I(f"s_lshl_b32 s{T0}, s{T0}, 11", SALU, rd=sr(T0), wr=sr(T0)),
                        I(f"s_lshr_b32 s{T1}, s{G.S_WAVE}, 1", SALU, rd=sr(G.S_WAVE), wr=sr(T1)),
                        I(f"s_lshl_b32 s{T1}, s{T1}, 10", SALU, rd=sr(T1), wr=sr(T1)),
                        I(f"s_add_u32 s{G.S_W2K}, s{T0}, s{T1}", SALU, rd=sr(T0) + sr(T1), wr=sr(G.S_W2K))]
                continue
            if x.kind == VALU and x.text == f"v_lshlrev_b32_e32 v{G.V_L4}, 2, v{G.V_LANE}":
                # DMA voffsets (replacing gen_bwd's 2 x 2 pieces): row = 16 (w >> 1) + lane / 4,
                # col = 64 (w & 1) + 16 ((lane & 3) ^ ((lane >> 4) & 3)); group 1's K / V offsets
                t = G.V_TMP + 4
                out += [I(f"v_lshrrev_b32_e32 v{t}, 2, v{G.V_LANE}", VALU, rd=vr(G.V_LANE), wr=vr(t)),
                        I(f"s_lshr_b32 s{T0}, s{G.S_WAVE}, 1", SALU, rd=sr(G.S_WAVE), wr=sr(T0)),
                        I(f"s_lshl_b32 s{T0}, s{T0}, 4", SALU, rd=sr(T0), wr=sr(T0)),
                        I(f"v_add_u32_e32 v{t}, s{T0}, v{t}", VALU, rd=sr(T0) + vr(t), wr=vr(t)),
                        I(f"v_bfe_u32 v{t + 1}, v{G.V_LANE}, 4, 2", VALU, rd=vr(G.V_LANE), wr=vr(t + 1)),
                        I(f"v_and_b32_e32 v{t + 2}, 3, v{G.V_LANE}", VALU, rd=vr(G.V_LANE), wr=vr(t + 2)),
                        I(f"v_xor_b32_e32 v{t + 1}, v{t + 1}, v{t + 2}", VALU, rd=vr(t + 1, 2), wr=vr(t + 1)),
                        I(f"v_lshlrev_b32_e32 v{t + 1}, 4, v{t + 1}", VALU, rd=vr(t + 1), wr=vr(t + 1)),
                        I(f"s_and_b32 s{T0}, s{G.S_WAVE}, 1", SALU, rd=sr(G.S_WAVE), wr=sr(T0)),
                        I(f"s_lshl_b32 s{T0}, s{T0}, 6", SALU, rd=sr(T0), wr=sr(T0)),
                        I(f"v_add_u32_e32 v{t + 1}, s{T0}, v{t + 1}", VALU, rd=sr(T0) + vr(t + 1), wr=vr(t + 1)),
                        I(f"v_mul_lo_u32 v{G.V_QV0}, v{t}, s{Rq}", VALU, rd=vr(t) + sr(Rq), wr=vr(G.V_QV0)),
                        I(f"v_add_u32_e32 v{G.V_QV0}, v{G.V_QV0}, v{t + 1}", VALU, rd=vr(G.V_QV0) + vr(t + 1), wr=vr(G.V_QV0)),
                        I(f"v_mul_lo_u32 v{G.V_OV0}, v{t}, s{Rdo}", VALU, rd=vr(t) + sr(Rdo), wr=vr(G.V_OV0)),
                        I(f"v_add_u32_e32 v{G.V_OV0}, v{G.V_OV0}, v{t + 1}", VALU, rd=vr(G.V_OV0) + vr(t + 1), wr=vr(G.V_OV0))]
            out.append(x)
            if x.kind == VLOAD and x.text.startswith(f"buffer_load_dwordx4 {rtxt('a', VFg(0) + 4 * (KS - 1), 4)}"):
                # key group 1 (32 rows on): its K / V fragments (the descriptors' records already count
                # from the wave's first key, so rows past seqlen_k read zero)
                out += [I(f"s_lshl_b32 s{T0}, s{Rk}, 5", SALU, rd=sr(Rk), wr=sr(T0)),
                        I(f"v_add_u32_e32 v{V_KOFF1}, s{T0}, v{G.V_TMP + 2}", VALU, rd=sr(T0) + vr(G.V_TMP + 2), wr=vr(V_KOFF1)),
                        I(f"s_lshl_b32 s{T0}, s{Rv}, 5", SALU, rd=sr(Rv), wr=sr(T0)),
                        I(f"v_add_u32_e32 v{V_VOFF1}, s{T0}, v{G.V_TMP + 3}", VALU, rd=sr(T0) + vr(G.V_TMP + 3), wr=vr(V_VOFF1))]
                for base, lo, d0 in ((KFg(1), V_KOFF1, 72), (VFg(1), V_VOFF1, 76)):
                    for ks in range(KS):
                        out.append(I(f"buffer_load_dwordx4 {rtxt('a', base + 4 * ks, 4)}, v{lo}, s[{d0}:{d0 + 3}], 0 offen offset:{32 * ks}",
                                     VLOAD, rd=vr(lo) + sr(d0, 4), wr=ar(base + 4 * ks, 4)))
        assert n_fix == 2, "gen_bwd64: the prologue's key-block / wave-key shifts moved"
        # group 1's mask lane value (before the final nothing-to-sweep branch)
        out.insert(len(out) - 2, I(f"v_add_u32_e32 v{V_LANEK1}, 32, v{G.V_LANEK}", VALU, rd=vr(G.V_LANEK), wr=vr(V_LANEK1)))
        return out

    # ------------------------------------------------------------------ epilogue: both key groups
    def epilogue(self, stash=G.V_ST, zero=False):
        """gen_bwd's epilogue for key group 0, then for group 1 (the stash's first key + 32)"""
        I = Inst
        a = self._epi_group(0)
        out = [x for x in a]
        # group 1: its first key is 32 on (the stashed KW0 is group 0's)
        out += [I(f"v_add_u32_e32 v{G.V_ST}, 32, v{G.V_ST}", VALU, rd=vr(G.V_ST), wr=vr(G.V_ST))]
        out += [x for x in self._epi_group(1) if not x.text.startswith("s_waitcnt vmcnt(0)")]
        return out

    def _epi_group(self, g):
        save = (G.DV, G.DK)
        G.DV, G.DK = DVg(g), DKg(g)
        try:
            return super().epilogue(stash=G.V_ST)   # (its default was bound to gen_bwd's V_ST)
        finally:
            G.DV, G.DK = save

    def build(self):
        code = super().build()
        for x in code:
            if x.text == f"s_cmp_lt_u32 s{G.S_LOCV}, 4":          # the diagonal crosses 8 subtiles
                x.text = f"s_cmp_lt_u32 s{G.S_LOCV}, 8"
            elif x.text == "s_waitcnt vmcnt(21)":
                x.text = f"s_waitcnt vmcnt({PRO_VMCNT})"
        return code


def main():
    kernels = [K64(bf, ca, u) for u in (False, True) for bf in (True, False) for ca in (True, False)]
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
