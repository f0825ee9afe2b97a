#!/usr/bin/env python3
"""Generates fa_bwd2_asm.s: the gfx950 dK / dV kernel for head dim 128 with TWO waves per SIMD, the
waves specialised by role (round 6; the one-wave-per-SIMD kernel is gen_bwd.py).

    python3 gen_bwd2.py > fa_bwd2_asm.s

Same algorithm, work order, kernel arguments, LSE / D scratch and epilogue layout as gen_bwd.py (the
reference's compute_dq_dk_dv_1colblock dK / dV half, csrc/flash_attn/src/flash_bwd_kernel.h:421-1046):
    S' = Q K^T - LSE / scale,  P = exp2(c S'),  dP' = dO V^T - D,  dS = P o dP',
    dV^T += dO^T P,  dK^T += Q^T dS.

Why: the one-wave kernel is issue-bound -- a wave alone on its SIMD issues one instruction per turn, so
its 56 LDS reads, ~40 SALU and 5 LDS-DMA pieces per 32-MFMA phase queue behind its own VALU and MFMAs
("where the time goes").  Two waves per SIMD let one wave's LDS / SALU / DMA issue in the
same turn as the other's VALU or MFMA (MI355X_MICROARCH.md "Two waves per SIMD").  A wave then has
256 registers, which is one accumulator, not two, so the waves split the work by role:
  * workgroup = 8 waves x 64 lanes, 128 keys; wave w: key group kg = w & 3 (keys 32 kg ..), role w >> 2
    (waves w and w + 4 share a SIMD and a key group);
  * "P" waves (role 0) hold K (a[64:95]) and dV^T (a[0:63]): per 32-row subtile p they compute
    S(p) = chain(-LSE) + Q K^T, P(p) = exp2(c S') (masked on the causal diagonal), write P(p) as fp32
    to an LDS exchange buffer, pack it and accumulate dV^T += dO(p)^T P(p);
  * "dS" waves (role 1) hold V (a[64:95]) and dK^T (a[0:63]): dP'(p) = chain(-D) + dO V^T, then --
    one phase later, once P(p) is in LDS -- dS(p) = P(p) o dP'(p), packed, dK^T += Q(p)^T dS(p).
  * phase p (one barrier each): P waves: S(p+1) || dV(p-1), VALU P(p); dS waves: dP(p) || dK(p-2),
    VALU dS(p-1).  16 MFMAs per wave and phase, 32 per SIMD, as the one-wave kernel.
  * LDS: Q / dO ring of 7 x 16 KiB (subtile j lives from phase j-1, its Q rows, to phase j+2, its
    Q^T for dK(j)), issued 4 subtiles ahead; the -LSE / -D rows (16 x 256 B, 6 ahead); the P
    exchange, 2 buffers x 4 key groups x 4 KiB.  148 KiB, one workgroup per CU.
  * registers (256 per wave: v0..v127, a0..a127): a[0:63] the accumulator, a[64:95] the B fragments
    (K or V), a[96:127] a ring of 8 A fragments; v[0:31] two S (dP) tiles, v[32:47] exp / dS
    temporaries, v[48:63] two packs, then addresses and the epilogue's scalars.
  * DMA: the P waves load the Q pieces, the dS waves the dO pieces (2 x 1 KiB per wave and phase),
    every wave the subtile's 256 B of -LSE / -D rows; one s_waitcnt vmcnt(7) + barrier per phase.
The P waves end with dV of the last subtile; the dS waves with two tail phases (dS of the last
subtile, dK of the last two) and no barrier: the next item starts with the item loop's barrier.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bwd as G  # noqa: E402
import isa as _isa  # noqa: E402
from isa import (ACCW, BARRIER, BRANCH, DMA, LDS, MFMA, RFL, SALU, SMEM, SOPP, TRANS, VALU, VLOAD, VSTORE,  # noqa: E402,F401
                 WAIT, Inst, add_waits, ar, fix_hazards, item_pos_ops, label, nop, rtxt, schedule, sr, vr)

_isa.apply_costs(os.environ.get("FA_G2_COST", ""))
assert not G.OPT_CONT and not G.OPT_STAMP and not G.OPT_STEPSTAMP, "gen_bwd2: the dev loop / stamp builds are gen_bwd.py's"

D, SUB, QT, SLOT = G.D, G.SUB, G.QT, G.SLOT
# ---- LDS ----
G.NS = 7
G.RING = G.NS * G.SLOT            # 114688
G.LBASE = G.RING
XBASE = G.LBASE + G.NLS * G.LSLOT  # 118784: P exchange
XBUF = 4 * 4096                    # one buffer: 4 key groups x (32 x 32 fp32)
G.LDS_BYTES = XBASE + 2 * XBUF     # 151552
assert G.LDS_BYTES <= 163840 and G.LBASE % 4096 == 0
KQ, KL = 4, 6                      # Q / dO subtile j DMA'd in phase j - KQ, LSE / D rows j in j - KL
VM_PHASE = 7                       # vmcnt at the end of a phase (3 VMEM ops per wave and phase)
# ---- AGPRs ----
ACC, BF, RGB, NRING = 0, 64, 96, 8
G.DV = G.DK = ACC
G.KF = G.VF = BF


def ring(m):
    return RGB + 4 * (m % NRING)


G.ring = ring
WIN = int(os.environ.get("FA_G2_WIN", str(NRING)))
assert 2 <= WIN <= NRING
LEAD = int(os.environ.get("FA_G2_LEAD", "2"))


# ---- VGPRs ----
def TB(par):
    return 16 * par


T = 32


def PK(par):
    return 48 + 8 * par


G.T = T
(G.V_RB0, G.V_RB1, G.V_TB0, G.V_TB1, G.V_KB0, G.V_KB1, G.V_VB0, G.V_VB1) = range(64, 72)
G.V_LB, G.V_LCUR = 72, 73
G.V_QV0, G.V_QV1, G.V_OV0, G.V_OV1 = 74, 75, 76, 77
G.V_L4, G.V_LANEK, G.V_LM, G.V_NINF = 78, 79, 80, 81
G.V_LANE, G.V_ROUND = 82, 83
V_X = 84                           # P exchange lane address: XBASE + 4096 kg + 16 lane
G.V_TMP = 85                       # 85..93 (prologue)
G.V_ST = 94                        # 94..108 (the epilogue's scalars)
NVGPR = 128
assert G.V_ST + 15 <= NVGPR
V_RB0, V_RB1, V_TB0, V_TB1, V_KB0, V_KB1, V_VB0, V_VB1 = range(64, 72)
S_TMP, S_SROW, S_STR, S_LRD, S_SDMA, S_LDMA, S_W2K = G.S_TMP, G.S_SROW, G.S_STR, G.S_LRD, G.S_SDMA, G.S_LDMA, G.S_W2K
S_QD, S_OD, S_LD, S_C = G.S_QD, G.S_OD, G.S_LD, G.S_C
# scheduling weights (the one-wave kernel's; a partner wave shares the issue, FA_G2_COST for A/B)
# static priority (MI355X_MICROARCH.md "Two waves per SIMD" item 4): "ds" the younger half (waves 4-7,
# the dS waves), "p" the P waves, "none"
PRIO = os.environ.get("FA_G2_PRIO", "none")   # (r06d: "ds" +6 %, "p" +0.6 % vs none)
# only the P waves DMA the -LSE / -D rows (the dS waves read them after the barrier); else every wave
L_P_ONLY = os.environ.get("FA_G2_LALL", "0") != "1"
# timing ablations (WRONG results; which resource bounds the steady state): "nobar" drops the phases'
# barriers, "noxb" the P exchange (stores and loads)
ABL = os.environ.get("FA_G2_ABL", "")
BUDGET = int(os.environ.get("FA_G2_BUDGET", "24"))   # gap-scheduler issue budget per MFMA gap


class K2(G.K):
    """one kernel variant: both roles' item loops, chosen per wave at the start"""

    def __init__(self, bf16, causal, unit_c=False):
        super().__init__(bf16, causal, unit_c)
        self.name = f"fa_bwd2_dkdv_asm_d{D}_{self.ty}_{'causal' if causal else 'full'}{'_c1' if unit_c else ''}"
        self.role = 0

    # ------------------------------------------------------------------ MFMAs of a phase
    def mfmas(self, par, first, second):
        """(inst, type, index) of a phase with VALU parity par; first: S(p+1) / dP(p), second:
        dV(p-1) / dK(p-2); interleaved so the two chains alternate"""
        if self.role == 0:
            ta, tb = "S", "dV"
            acc_a, pk = TB(1 - par), PK(1 - par)
        else:
            ta, tb = "dP", "dK"
            acc_a, pk = TB(par), PK(par)
        order = []
        for i in range(8):
            if first:
                order.append((ta, i))
            if second:
                order.append((tb, i))
        out = []
        for m, (t, i) in enumerate(order):
            if t in ("S", "dP"):
                out.append((self.mf(("v", acc_a), ("a", ring(m)), ("a", BF + 4 * i), "v"), t, i))
            else:
                dt, kk = i // 2, i % 2
                out.append((self.mf(("a", ACC + 16 * dt), ("a", ring(m)), ("v", pk + 4 * kk), "a"), t, i))
        return out

    @staticmethod
    def pref(mf):
        """the MFMAs of a phase whose A fragments the previous phase reads ahead: of the first three,
        all but S -- the Q rows of S(p+1) land only at the end of phase p-1 (vmcnt), after the
        previous phase's reads could have run"""
        return [m for m in range(min(3, len(mf))) if mf[m][1] != "S"]

    # ------------------------------------------------------------------ VALU
    def valu_p(self, par, masked, q0_add):
        """P waves: P = exp2(c S') of TB(par) -> T, packs PK(par), T -> exchange buffer par"""
        ops = []
        S, PKp = TB(par), PK(par)
        if masked:
            ops.append(Inst(f"v_subrev_u32 v{G.V_LM}, s{G.S_Q0V}, v{G.V_LANEK}", VALU, rd=sr(G.S_Q0V) + vr(G.V_LANEK),
                            wr=vr(G.V_LM), key=0))
            if q0_add:
                ops.append(Inst(f"v_subrev_u32 v{G.V_LM}, {q0_add}, v{G.V_LM}", VALU, rd=vr(G.V_LM), wr=vr(G.V_LM), key=0))
        for g in range(16):
            src = T + g
            if not self.unit_c:
                ops.append(Inst(f"v_mul_f32_e32 v{T + g}, s{S_C}, v{S + g}", VALU, rd=sr(S_C) + vr(S + g), wr=vr(T + g),
                                key=4 * g))
            elif not masked:
                src = S + g
            if masked:
                const = (g & 3) + 8 * (g >> 2)
                ops.append(Inst(f"v_cmp_lt_i32_e32 vcc, {const}, v{G.V_LM}", VALU, rd=vr(G.V_LM), wr=[("vcc", 0)], key=4 * g))
                x = S + g if self.unit_c else T + g
                ops.append(Inst(f"v_cndmask_b32_e32 v{T + g}, v{x}, v{G.V_NINF}, vcc", VALU,
                                rd=vr(x) + vr(G.V_NINF) + [("vcc", 0)], wr=vr(T + g), key=4 * g))
            ops.append(Inst(f"v_exp_f32_e32 v{T + g}, v{src}", TRANS, rd=vr(src), wr=vr(T + g), key=4 * g + 1))
            if g % 2 == 1:
                ops.append(self.cvt(PKp + g // 2, T + g - 1, T + g, key=4 * g + 2))
            if g % 4 == 3:
                # (after the pack that reads the last exp result: an exp -> LDS-store read of its
                # result is not in the hazard model, the pack in between gives the wait state)
                u = g // 4
                ops.append(Inst(f"ds_write_b128 v{V_X}, v[{T + 4 * u}:{T + 4 * u + 3}] offset:{par * XBUF + 1024 * u}",
                                LDS, rd=vr(V_X) + vr(T + 4 * u, 4), key=4 * g + 3, deps=[ops[-1]]))
        return ops

    def valu_ds(self, par):
        """dS waves: dS(p-1) = P(p-1) (exchange buffer 1 - par) o dP'(p-1) (TB(1 - par)) -> PK(1 - par)"""
        ops = []
        DP, PKq = TB(1 - par), PK(1 - par)
        for u in range(4):
            ops.append(Inst(f"ds_read_b128 v[{T + 4 * u}:{T + 4 * u + 3}], v{V_X} offset:{(1 - par) * XBUF + 1024 * u}",
                            LDS, rd=vr(V_X), wr=vr(T + 4 * u, 4), key=u))
        for g in range(16):
            ops.append(Inst(f"v_mul_f32_e32 v{T + g}, v{T + g}, v{DP + g}", VALU, rd=vr(T + g) + vr(DP + g),
                            wr=vr(T + g), key=8 + 2 * g))
            if g % 2 == 1:
                ops.append(self.cvt(PKq + g // 2, T + g - 1, T + g, key=8 + 2 * g + 1))
        return ops

    def init_reads2(self, dst, half):
        """the chain start of a subtile from the LSE / D slot at V_LCUR: half 0 -LSE / scale, 1 -D"""
        return [Inst(f"ds_read_b128 v[{dst + 4 * u}:{dst + 4 * u + 3}], v{G.V_LCUR} offset:{128 * half + 32 * u}", LDS,
                     rd=vr(G.V_LCUR), wr=vr(dst + 4 * u, 4), key=200) for u in range(4)]

    # ------------------------------------------------------------------ DMA
    def dma2(self, key=-40, eg=2):
        """this wave's 2 pieces of the next Q / dO subtile (P waves: Q, dS waves: dO) and the 256 B of
        the LSE / D cursor's subtile (every wave, the same bytes); both cursors advance"""
        I = Inst
        t = S_TMP
        ops = [I(f"s_add_u32 s{t}, s{S_SDMA}, s{S_W2K}", SALU, rd=sr(S_SDMA) + sr(S_W2K), wr=sr(t) + [("scc", 0)], key=key)]
        pieces = ((G.V_QV0, S_QD, 0), (G.V_QV1, S_QD, 1024)) if self.role == 0 else \
            ((G.V_OV0, S_OD, QT), (G.V_OV1, S_OD, QT + 1024))
        for j, (voff, desc, add) in enumerate(pieces):
            e = None if eg is None else eg + 2 * j
            ops.append(I(f"s_add_u32 m0, s{t}, {add}", SALU, rd=sr(t), wr=[("m0", 0)] + [("scc", 0)], key=key, earliest=e))
            ops.append(I(f"buffer_load_dwordx4 v{voff}, s[{desc}:{desc + 3}], 0 offen lds", DMA,
                         rd=vr(voff) + sr(desc, 4) + [("m0", 0)], key=key, earliest=e))
        e = None if eg is None else eg + 4
        if self.role == 0 or not L_P_ONLY:
            ops.append(I(f"s_mov_b32 m0, s{S_LDMA}", SALU, rd=sr(S_LDMA), wr=[("m0", 0)], key=key, earliest=e))
            ops.append(I(f"buffer_load_dword v{G.V_L4}, s[{S_LD}:{S_LD + 3}], 0 offen lds", DMA,
                         rd=vr(G.V_L4) + sr(S_LD, 4) + [("m0", 0)], key=key, earliest=e))
        for desc, step in ((S_QD, G.S_Q32), (S_OD, G.S_O32)):
            ops += [I(f"s_add_u32 s{desc}, s{desc}, s{step}", SALU, rd=sr(desc) + sr(step), wr=sr(desc) + [("scc", 0)], key=key + 1),
                    I(f"s_addc_u32 s{desc + 1}, s{desc + 1}, 0", SALU, rd=sr(desc + 1) + [("scc", 0)], wr=sr(desc + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_sub_u32 s{t + 1}, s{desc + 2}, s{step}", SALU, rd=sr(desc + 2) + sr(step), wr=sr(t + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_cselect_b32 s{desc + 2}, 0, s{t + 1}", SALU, rd=sr(t + 1) + [("scc", 0)], wr=sr(desc + 2), key=key + 1)]
        ops += [I(f"s_add_u32 s{G.S_LOCD}, s{G.S_LOCD}, 1", SALU, rd=sr(G.S_LOCD), wr=sr(G.S_LOCD) + [("scc", 0)], key=key + 1)]
        ops += self.slot_advance(S_SDMA, key + 1)
        if self.role == 1 and L_P_ONLY:
            return ops
        ops += [I(f"s_add_u32 s{S_LD}, s{S_LD}, {G.LSLOT}", SALU, rd=sr(S_LD), wr=sr(S_LD) + [("scc", 0)], key=key + 1),
                I(f"s_addc_u32 s{S_LD + 1}, s{S_LD + 1}, 0", SALU, rd=sr(S_LD + 1) + [("scc", 0)], wr=sr(S_LD + 1) + [("scc", 0)], key=key + 1),
                I(f"s_sub_u32 s{t + 1}, s{S_LD + 2}, {G.LSLOT}", SALU, rd=sr(S_LD + 2), wr=sr(t + 1) + [("scc", 0)], key=key + 1),
                I(f"s_cselect_b32 s{S_LD + 2}, 0, s{t + 1}", SALU, rd=sr(t + 1) + [("scc", 0)], wr=sr(S_LD + 2), key=key + 1),
                I(f"s_add_u32 s{G.S_LOCL}, s{G.S_LOCL}, 1", SALU, rd=sr(G.S_LOCL), wr=sr(G.S_LOCL) + [("scc", 0)], key=key + 1)]
        ops += self.lslot_advance(S_LDMA, key + 1)
        return ops

    def bases_next(self, l_adv=True):
        """slots and lane bases of the next phase (row reads, transposed reads, chain starts; l_adv:
        the chain-start slot moves on too -- not in phase -1, which reads its slots explicitly)"""
        I = Inst
        nxt = self.slot_advance(S_SROW, key=400) + self.slot_advance(S_STR, key=400)
        if l_adv:
            nxt += self.lslot_advance(S_LRD, key=400)
        nxt += [I(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0), key=401),
                I(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1), key=401),
                I(f"v_add_u32_e32 v{V_VB0}, s{S_STR}, v{V_TB0}", VALU, rd=sr(S_STR) + vr(V_TB0), wr=vr(V_VB0), key=401),
                I(f"v_add_u32_e32 v{V_VB1}, s{S_STR}, v{V_TB1}", VALU, rd=sr(S_STR) + vr(V_TB1), wr=vr(V_VB1), key=401),
                I(f"v_add_u32_e32 v{G.V_LCUR}, s{S_LRD}, v{G.V_LB}", VALU, rd=sr(S_LRD) + vr(G.V_LB), wr=vr(G.V_LCUR), key=401)]
        return nxt

    # ------------------------------------------------------------------ one phase
    def phase2(self, par, first, second, valu, masked=False, q0_add=0, dma=True, nxt=None, first_pref=True,
               init=True, tail_of_step=None):
        """phase p (VALU parity par): the role's MFMAs (first: S(p+1) / dP(p), second: dV(p-1) /
        dK(p-2)), its VALU, the chain starts of the subtile it prepares (P: -LSE(p+2) into TB(par);
        dS: -D(p+1) into TB(1 - par)), one subtile of DMA, the next phase's bases and, nxt = (first,
        second) of the next phase, its first three A fragments"""
        mf = self.mfmas(par, first, second)
        n = len(mf)
        fill = []
        skip = self.pref(mf) if first_pref else []
        for m, (_, t, i) in enumerate(mf):
            if m in skip:
                continue
            fill += self.frag_reads(m, t, i, key=-100 + m, earliest=(m - WIN) if m >= WIN else None,
                                    deadline=max(m - LEAD, 0))
        if valu:
            v = self.valu_p(par, masked, q0_add) if self.role == 0 else self.valu_ds(par)
            if ABL == "noxb":
                v = [x for x in v if "v" + str(V_X) not in x.text.split()[1:2] and f"v{V_X}" not in x.text]
            fill += v
        if init:
            fill += self.init_reads2(TB(par), 0) if self.role == 0 else self.init_reads2(TB(1 - par), 1)
        if dma:
            fill += self.dma2()
        fill += self.bases_next()
        if nxt is not None:
            nm = self.mfmas(1 - par, *nxt)
            for m in self.pref(nm):
                _, t, i = nm[m]
                last_user = max([k for k in range(n) if k % NRING == m % NRING], default=None)
                fill += self.frag_reads(m, t, i, key=600 + m, earliest=last_user)
        if tail_of_step:
            fill += tail_of_step
        return schedule([x[0] for x in mf], fill, budget=BUDGET)

    def vm_phase(self):
        """vmcnt at the end of a phase: everything but the DMA of the last two phases and, for the P
        waves (the only ones loading the LSE / D rows with L_P_ONLY), the L piece before them"""
        return 4 if (self.role == 1 and L_P_ONLY) else VM_PHASE

    def l_wrap(self):
        return [] if (self.role == 1 and L_P_ONLY) else self.wrap_check("l")

    def phase_end(self, wraps=False):
        ins = (self.wrap_check("d") + self.l_wrap()) if wraps else []
        return ins + [Inst(f"s_waitcnt vmcnt({self.vm_phase()}) lgkmcnt(0)", WAIT)] + \
            ([] if ABL == "nobar" else [Inst("s_barrier", BARRIER)])

    def step2(self, first, last, masked):
        """phases A (p = 2n) and B (2n + 1) of step n, each ending in a barrier"""
        if self.role == 0:
            a = self.phase2(0, True, not first, True, masked, 0, nxt=(True, True) if not last else (False, True))
            b = self.phase2(1, not last, True, True, masked, SUB, nxt=(True, True) if not last else (False, True),
                            tail_of_step=self.step_tail_ops())
        else:
            a = self.phase2(0, True, not first, not first, nxt=(True, not first))
            b = self.phase2(1, True, not first, True, nxt=(True, True) if not last else (False, True),
                            tail_of_step=self.step_tail_ops())
        return a + self.phase_end() + b + self.phase_end(wraps=True)

    def tails(self):
        """after the last phase: P waves dV(N-1); dS waves dS(N-1) || dK(N-2), then dK(N-1)"""
        if self.role == 0:
            mf = self.mfmas(0, False, True)
            fill = []
            for m, (_, t, i) in enumerate(mf):
                if m in self.pref(mf):
                    continue
                fill += self.frag_reads(m, t, i, key=-100 + m, earliest=(m - WIN) if m >= WIN else None,
                                        deadline=max(m - LEAD, 0))
            return schedule([x[0] for x in mf], fill, budget=BUDGET)
        a = self.phase2(0, False, True, True, dma=False, init=False, nxt=(False, True))
        mf = self.mfmas(1, False, True)
        fill = []
        for m, (_, t, i) in enumerate(mf):
            if m in self.pref(mf):
                continue
            fill += self.frag_reads(m, t, i, key=-100 + m, earliest=(m - WIN) if m >= WIN else None,
                                    deadline=max(m - LEAD, 0))
        return a + schedule([x[0] for x in mf], fill, budget=BUDGET)

    # ------------------------------------------------------------------ prologue pieces
    def prologue2(self, l_epi):
        """gen_bwd's item prologue, keeping only this role's B-fragment loads (K or V into a[64:95])"""
        ins = self.prologue(l_epi)
        keep = "s[72:75]" if self.role == 0 else "s[76:79]"
        return [x for x in ins if not (x.kind == VLOAD and keep not in x.text)]

    def prologue_dma2(self):
        """LSE / D(0, 1), Q / dO(0), L(2), Q / dO(1), L(3) (then the cursors' head wraps, at even
        counts), Q / dO(2), L(4); phase -1 issues Q / dO(3), L(5), phase p Q / dO(p + 4), L(p + 6)"""
        loads_l = self.role == 0 or not L_P_ONLY
        ins = (self.dma_l_only() + self.dma_l_only() + self.wrap_check("l")) if loads_l else []
        ins += self.dma2(eg=None) + self.dma2(eg=None) + self.wrap_check("d") + self.l_wrap()
        ins += [Inst(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i)) for i in range(64)]
        ins += self.dma2(eg=None)
        return ins

    def dma_l_only(self):
        ops = super().dma_l_only()
        return ops

    def phase_m1(self):
        """phase -1: P waves: chain starts -LSE(0), -LSE(1), S(0); dS waves: -D(0); both: DMA of
        Q / dO(3), L(5); the ring read slots of phase 0"""
        I = Inst
        if self.role == 0:
            srow, stro = 0, G.RING - 2 * SLOT          # slots of subtiles 0 (rows), -2 (transposed)
        else:
            srow, stro = G.RING - SLOT, G.RING - 3 * SLOT   # -1 (rows), -3 (transposed)
        ph = [I(f"s_mov_b32 s{S_SROW}, {srow}", SALU, wr=sr(S_SROW)),
              I(f"s_mov_b32 s{S_STR}, {stro}", SALU, wr=sr(S_STR)),
              I(f"s_mov_b32 s{S_LRD}, {G.LBASE}", SALU, wr=sr(S_LRD)),
              I(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0)),
              I(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1)),
              I(f"v_add_u32_e32 v{G.V_LCUR}, s{S_LRD}, v{G.V_LB}", VALU, rd=sr(S_LRD) + vr(G.V_LB), wr=vr(G.V_LCUR))]
        def adv():
            return self.lslot_advance(S_LRD) + [I(f"v_add_u32_e32 v{G.V_LCUR}, s{S_LRD}, v{G.V_LB}", VALU,
                                                  rd=sr(S_LRD) + vr(G.V_LB), wr=vr(G.V_LCUR))]
        if self.role == 0:
            ini0 = self.init_reads2(TB(0), 0)
            for op in ini0:
                op.dl = 0
            ph += ini0 + adv() + self.init_reads2(TB(1), 0) + adv()
            mf = self.mfmas(1, True, False)          # S(0) -> TB(0)
            nxt = (True, False)                       # phase 0: S(1) only
        else:
            ph += self.init_reads2(TB(0), 1) + adv()
            mf = []
            nxt = (True, False)                       # phase 0: dP(0) only
        fill = []
        for m, (_, t, i) in enumerate(mf):
            fill += self.frag_reads(m, t, i, key=-100 + m, deadline=max(m - 2, 0))
        fill += self.dma2()
        fill += self.bases_next(l_adv=False)
        nm = self.mfmas(0, *nxt)
        for m in self.pref(nm):
            _, t, i = nm[m]
            fill += self.frag_reads(m, t, i, key=600 + m, earliest=m if mf else None)
        sch = schedule([x[0] for x in mf], ph + fill, budget=BUDGET)
        return sch + self.phase_end(wraps=True)

    def epilogue2(self):
        """gen_bwd's epilogue for this role's accumulator only: dV (P waves) or scale dK (dS waves)"""
        I = Inst
        ins = [I("s_waitcnt vmcnt(0)", WAIT)]
        stash = G.V_ST
        KW0v, HDv, DKO, DVO, PDK, PDV, RDK, RDV, HDK, HDV, SKv = (stash + i for i in (0, 1, 2, 4, 6, 8, 10, 11, 12, 13, 14))
        T0, T1, T2, T3, T4, T5, T6 = (S_TMP + i for i in range(7))

        def rf(v, s):
            return I(f"v_readfirstlane_b32 s{s}, v{v}", RFL, rd=vr(v), wr=sr(s))

        def sa(op, d, a, b, extra_rd=()):
            return I(f"{op} s{d}, s{a}, s{b}", SALU, rd=sr(a) + sr(b) + list(extra_rd), wr=sr(d) + [("scc", 0)])

        ins += [rf(KW0v, T4), rf(HDv, T5), rf(SKv, T6)]
        dst = S_QD
        ptr, off, rowv, headv, scale = (PDV, DVO, RDV, HDV, False) if self.role == 0 else (PDK, DKO, RDK, HDK, True)
        ins += [rf(ptr, T0), rf(ptr + 1, T1), rf(off, T2), rf(off + 1, T3),
                sa("s_add_u32", T0, T0, T2), sa("s_addc_u32", T1, T1, T3, [("scc", 0)]),
                rf(headv, T2),
                sa("s_mul_i32", T3, T5, T2), sa("s_mul_hi_u32", T2, T5, T2),
                sa("s_add_u32", T0, T0, T3), sa("s_addc_u32", T1, T1, T2, [("scc", 0)]),
                rf(rowv, T2),
                sa("s_mul_i32", T3, T4, T2), sa("s_mul_hi_u32", dst + 3, T4, T2),
                sa("s_add_u32", dst, T0, T3), sa("s_addc_u32", dst + 1, T1, dst + 3, [("scc", 0)]),
                I(f"s_and_b32 s{dst + 1}, s{dst + 1}, 0xffff", SALU, rd=sr(dst + 1), wr=sr(dst + 1)),
                sa("s_sub_i32", T3, T6, T4),
                I(f"s_max_i32 s{T3}, s{T3}, 0", SALU, rd=sr(T3), wr=sr(T3)),
                sa("s_mul_i32", dst + 2, T3, T2),
                I(f"s_mov_b32 s{dst + 3}, 0x20000", SALU, wr=sr(dst + 3)),
                I(f"v_and_b32_e32 v{G.V_TMP}, 31, v{G.V_LANE}", VALU, rd=vr(G.V_LANE), wr=vr(G.V_TMP)),
                I(f"v_mul_lo_u32 v{G.V_TMP}, v{G.V_TMP}, s{T2}", VALU, rd=vr(G.V_TMP) + sr(T2), wr=vr(G.V_TMP)),
                I(f"v_lshrrev_b32_e32 v{G.V_TMP + 1}, 5, v{G.V_LANE}", VALU, rd=vr(G.V_LANE), wr=vr(G.V_TMP + 1)),
                I(f"v_lshl_add_u32 v{G.V_TMP + 2}, v{G.V_TMP + 1}, 4, v{G.V_TMP}", VALU, rd=vr(G.V_TMP, 2), wr=vr(G.V_TMP + 2))]
        x = 0
        for dt in range(G.NP):
            for u0 in (0, 2):
                w = x + 8
                for uu in range(2):
                    a = ACC + 16 * dt + 4 * (u0 + uu)
                    xs = x + 4 * uu
                    ins += [I(f"v_accvgpr_read_b32 v{xs + k}, a{a + k}", G.ACCR, rd=ar(a + k), wr=vr(xs + k)) for k in range(4)]
                    if scale:
                        ins += [I(f"v_mul_f32_e32 v{xs + k}, s{G.S_SCALE}, v{xs + k}", VALU, rd=sr(G.S_SCALE) + vr(xs + k), wr=vr(xs + k))
                                for k in range(4)]
                    ins += [self.cvt(w + 2 * uu, xs, xs + 1), self.cvt(w + 2 * uu + 1, xs + 2, xs + 3)]
                ins += [I(f"v_permlane32_swap_b32_e32 v{w}, v{w + 2}", G.PERM, rd=vr(w) + vr(w + 2), wr=vr(w) + vr(w + 2)),
                        I(f"v_permlane32_swap_b32_e32 v{w + 1}, v{w + 3}", G.PERM, rd=vr(w + 1) + vr(w + 3), wr=vr(w + 1) + vr(w + 3))]
                ins.append(I(f"buffer_store_dwordx4 v[{w}:{w + 3}], v{G.V_TMP + 2}, s[{dst}:{dst + 3}], 0 offen offset:{64 * dt + 16 * u0}",
                             VSTORE, rd=vr(w, 4) + vr(G.V_TMP + 2) + sr(dst, 4)))
                x = (x + 12) % 60
        return ins

    # ------------------------------------------------------------------ one role's item loop
    def body(self, code, emit):
        self.lab_next = self.lab("next")
        l_epi = self.lab("epi")
        l_item = self.lab("item")
        code.append(label(l_item))
        T0, T1, T2, T3, T4 = (S_TMP + i for i in range(5))
        head = [Inst("s_barrier", BARRIER),
                Inst(f"s_load_dwordx2 s[{T1}:{T2}], s[0:1], {G.NITEMS_OFF}", SMEM),
                Inst(f"v_readfirstlane_b32 s{T0}, v{G.V_ROUND}", RFL),
                Inst("s_waitcnt lgkmcnt(0)", WAIT)]
        head += self.n_items_ops(T1)
        head += item_pos_ops(G.S_ITEM, T0, 2, T2, T3, T4)
        head += [Inst(f"s_cmp_ge_u32 s{G.S_ITEM}, s{T1}", SALU), Inst(f"s_cbranch_scc1 {self.lab_end}", BRANCH)]
        ool0 = len(self.ool)
        pro = head + self.prologue2(l_epi)
        # (the out-of-line empty-item block zeroes a[0:127]: harmless, it only stores zeros)
        assert len(self.ool) >= ool0
        pro += self.prologue_dma2()
        # Q / dO(0), LSE / D(0, 1) landed; younger than Q / dO(0): L2, Q1, L3, Q2, L4 = 7
        pro += [Inst(f"s_waitcnt vmcnt({self.vm_phase()})", WAIT), Inst("s_barrier", BARRIER)]
        emit(pro, pre=[nop(15)])
        emit(self.phase_m1(), pre=[nop(15)])
        L = {}
        masks = (True, False) if (self.causal and self.role == 0) else (False,)
        variants = [(f, l, m) for f in (True, False) for l in (True, False) for m in masks
                    if not (f and self.causal and self.role == 0 and not m)]
        for v in variants:
            L[v] = self.lab("step_" + ("".join(c for c, on in zip("FLM", v) if on) or "R"))
        l_tail, l_disp, l_notlast = self.lab("tail"), self.lab("dispatch"), self.lab("notlast")
        fm = self.causal and self.role == 0
        code += [Inst(f"s_cmp_eq_u32 s{G.S_NLAST}, 0", SALU), Inst(f"s_cbranch_scc1 {L[(True, True, fm)]}", BRANCH),
                 Inst(f"s_branch {L[(True, False, fm)]}", BRANCH)]
        code += [label(l_disp), Inst(f"s_cmp_gt_u32 s{G.S_N}, s{G.S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_tail}", BRANCH),
                 Inst(f"s_cmp_lt_u32 s{G.S_N}, s{G.S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_notlast}", BRANCH)]
        if fm:
            code += [Inst(f"s_cmp_lt_u32 s{G.S_LOCV}, 4", SALU), Inst(f"s_cbranch_scc1 {L[(False, True, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, True, False)]}", BRANCH), label(l_notlast)]
        if fm:
            code += [Inst(f"s_cmp_lt_u32 s{G.S_LOCV}, 4", SALU), Inst(f"s_cbranch_scc1 {L[(False, False, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, False, False)]}", BRANCH)]
        pad = [nop(15)]
        for v in variants:
            f, l, m = v
            code.append(label(L[v]))
            emit(self.step2(f, l, m), pre=pad)
            code.append(Inst(f"s_branch {l_disp}", BRANCH))
        code.append(label(l_tail))
        emit(self.tails(), pre=pad)
        code.append(label(l_epi))
        emit([nop(15)] + self.epilogue2(), pre=pad)
        code.append(label(self.lab_next))
        code += [Inst(f"v_add_u32_e32 v{G.V_ROUND}, 1, v{G.V_ROUND}", VALU), Inst(f"s_branch {l_item}", BRANCH)]

    def build(self):
        self.ool = []
        code = []

        def emit(insts, pre=()):
            out, _ = add_waits(insts)
            out, _ = fix_hazards(out, pre=pre)
            code.extend(out)

        l_ds = self.lab("role_ds")
        T0 = S_TMP
        start = [Inst("v_lshrrev_b32_e32 v1, 6, v0", VALU, rd=vr(0), wr=vr(1)),
                 Inst(f"v_readfirstlane_b32 s{G.S_WAVE}, v1", RFL, rd=vr(1), wr=sr(G.S_WAVE)),
                 Inst(f"v_and_b32_e32 v{G.V_LANE}, 63, v0", VALU, rd=vr(0), wr=vr(G.V_LANE)),
                 Inst(f"v_mov_b32_e32 v{G.V_ROUND}, 0", VALU, wr=vr(G.V_ROUND)),
                 Inst(f"s_lshr_b32 s{T0}, s{G.S_WAVE}, 2", SALU, rd=sr(G.S_WAVE), wr=sr(T0)),
                 Inst(f"s_and_b32 s{G.S_WAVE}, s{G.S_WAVE}, 3", SALU, rd=sr(G.S_WAVE), wr=sr(G.S_WAVE)),
                 # the P exchange lane address: XBASE + 4096 kg + 16 lane
                 Inst(f"s_lshl_b32 s{T0 + 1}, s{G.S_WAVE}, 12", SALU, rd=sr(G.S_WAVE), wr=sr(T0 + 1)),
                 Inst(f"s_add_u32 s{T0 + 1}, s{T0 + 1}, {XBASE}", SALU, rd=sr(T0 + 1), wr=sr(T0 + 1)),
                 Inst(f"v_lshlrev_b32_e32 v{V_X}, 4, v{G.V_LANE}", VALU, rd=vr(G.V_LANE), wr=vr(V_X)),
                 Inst(f"v_add_u32_e32 v{V_X}, s{T0 + 1}, v{V_X}", VALU, rd=sr(T0 + 1) + vr(V_X), wr=vr(V_X)),
                 Inst(f"s_cmp_eq_u32 s{T0}, 0", SALU, rd=sr(T0), wr=[("scc", 0)]),
                 Inst(f"s_cbranch_scc0 {l_ds}", BRANCH)]
        emit(start)
        if PRIO == "p":      # (the P body follows the branch)
            code.append(Inst("s_setprio 1", SOPP))
        self.lab_end = self.lab("end")
        self.role = 0
        self.body(code, emit)
        code.append(label(self.lab_end))
        code.append(Inst("s_endpgm", SOPP))
        code.append(label(l_ds))
        if PRIO == "ds":
            code.append(Inst("s_setprio 1", SOPP))
        self.role = 1
        self.lab_end = self.lab("end")
        self.body(code, emit)
        code.append(label(self.lab_end))
        code.append(Inst("s_endpgm", SOPP))
        code.extend(self.ool)
        return code

    def render(self):
        code = self.build()
        out = [f"\t.globl {self.name}", "\t.p2align 8", f"\t.type {self.name},@function", f"{self.name}:"]
        for ins in code:
            out.append(ins.text if ins.kind == _isa.LABEL else "\t" + ins.text)
        out.append(f".L{self.name}_fend:")
        out.append(f"\t.size {self.name}, .L{self.name}_fend-{self.name}")
        return "\n".join(out)

    def descriptor(self):
        return f"""
	.rodata
	.p2align 6
	.amdhsa_kernel {self.name}
		.amdhsa_group_segment_fixed_size {G.LDS_BYTES}
		.amdhsa_private_segment_fixed_size 0
		.amdhsa_kernarg_size {G.KARG_SIZE}
		.amdhsa_user_sgpr_count 2
		.amdhsa_user_sgpr_kernarg_segment_ptr 1
		.amdhsa_system_sgpr_workgroup_id_x 1
		.amdhsa_system_vgpr_workitem_id 0
		.amdhsa_next_free_vgpr 256
		.amdhsa_next_free_sgpr {G.NSGPR}
		.amdhsa_accum_offset {NVGPR}
		.amdhsa_reserve_vcc 1
		.amdhsa_float_denorm_mode_32 3
		.amdhsa_float_denorm_mode_16_64 3
		.amdhsa_dx10_clamp 1
		.amdhsa_ieee_mode 0
	.end_amdhsa_kernel
	.text
"""

    def metadata(self):
        return f"""  - .agpr_count: 128
    .args:
      - .offset: 0
        .size: {G.KARG_SIZE}
        .value_kind: by_value
    .group_segment_fixed_size: {G.LDS_BYTES}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {G.KARG_SIZE}
    .max_flat_workgroup_size: 512
    .name: {self.name}
    .private_segment_fixed_size: 0
    .sgpr_count: {G.NSGPR + 2}
    .sgpr_spill_count: 0
    .symbol: {self.name}.kd
    .uniform_work_group_size: 1
    .vgpr_count: 256
    .vgpr_spill_count: 0
    .wavefront_size: 64
"""


def main():
    kernels = [K2(bf, ca, u) for u in (False, True) for bf in (True, False) for ca in (True, False)]
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
