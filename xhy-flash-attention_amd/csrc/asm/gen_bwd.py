#!/usr/bin/env python3
"""Generates fa_bwd_asm.s: the gfx950 FlashAttention-2 dK / dV kernel for head dim 128, written as a
hand-scheduled assembly kernel (one wave per SIMD); gen_bwd64.py (head dim 64) and gen_bwd2.py (two
waves per SIMD) build on it.

    python3 gen_bwd.py > fa_bwd_asm.s

Algorithm: the reference's dK / dV half of compute_dq_dk_dv_1colblock
(csrc/flash_attn/src/flash_bwd_kernel.h:421-1046) for one block of keys, swept over every query row
that can see them (and, for GQA with a reduced dK / dV, over every query head of the group):
    S' = Q K^T - LSE / scale          (chain started from -LSE / scale)
    P  = exp2(c S')                   (c = scale log2 e; -inf where the causal mask hides the key;
                                       the _c1 kernels: c = 1, Q = the forward's bf16/f16(c Q))
    dP' = dO V^T - D                  (chain started from -D, D = rowsum(dO o O))
    dS = P o dP'
    dV^T += dO^T P,   dK^T += Q^T dS  (dK = scale dK^T^T at the end)

MI355X structure (cdna_hip_programming.md "one wave per SIMD", as the assembly forward gen_fwd.py):
  * workgroup = 4 waves x 32 keys = a 128-key block; each wave keeps its keys' operands and results in
    its 512 registers for the whole sweep:
      a[0:63] dV^T, a[64:127] dK^T (4 d-tiles x 16), a[128:159] K fragments, a[160:191] V fragments
      (B operands of S = Q K^T and dP = dO V^T: the key is the MFMA column), a[192:255] a ring of 16
      A-operand fragments read from LDS;
      v[0:63] S / dP tiles (two buffers), v[64:79] exp / dS temporaries, v[80:111] packed P and dS
      (two buffers: the B operands of dV^T and dK^T).
  * the query rows stream through LDS in 32-row subtiles (Q and dO, 16 KiB, a 9-slot ring) plus the
    subtile's -LSE/scale and -D rows (256 B, a 16-slot ring), by LDS-DMA (buffer_load ... lds), 6 / 8
    subtiles ahead; one s_waitcnt + s_barrier per step of two subtiles.
  * phase p (32 MFMAs, v_mfma_f32_32x32x16):  S(p+1), dP(p+1)  ||  dV^T, dK^T += ..(p-1)  and, in the
    gaps, the VALU of subtile p (P, dS, their bf16 / f16 packs), the LDS reads of every A operand
    (Q / dO rows with ds_read_b128, dO^T / Q^T with ds_read_b64_tr_b16), the chain starts of p+2 and
    the DMA of later subtiles -- placed by isa.schedule, hazards by isa.fix_hazards, waits by
    isa.add_waits.
  * causal: the sweep starts at the block's first key (rows above it see none of its keys); the first
    4 subtiles of each head's sweep cross the diagonal and run a MASKED step variant.  Rows past
    seqlen_q read zero Q / dO / LSE / D (range-checked descriptors) and contribute nothing; keys past
    seqlen_k are computed on zero K / V and never stored.
  * work order: a host-built table (block -> batch, head, kv head, key block), heaviest causal blocks
    first, the blocks of one head on one XCD (fa_common.h xcd_order).
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
_isa.apply_costs(os.environ.get("FA_GBW_COST", ""))
D = 128
KS = D // 16            # k-steps of S / dP
NP = D // 32            # d-tiles of dV^T / dK^T
SUB = 32                # query rows per subtile
BKN = 128               # keys per workgroup
QT = SUB * D * 2        # bytes of a Q (or dO) subtile = 8 KiB
SLOT = 2 * QT           # Q | dO
NS = int(os.environ.get("FA_GBW_NS", "9"))   # Q / dO ring slots (a power of two wraps with one s_and)
RING = NS * SLOT        # 147456
LBASE = RING            # -LSE/scale | -D ring (16 x 256 B)
NLS = 16
LSLOT = 256
LDS_BYTES = LBASE + NLS * LSLOT
assert LDS_BYTES <= 163840 and LBASE % 4096 == 0
KQ = 6                  # Q / dO subtile s is DMA'd in step (s - KQ) / 2
KL = 8                  # LSE / D subtile s in step (s - KL) / 2
# Outstanding VMEM ops allowed at the end of step n-1: step n reads the rows of Q / dO subtiles up to
# 2n+3 (phase 2n+1 reads 2n+2; its tail prefetches the first fragments of 2n+3) and the chain starts
# of LSE / D subtiles up to 2n+3.  Issue order per step m: Q/dO(2m+6) [4], L(2m+8) [1], Q/dO(2m+7) [4],
# L(2m+9) [1]; younger than Q/dO(2n+3) (issued in step n-2) at the end of step n-1: L(2n+5) and the
# 10 of step n-1.
VMCNT_STEP = 11

# ---- AGPRs ----
DV = 0
DK = 64
KF = 128
VF = 160
RG = 192                # 16 x 4 ring


def ring(m):
    return RG + 4 * (m % 16)


# ---- VGPRs ----
def SB(par):
    return 16 * par


def DPB(par):
    return 32 + 16 * par


T = 64                  # 16 temporaries (exp / dS of the VALU subtile)


def PP(par):
    return 80 + 8 * par


def DSP(par):
    return 96 + 8 * par


V_RB0, V_RB1, V_TB0, V_TB1 = 112, 113, 114, 115     # lane LDS bases (no slot)
V_KB0, V_KB1, V_VB0, V_VB1 = 116, 117, 118, 119     # current row-read / transposed-read bases
V_LB = 120              # lane part of the chain-start reads (16 hh)
V_LCUR = 121            # chain-start read base of the subtile two ahead
V_QV0, V_QV1, V_OV0, V_OV1 = 122, 123, 124, 125     # DMA voffsets (Q, dO; halves 0 / 1)
V_L4 = 126              # 4 lane (LSE / D DMA)
V_LANEK = 127           # key - 4 hh (mask)
V_LM = 128              # mask limit of the VALU subtile
V_NINF = 129
V_LANE = 130
V_TMP = 131             # prologue temporaries 131..138
V_ST = 144              # the epilogue's scalars, stashed (144..158)
NVGPR = 159

# ---- SGPRs ----
S_QD, S_OD, S_LD = 4, 8, 12          # DMA cursors (buffer descriptors)
S_C = 16                             # scale log2 e
S_SCALE = 17
S_SROW, S_STR, S_SDMA, S_LRD, S_LDMA = 18, 19, 20, 21, 22   # ring offsets
S_W2K = 23                           # wave * 2048
S_N, S_NLAST = 24, 25                # step, last step index
S_LOCV, S_Q0V, S_QF, S_NSP = 26, 27, 28, 29
S_LOCD, S_HLD, S_LOCL, S_HLL = 30, 31, 32, 33
S_QH, S_OH, S_LH = 34, 36, 38        # head bases (64-bit)
S_QREC0, S_OREC0, S_LREC0 = 40, 41, 42
S_QHS, S_OHS, S_LHS = 43, 44, 45     # head strides (bytes)
S_Q32, S_O32 = 46, 47                # 32 rows of Q / dO (bytes)
S_WAVE = 48
S_TMP = 49                           # 49..55 (the prologue keeps kernargs in 56..101)
NSGPR = 102

KARG_SIZE = 272
DEC_OFF = 224    # fa_params.h ItemDecode (40 bytes) after BwdAsmArgs' 224
NITEMS_OFF = 264  # n_items, grid (persistent item loop)

# dev A/B switches, read when the .s is generated (tools/asm_variant.sh)
OPT_WIN = int(os.environ.get("FA_GBW_WIN", "16"))     # an A fragment may be read up to WIN MFMAs ahead
# (a read more than 16 MFMAs ahead would overwrite the ring slot (16 fragments) an earlier MFMA
# still reads: the scheduler orders fillers among themselves, the MFMA sequence only by earliest)
assert 2 <= OPT_WIN <= 16, "FA_GBW_WIN must be within the 16-slot fragment ring"
OPT_LEAD = int(os.environ.get("FA_GBW_LEAD", "2"))    # ... and at least LEAD MFMAs ahead
OPT_DECBURST = os.environ.get("FA_GBW_DECBURST") == "1"
# dev timeline: every workgroup stores {start, end} s_memtime, HW_ID, XCC_ID, id at the `stamps`
# kernarg address + 32 id (tools/bwd_stamps.py)
OPT_STAMP = os.environ.get("FA_GBW_STAMP") == "1"
# FA_GBW_STAMP=2: per wave, over all its items, the cycles of the steps' compute, their end-of-step
# vmcnt wait and barrier, the prologues (item start .. phase -1's barrier) and the tails + epilogues;
# record (workgroup * 4 + wave) * 64 bytes at the `stamps` kernarg (tools/bwd_stamps.py --steps)
OPT_STEPSTAMP = os.environ.get("FA_GBW_STAMP") == "2"
# dV^T / dK^T zeroed after the first subtiles' DMAs are issued (under their latency) instead of ahead
OPT_ZLATE = os.environ.get("FA_GBW_ZEARLY") != "1"
# ablations (wrong results; which resource bounds the steady state): novalu / nofrag / nodma
OPT_ABL = os.environ.get("FA_GBW_ABL", "")
V_SS = 186             # 186..193: compute, wait, barrier, steps, last stamp, prologue, epilogue, items
                       # (194, 195: temporaries); 196..201: the prologue's parts (head, kernargs + work
                       # order, geometry, fragment loads + lane values, DMA issue, first wait; phase -1 is
                       # `prologue` above)
V_ROUND = 184          # round r of the persistent item loop (uniform)
S_ITEM = 28            # the item index, until the sweep geometry takes the register (S_QF)
V_STAMP = 164          # 164..177: start lo / hi, HW_ID, XCC_ID, wg, end lo / hi, wave, -, -, loop start lo / hi,
                       # epilogue start lo / hi (with OPT_STAMP)

# ---- the pipelined item loop (OPT_CONT): the DMA of the next item's first subtiles and the loads of
# its K / V fragments run under the current item's last steps; the next item's geometry is computed
# at the start of the current one (geometry(), into the record N) ----
# (dev switch, off: C3 +-0, C4 +1..3 % -- the last step's K / V loads and slower steps ate the
# prologue it saves, profiles/r05/ab_cont_*_r05h.txt)
OPT_CONT = os.environ.get("FA_GBW_CONT", "0") == "1"
V_N = 202               # record of the next item (202..236), fields:
N_QH, N_OH, N_LH = 0, 2, 4          # head bases (64-bit)
N_QREC, N_OREC, N_LREC, N_NSP = 6, 7, 8, 9
N_KD, N_VD = 10, 13                 # K / V fragment descriptors (base lo, hi, records)
N_QF, N_NLAST, N_LANEK = 16, 17, 18
N_ST = 19                           # the epilogue's scalars (15, as V_ST)
N_HL0 = 34                          # heads of the sweep - 1
N_LEN = 35
V_C = 64                # the record of the item starting (transient, at the item switch: v64..98)
V_SAVE = 0              # the DMA side's registers across geometry() (v0..v32, at the item switch)
V_ZERO = 140            # 140..143: zeros (the stores of an item with keys and no rows)
V_KLO, V_VLO = 160, 161 # lane offsets of the K / V fragment loads (launch constants)
# where the next item's K / V fragment loads go (dev A/B): the last step's phase B, the tail, the epilogue
OPT_KVAT = os.environ.get("FA_GBW_KVAT", "last")
# DMA-side registers of the pipelined loop (beside S_QD .. S_LREC0); the kernarg block s56.. is free
# during the steps, geometry() clobbers them (saved across it)
S_NSPD, S_NSPL = (96, 97) if OPT_CONT else (S_NSP, S_NSP)   # subtiles per head of the DMA cursors' items
S_DSW, S_LSW = 98, 99              # the cursor has switched to the next item (ahead of the compute)
S_DSTALL, S_LSTALL = 100, 101      # slot where the cursor stalled (-1: running): a second switch must
                                   # wait for the item switch, which re-issues the stalled subtiles
S_KVN = 88                         # 88..95: the next item's K / V descriptors
S_EPD = 80                         # 80..87: the epilogue's store descriptors
# ... and the launch constants the DMA uses: a geometry() pass that ends on an item without keys or on
# no item at all leaves them clobbered (the work order's loads land in s36..45)
DMA_SIDE = (list(range(S_QD, S_QD + 12)) + [S_SDMA, S_LDMA, S_LOCD, S_HLD, S_LOCL, S_HLL] +
            list(range(S_QH, S_QH + 6)) + [S_QREC0, S_OREC0, S_LREC0, S_NSPD, S_NSPL, S_DSW, S_LSW, S_DSTALL, S_LSTALL] +
            [S_W2K, S_QHS, S_OHS, S_LHS, S_Q32, S_O32])


class K:
    """one kernel variant"""

    def __init__(self, bf16, causal, unit_c=False):
        self.bf16 = bf16
        self.causal = causal
        # unit_c: the launch passes c = 1 (the backward of a forward that held Q as bf16/f16(c Q): the
        # Q rows are the prescaled Q', launch_bwd), so P = exp2(S') with no multiply per score
        self.unit_c = unit_c
        self.ty = "bf16" if bf16 else "f16"
        self.name = f"fa_bwd_dkdv_asm_d{D}_{self.ty}_{'causal' if causal else 'full'}{'_c1' if unit_c else ''}"
        self.uid = 0

    def lab(self, s):
        self.uid += 1
        return f".L{self.name}_{s}_{self.uid}"

    # ------------------------------------------------------------------ MFMA builders
    def mf(self, dst, a, b, acc_kind):
        """D = A B + D (chain); dst / a / b are (kind, base) pairs"""
        dk, dr = dst
        ak, ab = a
        bk, bb = b
        t = (f"v_mfma_f32_32x32x16_{self.ty} {rtxt(dk, dr, 16)}, {rtxt(ak, ab, 4)}, {rtxt(bk, bb, 4)}, "
             f"{rtxt(dk, dr, 16)}")
        regs = {"v": vr, "a": ar}
        d = regs[dk](dr, 16)
        return Inst(t, MFMA, rd=regs[ak](ab, 4) + regs[bk](bb, 4) + d, wr=d, rd_c=d)

    def phase_mfmas(self, par, sdp, dvdk):
        """(mfma list, list of (m, kind, args)) for a phase; par = parity of the VALU subtile p:
        S / dP(p+1) write buffers 1 - par, dV / dK(p-1) read packs 1 - par"""
        out = []
        nb = 1 - par
        if sdp and dvdk:
            order = [(t, i) for i in range(8) for t in ("S", "dV", "dP", "dK")]
        elif sdp:
            order = [(t, i) for i in range(8) for t in ("S", "dP")]
        else:
            order = [(t, i) for i in range(8) for t in ("dV", "dK")]
        for m, (t, i) in enumerate(order):
            if t == "S":
                out.append((self.mf(("v", SB(nb)), ("a", ring(m)), ("a", KF + 4 * i), "v"), t, i))
            elif t == "dP":
                out.append((self.mf(("v", DPB(nb)), ("a", ring(m)), ("a", VF + 4 * i), "v"), t, i))
            elif t == "dV":
                dt, kk = i // 2, i % 2
                out.append((self.mf(("a", DV + 16 * dt), ("a", ring(m)), ("v", PP(nb) + 4 * kk), "a"), t, i))
            else:
                dt, kk = i // 2, i % 2
                out.append((self.mf(("a", DK + 16 * dt), ("a", ring(m)), ("v", DSP(nb) + 4 * kk), "a"), t, i))
        return out

    def frag_reads(self, m, t, i, **kw):
        """LDS read(s) of the A operand of MFMA m (type t, index i) into its ring slot"""
        dst = ring(m)
        if t in ("S", "dP"):
            base = V_KB0 if i % 2 == 0 else V_KB1
            off = (i // 2) * 2048 + (QT if t == "dP" else 0)
            return [Inst(f"ds_read_b128 {rtxt('a', dst, 4)}, v{base} offset:{off}", LDS,
                         rd=vr(base), wr=ar(dst, 4), **kw)]
        dt, kk = i // 2, i % 2
        out = []
        for h in range(2):
            base = V_VB0 if h == 0 else V_VB1
            off = (QT if t == "dV" else 0) + dt * 2048 + kk * 1024 + h * 512
            out.append(Inst(f"ds_read_b64_tr_b16 {rtxt('a', dst + 2 * h, 2)}, v{base} offset:{off}", LDS,
                            rd=vr(base), wr=ar(dst + 2 * h, 2), **kw))
        return out

    def cvt(self, dst, s0, s1, **kw):
        return Inst(f"v_cvt_pk_{self.ty}_f32 v{dst}, v{s0}, v{s1}", VALU, rd=vr(s0) + vr(s1), wr=vr(dst), **kw)

    # ------------------------------------------------------------------ VALU of one subtile
    def valu_ops(self, par, masked, q0_add):
        """P, dS of the subtile in buffers `par` -> packs `par`; q0 of the subtile = S_Q0V + q0_add"""
        ops = []
        S, DP, PK, DSK = SB(par), DPB(par), PP(par), DSP(par)
        if masked:
            ops.append(Inst(f"v_subrev_u32 v{V_LM}, s{S_Q0V}, v{V_LANEK}", VALU, rd=sr(S_Q0V) + vr(V_LANEK),
                            wr=vr(V_LM), key=0))
            if q0_add:
                ops.append(Inst(f"v_subrev_u32 v{V_LM}, {q0_add}, v{V_LM}", VALU, rd=vr(V_LM), wr=vr(V_LM), key=0))
        for g in range(16):
            src = T + g      # the exponent's operand
            if not self.unit_c:
                ops.append(Inst(f"v_mul_f32_e32 v{T + g}, s{S_C}, v{S + g}", VALU, rd=sr(S_C) + vr(S + g), wr=vr(T + g),
                                key=4 * g))
            elif not masked:
                src = S + g
            if masked:
                const = (g & 3) + 8 * (g >> 2)
                ops.append(Inst(f"v_cmp_lt_i32_e32 vcc, {const}, v{V_LM}", VALU, rd=vr(V_LM), wr=[("vcc", 0)], key=4 * g))
                x = S + g if self.unit_c else T + g
                ops.append(Inst(f"v_cndmask_b32_e32 v{T + g}, v{x}, v{V_NINF}, vcc", VALU,
                                rd=vr(x) + vr(V_NINF) + [("vcc", 0)], wr=vr(T + g), key=4 * g))
            ops.append(Inst(f"v_exp_f32_e32 v{T + g}, v{src}", TRANS, rd=vr(src), wr=vr(T + g), key=4 * g + 1))
            if g % 2 == 1:
                ops.append(self.cvt(PK + g // 2, T + g - 1, T + g, key=4 * g + 2))
        for g in range(16):
            ops.append(Inst(f"v_mul_f32_e32 v{T + g}, v{T + g}, v{DP + g}", VALU, rd=vr(T + g) + vr(DP + g),
                            wr=vr(T + g), key=64 + 2 * g))
            if g % 2 == 1:
                ops.append(self.cvt(DSK + g // 2, T + g - 1, T + g, key=64 + 2 * g + 1))
        return ops

    def init_reads(self, par):
        """chain starts of the subtile two ahead (-LSE/scale -> S buffer par, -D -> dP buffer par)"""
        ops = []
        for u in range(4):
            ops.append(Inst(f"ds_read_b128 v[{SB(par) + 4 * u}:{SB(par) + 4 * u + 3}], v{V_LCUR} offset:{32 * u}", LDS,
                            rd=vr(V_LCUR), wr=vr(SB(par) + 4 * u, 4), key=200))
        for u in range(4):
            ops.append(Inst(f"ds_read_b128 v[{DPB(par) + 4 * u}:{DPB(par) + 4 * u + 3}], v{V_LCUR} offset:{128 + 32 * u}",
                            LDS, rd=vr(V_LCUR), wr=vr(DPB(par) + 4 * u, 4), key=300))
        return ops

    # ------------------------------------------------------------------ DMA of one subtile
    def dma_subtile(self, with_l, key=-50, eg=None):
        """Q / dO pieces of the next DMA subtile (slot S_SDMA) and, with_l, the LSE / D rows of the
        LSE cursor's subtile (slot S_LDMA); then advance the cursors and slots"""
        t = S_TMP
        I = Inst
        ops = [I(f"s_add_u32 s{t}, s{S_SDMA}, s{S_W2K}", SALU, rd=sr(S_SDMA) + sr(S_W2K), wr=sr(t) + [("scc", 0)], key=key)]
        for j, (voff, desc, add) in enumerate(((V_QV0, S_QD, 0), (V_QV1, S_QD, 1024), (V_OV0, S_OD, QT),
                                               (V_OV1, S_OD, QT + 1024))):
            e = None if eg is None else eg + 2 * j
            ops.append(I(f"s_add_u32 m0, s{t}, {add}", SALU, rd=sr(t), wr=[("m0", 0)] + [("scc", 0)], key=key, earliest=e))
            ops.append(I(f"buffer_load_dwordx4 v{voff}, s[{desc}:{desc + 3}], 0 offen lds", DMA,
                         rd=vr(voff) + sr(desc, 4) + [("m0", 0)], key=key, earliest=e))
        if with_l:
            e = None if eg is None else eg + 8
            ops.append(I(f"s_mov_b32 m0, s{S_LDMA}", SALU, rd=sr(S_LDMA), wr=[("m0", 0)], key=key, earliest=e))
            ops.append(I(f"buffer_load_dword v{V_L4}, s[{S_LD}:{S_LD + 3}], 0 offen lds", DMA,
                         rd=vr(V_L4) + sr(S_LD, 4) + [("m0", 0)], key=key, earliest=e))
        # cursors: base += 32 rows, records = max(records - 32 rows, 0)
        for desc, step in ((S_QD, S_Q32), (S_OD, S_O32)):
            ops += [I(f"s_add_u32 s{desc}, s{desc}, s{step}", SALU, rd=sr(desc) + sr(step), wr=sr(desc) + [("scc", 0)], key=key + 1),
                    I(f"s_addc_u32 s{desc + 1}, s{desc + 1}, 0", SALU, rd=sr(desc + 1) + [("scc", 0)], wr=sr(desc + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_sub_u32 s{t + 1}, s{desc + 2}, s{step}", SALU, rd=sr(desc + 2) + sr(step), wr=sr(t + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_cselect_b32 s{desc + 2}, 0, s{t + 1}", SALU, rd=sr(t + 1) + [("scc", 0)], wr=sr(desc + 2), key=key + 1)]
        ops += [I(f"s_add_u32 s{S_LOCD}, s{S_LOCD}, 1", SALU, rd=sr(S_LOCD), wr=sr(S_LOCD) + [("scc", 0)], key=key + 1)]
        ops += self.slot_advance(S_SDMA, key + 1)
        if with_l:
            ops += [I(f"s_add_u32 s{S_LD}, s{S_LD}, {LSLOT}", SALU, rd=sr(S_LD), wr=sr(S_LD) + [("scc", 0)], key=key + 1),
                    I(f"s_addc_u32 s{S_LD + 1}, s{S_LD + 1}, 0", SALU, rd=sr(S_LD + 1) + [("scc", 0)], wr=sr(S_LD + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_sub_u32 s{t + 1}, s{S_LD + 2}, {LSLOT}", SALU, rd=sr(S_LD + 2), wr=sr(t + 1) + [("scc", 0)], key=key + 1),
                    I(f"s_cselect_b32 s{S_LD + 2}, 0, s{t + 1}", SALU, rd=sr(t + 1) + [("scc", 0)], wr=sr(S_LD + 2), key=key + 1),
                    I(f"s_add_u32 s{S_LOCL}, s{S_LOCL}, 1", SALU, rd=sr(S_LOCL), wr=sr(S_LOCL) + [("scc", 0)], key=key + 1)]
            ops += self.lslot_advance(S_LDMA, key + 1)
        return ops

    def slot_advance(self, reg, key=0):
        t = S_TMP + 2
        I = Inst
        if RING & (RING - 1) == 0:     # (the ring starts at LDS 0)
            return [I(f"s_add_u32 s{reg}, s{reg}, {SLOT}", SALU, rd=sr(reg), wr=sr(reg) + [("scc", 0)], key=key),
                    I(f"s_and_b32 s{reg}, s{reg}, {RING - 1}", SALU, rd=sr(reg), wr=sr(reg) + [("scc", 0)], key=key)]
        return [I(f"s_add_u32 s{reg}, s{reg}, {SLOT}", SALU, rd=sr(reg), wr=sr(reg) + [("scc", 0)], key=key),
                I(f"s_sub_u32 s{t}, s{reg}, {RING}", SALU, rd=sr(reg), wr=sr(t) + [("scc", 0)], key=key),
                I(f"s_cmp_ge_u32 s{reg}, {RING}", SALU, rd=sr(reg), wr=[("scc", 0)], key=key),
                I(f"s_cselect_b32 s{reg}, s{t}, s{reg}", SALU, rd=sr(t) + sr(reg) + [("scc", 0)], wr=sr(reg), key=key)]

    def lslot_advance(self, reg, key=0):
        I = Inst
        return [I(f"s_add_u32 s{reg}, s{reg}, {LSLOT}", SALU, rd=sr(reg), wr=sr(reg) + [("scc", 0)], key=key),
                I(f"s_and_b32 s{reg}, s{reg}, {NLS * LSLOT - 1}", SALU, rd=sr(reg), wr=sr(reg) + [("scc", 0)], key=key),
                I(f"s_or_b32 s{reg}, s{reg}, {LBASE}", SALU, rd=sr(reg), wr=sr(reg) + [("scc", 0)], key=key)]

    # ------------------------------------------------------------------ one phase
    def phase(self, par, sdp, dvdk, valu, masked, q0_add, dma, next_kind, first_pref, tail_of_step):
        """phase p: MFMAs S / dP(p+1) (sdp) and dV / dK(p-1) (dvdk); VALU(p) (valu); DMA of one Q / dO
        subtile and one LSE / D subtile (dma); the bases and the first three A fragments of the next
        phase, whose MFMA layout is next_kind ('full', 'sdp', 'dvdk' or None).  first_pref: this
        phase's first three fragments were prefetched by its predecessor."""
        mf = self.phase_mfmas(par, sdp, dvdk)
        mfmas = [x[0] for x in mf]
        n = len(mfmas)
        fill = []
        # A-operand reads of this phase (the first three prefetched)
        for m, (_, t, i) in enumerate(mf):
            if m < 3 and first_pref:
                continue
            fill += self.frag_reads(m, t, i, key=-100 + m, earliest=max(m - OPT_WIN, -1) if m >= OPT_WIN else None,
                                    deadline=max(m - OPT_LEAD, 0))
        if OPT_ABL == "nofrag":
            fill = []
        if valu:
            fill += [] if OPT_ABL == "novalu" else self.valu_ops(par, masked, q0_add)
            fill += self.init_reads(par)
        if dma:
            d = self.dma_subtile(True, key=-40, eg=2)
            fill += [x for x in d if x.kind != DMA] if OPT_ABL == "nodma" else d
        # slots and bases of the next phase: rows of p+2, transposed of p, chain starts of p+3
        nxt = []
        nxt += self.slot_advance(S_SROW, key=400) + self.slot_advance(S_STR, key=400) + self.lslot_advance(S_LRD, key=400)
        nxt += [Inst(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0), key=401),
                Inst(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1), key=401),
                Inst(f"v_add_u32_e32 v{V_VB0}, s{S_STR}, v{V_TB0}", VALU, rd=sr(S_STR) + vr(V_TB0), wr=vr(V_VB0), key=401),
                Inst(f"v_add_u32_e32 v{V_VB1}, s{S_STR}, v{V_TB1}", VALU, rd=sr(S_STR) + vr(V_TB1), wr=vr(V_VB1), key=401),
                Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR), key=401)]
        # the bases may change only after this phase's last reads through them (auto deps in fill)
        fill += nxt
        if next_kind is not None:
            nm = self.phase_mfmas(0, next_kind in ("full", "sdp"), next_kind in ("full", "dvdk"))
            for m in range(3):
                _, t, i = nm[m]
                # ring slot m is free once this phase's last MFMA reading it has issued
                last_user = max([k for k in range(n) if k % 16 == m % 16], default=None)
                eg = last_user if last_user is not None else None
                fill += self.frag_reads(m, t, i, key=600 + m, earliest=eg)
        if tail_of_step:
            fill += tail_of_step
        return schedule(mfmas, fill)

    # ------------------------------------------------------------------ step blocks
    def step_tail_ops(self):
        """scalar bookkeeping at the end of a step: VALU subtile counters"""
        I = Inst
        t = S_TMP + 3
        return [I(f"s_add_u32 s{S_N}, s{S_N}, 1", SALU, rd=sr(S_N), wr=sr(S_N) + [("scc", 0)], key=900),
                I(f"s_add_u32 s{S_LOCV}, s{S_LOCV}, 2", SALU, rd=sr(S_LOCV), wr=sr(S_LOCV) + [("scc", 0)], key=900),
                I(f"s_add_u32 s{t}, s{S_Q0V}, {2 * SUB}", SALU, rd=sr(S_Q0V), wr=sr(t) + [("scc", 0)], key=900),
                I(f"s_cmp_ge_u32 s{S_LOCV}, s{S_NSP}", SALU, rd=sr(S_LOCV) + sr(S_NSP), wr=[("scc", 0)], key=900),
                I(f"s_cselect_b32 s{S_LOCV}, 0, s{S_LOCV}", SALU, rd=sr(S_LOCV) + [("scc", 0)], wr=sr(S_LOCV), key=900),
                I(f"s_cselect_b32 s{S_Q0V}, s{S_QF}, s{t}", SALU, rd=sr(S_QF) + sr(t) + [("scc", 0)], wr=sr(S_Q0V), key=900)]

    def step(self, first, last, masked):
        """phases A (p = 2n) and B (2n+1) of step n"""
        a = self.phase(0, sdp=True, dvdk=not first, valu=True, masked=masked, q0_add=0, dma=True,
                       next_kind="dvdk" if last else "full", first_pref=True, tail_of_step=None)
        # (OPT_CONT) the last step loads the next item's K / V fragments: phase A issued the item's
        # last S / dP MFMAs, the last readers of a[KF..], a[VF..]
        tail = self.step_tail_ops() + (self.kv_next_ops(earliest=4) if OPT_CONT and last and OPT_KVAT == "last" else [])
        b = self.phase(1, sdp=not last, dvdk=True, valu=True, masked=masked, q0_add=SUB, dma=True,
                       next_kind="dvdk" if last else "full", first_pref=True, tail_of_step=tail)
        return a + b

    def wrap_check(self, name):
        """(inline check, out-of-line block): the DMA cursor `name` ('d': Q / dO, 'l': LSE / D) reached
        the end of a head's sweep -> the next head of the group (or, none left, zero records)"""
        I = Inst
        t = S_TMP + 6
        loc, hl, curs = {"d": (S_LOCD, S_HLD, ((S_QD, S_QH, S_QHS, S_QREC0), (S_OD, S_OH, S_OHS, S_OREC0))),
                         "l": (S_LOCL, S_HLL, ((S_LD, S_LH, S_LHS, S_LREC0),))}[name]
        lab = self.lab("wrap" + name)
        nsp = S_NSPD if name == "d" else S_NSPL
        check = [I(f"s_cmp_ge_u32 s{loc}, s{nsp}", SALU, rd=sr(loc) + sr(nsp), wr=[("scc", 0)]),
                 I(f"s_cbranch_scc1 {lab}\n{lab}_back:", BRANCH, rd=[("scc", 0)])]
        if OPT_CONT:
            self.ool.extend(self.wrap_cont(name, lab))
            return check
        blk = [label(lab), I(f"s_mov_b32 s{loc}, 0", SALU),
               I(f"s_cmp_eq_u32 s{hl}, 0", SALU),
               I(f"s_cselect_b32 s{t}, 0, 1", SALU),
               I(f"s_sub_u32 s{hl}, s{hl}, s{t}", SALU)]
        for desc, hb, hs, rec0 in curs:
            blk += [I(f"s_add_u32 s{hb}, s{hb}, s{hs}", SALU), I(f"s_addc_u32 s{hb + 1}, s{hb + 1}, 0", SALU),
                    I(f"s_mov_b32 s{desc}, s{hb}", SALU), I(f"s_and_b32 s{desc + 1}, s{hb + 1}, 0xffff", SALU),
                    I(f"s_cmp_eq_u32 s{t}, 0", SALU),
                    I(f"s_cselect_b32 s{rec0}, 0, s{rec0}", SALU),
                    I(f"s_mov_b32 s{desc + 2}, s{rec0}", SALU)]
        blk.append(I(f"s_branch {lab}_back", BRANCH))
        self.ool.extend(blk)
        return check

    def wrap_cont(self, name, lab):
        """(OPT_CONT) out-of-line block of a head wrap: the next head of the group; none left -> the next
        item (record N), once per item switch of the compute; a second time -> stall (zero records,
        the slot noted: item_switch re-issues from there)"""
        I = Inst
        loc, hl, sw, stall, slot, curs = {
            "d": (S_LOCD, S_HLD, S_DSW, S_DSTALL, S_SDMA, ((S_QD, S_QH, S_QHS, S_QREC0, N_QH, N_QREC),
                                                           (S_OD, S_OH, S_OHS, S_OREC0, N_OH, N_OREC))),
            "l": (S_LOCL, S_HLL, S_LSW, S_LSTALL, S_LDMA, ((S_LD, S_LH, S_LHS, S_LREC0, N_LH, N_LREC),))}[name]
        l_item, l_stall = lab + "_item", lab + "_stall"
        blk = [label(lab), I(f"s_mov_b32 s{loc}, 0", SALU),
               I(f"s_cmp_eq_u32 s{hl}, 0", SALU), I(f"s_cbranch_scc1 {l_item}", BRANCH),
               I(f"s_sub_u32 s{hl}, s{hl}, 1", SALU)]
        for desc, hb, hs, rec0, _, _ in curs:
            blk += [I(f"s_add_u32 s{hb}, s{hb}, s{hs}", SALU), I(f"s_addc_u32 s{hb + 1}, s{hb + 1}, 0", SALU),
                    I(f"s_mov_b32 s{desc}, s{hb}", SALU), I(f"s_and_b32 s{desc + 1}, s{hb + 1}, 0xffff", SALU),
                    I(f"s_mov_b32 s{desc + 2}, s{rec0}", SALU)]
        blk += [I(f"s_branch {lab}_back", BRANCH),
                label(l_item), I(f"s_cmp_eq_u32 s{sw}, 0", SALU), I(f"s_cbranch_scc0 {l_stall}", BRANCH)]
        blk += self.switch_ops(name)
        blk += [I(f"s_branch {lab}_back", BRANCH),
                label(l_stall), I(f"s_cmp_eq_u32 s{stall}, -1", SALU), I(f"s_cselect_b32 s{stall}, s{slot}, s{stall}", SALU)]
        blk += [I(f"s_mov_b32 s{desc + 2}, 0", SALU) for desc, *_ in curs]
        blk += [I(f"s_branch {lab}_back", BRANCH)]
        return blk

    def switch_ops(self, name, rec=V_N):
        """(OPT_CONT) a DMA cursor ('d' or 'l') moves to the first head of the item in the record at
        v[rec]; the cursor's position resets, its side is marked switched"""
        I = Inst
        loc, hl, sw, nsp, curs = {
            "d": (S_LOCD, S_HLD, S_DSW, S_NSPD, ((S_QD, S_QH, S_QREC0, N_QH, N_QREC), (S_OD, S_OH, S_OREC0, N_OH, N_OREC))),
            "l": (S_LOCL, S_HLL, S_LSW, S_NSPL, ((S_LD, S_LH, S_LREC0, N_LH, N_LREC),))}[name]

        def rf(s_, f):
            return I(f"v_readfirstlane_b32 s{s_}, v{rec + f}", RFL, rd=vr(rec + f), wr=sr(s_))
        ops = [I(f"s_mov_b32 s{loc}, 0", SALU, wr=sr(loc)), I(f"s_mov_b32 s{sw}, 1", SALU, wr=sr(sw)),
               rf(hl, N_HL0), rf(nsp, N_NSP)]
        for desc, hb, rec0, fb, fr in curs:
            ops += [rf(hb, fb), rf(hb + 1, fb + 1), rf(rec0, fr),
                    I(f"s_mov_b32 s{desc}, s{hb}", SALU, rd=sr(hb), wr=sr(desc)),
                    I(f"s_and_b32 s{desc + 1}, s{hb + 1}, 0xffff", SALU, rd=sr(hb + 1), wr=sr(desc + 1)),
                    I(f"s_mov_b32 s{desc + 2}, s{rec0}", SALU, rd=sr(rec0), wr=sr(desc + 2)),
                    I(f"s_mov_b32 s{desc + 3}, 0x20000", SALU, wr=sr(desc + 3))]
        return ops

    def kv_next_ops(self, rec=V_N, key=700, earliest=None):
        """(OPT_CONT) the K / V fragments of the item in the record at v[rec] into a[KF..], a[VF..]
        (records 0: no item, zeros)"""
        I = Inst
        ops = []
        for d0, f in ((S_KVN, N_KD), (S_KVN + 4, N_VD)):
            ops += [I(f"v_readfirstlane_b32 s{d0 + i}, v{rec + f + i}", RFL, rd=vr(rec + f + i), wr=sr(d0 + i), key=key,
                      earliest=earliest) for i in range(3)]
            ops += [I(f"s_mov_b32 s{d0 + 3}, 0x20000", SALU, wr=sr(d0 + 3), key=key, earliest=earliest)]
        for base, d0, lo in ((KF, S_KVN, V_KLO), (VF, S_KVN + 4, V_VLO)):
            for ks in range(KS):
                ops.append(I(f"buffer_load_dwordx4 {rtxt('a', base + 4 * ks, 4)}, v{lo}, s[{d0}:{d0 + 3}], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(lo) + sr(d0, 4), wr=ar(base + 4 * ks, 4), key=key + 1, earliest=earliest))
        return ops

    def stamp(self, acc, count=None):
        """(FA_GBW_STAMP=2) v[acc] += now - last; last = now (acc None: only last = now); v[count] += 1"""
        if not OPT_STEPSTAMP:
            return []
        t = S_TMP + 1
        ins = [Inst(f"s_memtime s[{t}:{t + 1}]", SMEM), Inst("s_waitcnt lgkmcnt(0)", WAIT),
               Inst(f"v_mov_b32_e32 v{V_SS + 8}, s{t}", VALU)]
        if acc is not None:
            ins += [Inst(f"v_sub_u32_e32 v{V_SS + 9}, v{V_SS + 8}, v{V_SS + 4}", VALU),
                    Inst(f"v_add_u32_e32 v{acc}, v{acc}, v{V_SS + 9}", VALU)]
        ins += [Inst(f"v_mov_b32_e32 v{V_SS + 4}, v{V_SS + 8}", VALU)]
        if count is not None:
            ins += [Inst(f"v_add_u32_e32 v{count}, 1, v{count}", VALU)]
        return ins

    def step_end(self, last=False):
        """after a step: head wraps of the DMA cursors, wait for the subtiles the next step reads, barrier
        (the last step: the tail reads subtiles the step before waited for; OPT_CONT leaves the next
        item's K / V loads in flight)"""
        ins = self.wrap_check("d") + self.wrap_check("l")
        # (the last step's compute is also kept apart: v[V_SS + 12] under OPT_CONT)
        ins += self.stamp(V_SS + 12 if OPT_CONT and last else V_SS + 0, count=V_SS + 3)
        if OPT_STEPSTAMP and OPT_CONT and not last:
            # the two steps before the last (their DMA runs into the next item) also into v[V_SS + 13]
            t = S_TMP + 1
            ins += [Inst(f"s_sub_u32 s{t}, s{S_NLAST}, s{S_N}", SALU), Inst(f"s_cmp_le_u32 s{t}, 1", SALU),
                    Inst("s_cselect_b64 vcc, -1, 0", SALU),
                    Inst(f"v_cndmask_b32_e32 v{V_SS + 9}, 0, v{V_SS + 9}, vcc", VALU),
                    Inst(f"v_add_u32_e32 v{V_SS + 13}, v{V_SS + 13}, v{V_SS + 9}", VALU)]
        ins += [Inst(f"s_waitcnt vmcnt({VMCNT_STEP + (2 * KS if OPT_CONT and last else 0)}) lgkmcnt(0)", WAIT)]
        ins += self.stamp(V_SS + 1)
        ins += [Inst("s_barrier", BARRIER)]
        ins += self.stamp(V_SS + 2)
        return ins

    def tail(self):
        """dV^T, dK^T of the last subtile (parity 1), then the epilogue"""
        mf = self.phase_mfmas(0, False, True)   # par 0 -> packs 1
        fill = []
        for m, (_, t, i) in enumerate(mf):
            if m < 3:
                continue
            fill += self.frag_reads(m, t, i, key=-100 + m, earliest=max(m - 16, -1) if m >= 16 else None,
                                    deadline=max(m - 2, 0))
        if OPT_CONT and OPT_KVAT == "tail":
            fill += self.kv_next_ops(earliest=0)
        return schedule([x[0] for x in mf], fill)

    # ------------------------------------------------------------------ prologue
    def prologue(self, l_epi, l_nokeys=None, cont=False):
        """the item S_ITEM's geometry, DMA cursors and loop state (as the item loop head); cont
        (OPT_CONT, geometry()): only the geometry, packed into the record N -- no loads, no loop state,
        no zeroing; l_nokeys: no keys in the block (default: the next item), l_epi: keys and no rows"""
        I = Inst
        ins = []
        l_nokeys = l_nokeys or self.lab_next
        substamp = self.stamp if not OPT_CONT else (lambda *a, **k: [])
        # kernarg dwords 0..45 -> s56..s101; 46..49 (h, ng, nh, group) -> s20..s23 (free until the loop
        # state is set); 50, 51 (c, scale) -> S_C, S_SCALE; 52 (flags) -> s3
        ka = 56
        ins += [I(f"s_load_dwordx16 s[{ka}:{ka + 15}], s[0:1], 0x0", SMEM, rd=sr(0, 2), wr=sr(ka, 16)),
                I(f"s_load_dwordx16 s[{ka + 16}:{ka + 31}], s[0:1], 0x40", SMEM, rd=sr(0, 2), wr=sr(ka + 16, 16)),
                I(f"s_load_dwordx8 s[{ka + 32}:{ka + 39}], s[0:1], 0x80", SMEM, rd=sr(0, 2), wr=sr(ka + 32, 8)),
                I(f"s_load_dwordx4 s[{ka + 40}:{ka + 43}], s[0:1], 0xa0", SMEM, rd=sr(0, 2), wr=sr(ka + 40, 4)),
                I(f"s_load_dwordx2 s[{ka + 44}:{ka + 45}], s[0:1], 0xb0", SMEM, rd=sr(0, 2), wr=sr(ka + 44, 2)),
                I("s_load_dwordx4 s[20:23], s[0:1], 0xb8", SMEM, rd=sr(0, 2), wr=sr(20, 4)),
                I(f"s_load_dwordx2 s[{S_C}:{S_SCALE}], s[0:1], 0xc8", SMEM, rd=sr(0, 2), wr=sr(S_C, 2)),
                I("s_load_dword s3, s[0:1], 0xd0", SMEM, rd=sr(0, 2), wr=sr(3)),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        # the work order (fa_params.h ItemDecode) into s[36:45] (free until the geometry): (bidb, hx,
        # kvh, key block) of this item; FA_GBW_DECBURST=1 (dev switch, off in the shipped build): in the
        # kernargs' scalar round trip, one less per item
        dec = [I(f"s_load_dwordx8 s[36:43], s[0:1], {DEC_OFF}", SMEM),
               I(f"s_load_dwordx2 s[44:45], s[0:1], {DEC_OFF + 32}", SMEM)]
        if OPT_DECBURST:
            ins[-1:-1] = dec
        if OPT_STAMP:
            ins += [I(f"s_memtime s[{S_TMP + 1}:{S_TMP + 2}]", SMEM, wr=sr(S_TMP + 1, 2)),
                    I(f"s_getreg_b32 s{S_TMP + 3}, hwreg(HW_REG_HW_ID)", SALU, wr=sr(S_TMP + 3)),
                    I(f"s_getreg_b32 s{S_TMP + 4}, hwreg(HW_REG_XCC_ID)", SALU, wr=sr(S_TMP + 4)),
                    I("s_waitcnt lgkmcnt(0)", WAIT)]
            ins += [I(f"v_mov_b32_e32 v{V_STAMP + i}, s{S_TMP + 1 + i}", VALU, rd=sr(S_TMP + 1 + i), wr=vr(V_STAMP + i)) for i in range(4)]
            ins += [I(f"v_mov_b32_e32 v{V_STAMP + 4}, s{S_ITEM}", VALU, rd=sr(S_ITEM), wr=vr(V_STAMP + 4))]
        P = lambda i: ka + i   # noqa: E731
        Pq, Pk, Pv, Pdo, Pdk, Pdv, Pl, Psch, Pcq, Pck = (P(2 * i) for i in range(10))
        Bq, Bk, Bv, Bdo, Bdk, Bdv = (P(20 + 2 * i) for i in range(6))
        Rq, Rk, Rv, Rdo, Rdk, Rdv = (P(32 + i) for i in range(6))
        Hq, Hk, Hv, Hdo, Hdk, Hdv = (P(38 + i) for i in range(6))
        SQ, SK = P(44), P(45)
        H, NG, NHS, GRP = 20, 21, 22, 23
        FLG = 3
        T0, T1, T2, T3, T4, T5, T6 = (S_TMP + i for i in range(7))
        if not OPT_DECBURST:
            ins += dec + [I("s_waitcnt lgkmcnt(0)", WAIT)]
        ins += substamp(V_SS + 11)
        BIDB, HX, KVH, KB = 24, 25, 26, 27      # S_N .. S_Q0V, set at the end
        # varlen with a device-built work list (flags bit 2, fa_fwd_asm.cpp varlen_items_kernel: the
        # key blocks of every sequence, heaviest level first, none past a sequence's end): its entry
        # (bidb | head << 16, kvh | key block << 16); else decoded from the item index
        l_tab, l_dec = self.lab("tab"), self.lab("dec")
        ins += [I(f"s_bitcmp1_b32 s{FLG}, 2", SALU), I(f"s_cbranch_scc1 {l_tab}", BRANCH)]
        ins += item_decode_ops(L=S_ITEM, M=36, pa=T1, pb=T3, t=T5, u=T6, o_blk=KB, reverse=False)
        ins += [I(f"s_mov_b32 s{BIDB}, s{T3}", SALU), I(f"s_mov_b32 s{HX}, s{T6}", SALU),
                I(f"s_mov_b32 s{KVH}, s{T1}", SALU), I(f"s_branch {l_dec}", BRANCH), label(l_tab),
                I(f"s_lshl_b32 s{T0}, s{S_ITEM}, 3", SALU), I(f"s_add_u32 s{T0}, s{T0}, 8", SALU),
                I(f"s_load_dwordx2 s[{T1}:{T1 + 1}], s[{Psch}:{Psch + 1}], s{T0}", SMEM),
                I("s_waitcnt lgkmcnt(0)", WAIT),
                I(f"s_and_b32 s{BIDB}, s{T1}, 0xffff", SALU), I(f"s_lshr_b32 s{HX}, s{T1}, 16", SALU),
                I(f"s_and_b32 s{KVH}, s{T1 + 1}, 0xffff", SALU), I(f"s_lshr_b32 s{KB}, s{T1 + 1}, 16", SALU),
                label(l_dec)]
        # varlen geometry (BlockInfo, block_info.h:14-31): 64-bit byte offsets of row 0 of this sequence;
        # seqlens into SQ / SK
        QOFF, DOOFF, KOFF, VOFF, DKOFF, DVOFF = (34, 35), (36, 37), (38, 39), (40, 41), (42, 43), (44, 45)

        def mul64(dst, a32, b32):
            return [I(f"s_mul_i32 s{dst[0]}, s{a32}, s{b32}", SALU, rd=sr(a32) + sr(b32), wr=sr(dst[0])),
                    I(f"s_mul_hi_u32 s{dst[1]}, s{a32}, s{b32}", SALU, rd=sr(a32) + sr(b32), wr=sr(dst[1]))]

        def mul64_i64(dst, a32, b64):
            return [I(f"s_mul_i32 s{dst[0]}, s{a32}, s{b64}", SALU, rd=sr(a32) + sr(b64), wr=sr(dst[0])),
                    I(f"s_mul_hi_u32 s{dst[1]}, s{a32}, s{b64}", SALU, rd=sr(a32) + sr(b64), wr=sr(dst[1])),
                    I(f"s_mul_i32 s{T0}, s{a32}, s{b64 + 1}", SALU, rd=sr(a32) + sr(b64 + 1), wr=sr(T0)),
                    I(f"s_add_u32 s{dst[1]}, s{dst[1]}, s{T0}", SALU, rd=sr(dst[1]) + sr(T0), wr=sr(dst[1]))]

        # varlen: the cu_seqlens loads of every part are issued together and waited for once (one
        # scalar-memory round trip per item start instead of one per part)
        parts = ((Pcq, Bq, Rq, QOFF, SQ), (Pcq, Bdo, Rdo, DOOFF, None),
                 (Pck, Bk, Rk, KOFF, SK), (Pck, Bv, Rv, VOFF, None),
                 (Pck, Bdk, Rdk, DKOFF, None), (Pck, Bdv, Rdv, DVOFF, None))
        ins += [I(f"s_lshl_b32 s{T1}, s{BIDB}, 2", SALU, rd=sr(BIDB), wr=sr(T1))]
        for cu, bstride, rstride, off, seq in parts:
            lf = self.lab("nold")
            ins += [I(f"s_cmp_eq_u64 s[{cu}:{cu + 1}], 0", SALU, rd=sr(cu, 2), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH),
                    I(f"s_load_dwordx2 s[{off[0]}:{off[1]}], s[{cu}:{cu + 1}], s{T1}", SMEM, rd=sr(cu, 2) + sr(T1), wr=sr(off[0], 2)),
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
                    I(f"s_mov_b32 s{T1}, s{off[0]}", SALU, rd=sr(off[0]), wr=sr(T1))]
            ins += mul64(off, T1, rstride)
            ins += [I(f"s_branch {ld}", BRANCH), label(lf)]
            ins += mul64_i64(off, BIDB, bstride)
            ins += [label(ld)]
        # key block: n0 = 128 kb (exit when n0 >= sk); this wave's keys from kw0 = n0 + 32 wave
        N0, KW0 = T4, T5
        ins += [I(f"s_lshl_b32 s{N0}, s{KB}, 7", SALU, rd=sr(KB), wr=sr(N0)),
                I(f"s_cmp_ge_i32 s{N0}, s{SK}", SALU, rd=sr(N0) + sr(SK), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_nokeys}", BRANCH),
                I(f"s_lshl_b32 s{KW0}, s{S_WAVE}, 5", SALU, rd=sr(S_WAVE), wr=sr(KW0)),
                I(f"s_add_u32 s{KW0}, s{KW0}, s{N0}", SALU, rd=sr(KW0) + sr(N0), wr=sr(KW0))]
        # dK / dV head: the kv head (reduced GQA, flags bit 1) or the query head
        HD = T3
        ins += [I(f"s_bitcmp1_b32 s{FLG}, 1", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                I(f"s_cselect_b32 s{HD}, s{KVH}, s{HX}", SALU, rd=sr(KVH) + sr(HX) + [("scc", 0)], wr=sr(HD))]
        # the epilogue's scalars, stashed in VGPRs (readfirstlane there)
        stash = [KW0, HD, DKOFF[0], DKOFF[1], DVOFF[0], DVOFF[1], Pdk, Pdk + 1, Pdv, Pdv + 1, Rdk, Rdv, Hdk, Hdv, SK]
        st0 = V_N + N_ST if cont else V_ST
        for i, x in enumerate(stash):
            ins.append(I(f"v_mov_b32_e32 v{st0 + i}, s{x}", VALU, rd=sr(x), wr=vr(st0 + i)))

        def desc_at(dst4, ptr, off64, head, hstride, row, rstride, nrec_rows):
            """descriptor for ptr + off64 + head * hstride + row * rstride, records nrec_rows * rstride"""
            o = [I(f"s_mul_i32 s{T0}, s{head}, s{hstride}", SALU, rd=sr(head) + sr(hstride), wr=sr(T0)),
                 I(f"s_mul_hi_u32 s{T1}, s{head}, s{hstride}", SALU, rd=sr(head) + sr(hstride), wr=sr(T1)),
                 I(f"s_add_u32 s{dst4}, s{ptr}, s{T0}", SALU, rd=sr(ptr) + sr(T0), wr=sr(dst4) + [("scc", 0)]),
                 I(f"s_addc_u32 s{dst4 + 1}, s{ptr + 1}, s{T1}", SALU, rd=sr(ptr + 1) + sr(T1) + [("scc", 0)], wr=sr(dst4 + 1)),
                 I(f"s_add_u32 s{dst4}, s{dst4}, s{off64[0]}", SALU, rd=sr(dst4) + sr(off64[0]), wr=sr(dst4) + [("scc", 0)]),
                 I(f"s_addc_u32 s{dst4 + 1}, s{dst4 + 1}, s{off64[1]}", SALU, rd=sr(dst4 + 1) + sr(off64[1]) + [("scc", 0)], wr=sr(dst4 + 1)),
                 I(f"s_mul_i32 s{T0}, s{row}, s{rstride}", SALU, rd=sr(row) + sr(rstride), wr=sr(T0)),
                 I(f"s_mul_hi_u32 s{T1}, s{row}, s{rstride}", SALU, rd=sr(row) + sr(rstride), wr=sr(T1)),
                 I(f"s_add_u32 s{dst4}, s{dst4}, s{T0}", SALU, rd=sr(dst4) + sr(T0), wr=sr(dst4) + [("scc", 0)]),
                 I(f"s_addc_u32 s{dst4 + 1}, s{dst4 + 1}, s{T1}", SALU, rd=sr(dst4 + 1) + sr(T1) + [("scc", 0)], wr=sr(dst4 + 1)),
                 I(f"s_max_i32 s{T0}, s{nrec_rows}, 0", SALU, rd=sr(nrec_rows), wr=sr(T0)),
                 I(f"s_mul_i32 s{dst4 + 2}, s{T0}, s{rstride}", SALU, rd=sr(T0) + sr(rstride), wr=sr(dst4 + 2)),
                 I(f"s_and_b32 s{dst4 + 1}, s{dst4 + 1}, 0xffff", SALU, rd=sr(dst4 + 1), wr=sr(dst4 + 1)),
                 I(f"s_mov_b32 s{dst4 + 3}, 0x20000", SALU, wr=sr(dst4 + 3))]
            return o

        # ---- K / V fragments of this wave's 32 keys (B operands), loaded once into AGPRs ----
        REM = T6
        ins += [I(f"s_sub_i32 s{REM}, s{SK}, s{KW0}", SALU, rd=sr(SK) + sr(KW0), wr=sr(REM))]
        # descriptors in the varlen kernargs' registers (dead now, never rewritten): the fragment loads
        # stay in flight while the Q / dO / LSE DMA of the prologue is issued
        KD, VD = 72, 76
        ins += desc_at(KD, Pk, KOFF, KVH, Hk, KW0, Rk, REM)
        ins += desc_at(VD, Pv, VOFF, KVH, Hv, KW0, Rv, REM)
        ins += substamp(V_SS + 12)
        r_, hh = V_TMP, V_TMP + 1
        ins += [I(f"v_and_b32_e32 v{r_}, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(r_)),
                I(f"v_lshrrev_b32_e32 v{hh}, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(hh)),
                I(f"v_mul_lo_u32 v{V_TMP + 2}, v{r_}, s{Rk}", VALU, rd=vr(r_) + sr(Rk), wr=vr(V_TMP + 2)),
                I(f"v_lshl_add_u32 v{V_TMP + 2}, v{hh}, 4, v{V_TMP + 2}", VALU, rd=vr(hh) + vr(V_TMP + 2), wr=vr(V_TMP + 2)),
                I(f"v_mul_lo_u32 v{V_TMP + 3}, v{r_}, s{Rv}", VALU, rd=vr(r_) + sr(Rv), wr=vr(V_TMP + 3)),
                I(f"v_lshl_add_u32 v{V_TMP + 3}, v{hh}, 4, v{V_TMP + 3}", VALU, rd=vr(hh) + vr(V_TMP + 3), wr=vr(V_TMP + 3))]
        if cont:
            ins += [I(f"v_mov_b32_e32 v{V_KLO}, v{V_TMP + 2}", VALU, rd=vr(V_TMP + 2), wr=vr(V_KLO)),
                    I(f"v_mov_b32_e32 v{V_VLO}, v{V_TMP + 3}", VALU, rd=vr(V_TMP + 3), wr=vr(V_VLO))]
        else:
            for ks in range(KS):
                ins.append(I(f"buffer_load_dwordx4 {rtxt('a', KF + 4 * ks, 4)}, v{V_TMP + 2}, s[{KD}:{KD + 3}], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(V_TMP + 2) + sr(KD, 4), wr=ar(KF + 4 * ks, 4)))
            for ks in range(KS):
                ins.append(I(f"buffer_load_dwordx4 {rtxt('a', VF + 4 * ks, 4)}, v{V_TMP + 3}, s[{VD}:{VD + 3}], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(V_TMP + 3) + sr(VD, 4), wr=ar(VF + 4 * ks, 4)))
        # ---- per-lane values (while the fragments load) ----
        # DMA voffsets: wave w, half f: row = 16 f + lane / 4, col = 64 w + 16 ((lane & 3) ^ ((lane >> 4) & 3))
        x = V_TMP + 2
        ins += [I(f"v_lshrrev_b32_e32 v{x + 2}, 2, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 2)),
                I(f"v_bfe_u32 v{x + 3}, v{V_LANE}, 4, 2", VALU, rd=vr(V_LANE), wr=vr(x + 3)),
                I(f"v_and_b32_e32 v{x + 4}, 3, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 4)),
                I(f"v_xor_b32_e32 v{x + 3}, v{x + 3}, v{x + 4}", VALU, rd=vr(x + 3, 2), wr=vr(x + 3)),
                I(f"v_lshlrev_b32_e32 v{x + 3}, 4, v{x + 3}", VALU, rd=vr(x + 3), wr=vr(x + 3)),
                I(f"s_lshl_b32 s{T0}, s{S_WAVE}, 6", SALU, rd=sr(S_WAVE), wr=sr(T0)),
                I(f"v_add_u32_e32 v{x + 3}, s{T0}, v{x + 3}", VALU, rd=sr(T0) + vr(x + 3), wr=vr(x + 3))]
        if OPT_ABL == "dmarows":   # timing ablation (wrong data): each DMA covers 4 whole rows
            ins += [I(f"v_lshrrev_b32_e32 v{x + 2}, 4, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 2)),
                    I(f"s_lshl_b32 s{T0}, s{S_WAVE}, 2", SALU, rd=sr(S_WAVE), wr=sr(T0)),
                    I(f"v_add_u32_e32 v{x + 2}, s{T0}, v{x + 2}", VALU, rd=sr(T0) + vr(x + 2), wr=vr(x + 2)),
                    I(f"v_and_b32_e32 v{x + 3}, 15, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 3)),
                    I(f"v_lshlrev_b32_e32 v{x + 3}, 4, v{x + 3}", VALU, rd=vr(x + 3), wr=vr(x + 3))]
        for vq, rs in ((V_QV0, Rq), (V_OV0, Rdo)):
            ins += [I(f"v_mul_lo_u32 v{vq}, v{x + 2}, s{rs}", VALU, rd=vr(x + 2) + sr(rs), wr=vr(vq)),
                    I(f"v_add_u32_e32 v{vq}, v{vq}, v{x + 3}", VALU, rd=vr(vq) + vr(x + 3), wr=vr(vq)),
                    I(f"s_lshl_b32 s{T0}, s{rs}, 4", SALU, rd=sr(rs), wr=sr(T0)),
                    I(f"v_add_u32_e32 v{vq + 1}, s{T0}, v{vq}", VALU, rd=sr(T0) + vr(vq), wr=vr(vq + 1))]
        ins += [I(f"v_lshlrev_b32_e32 v{V_L4}, 2, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(V_L4))]
        # LDS lane bases (as gen_fwd.py): rb = r 64 + ((c ^ xr) << 4), c = hh / 2 + hh, xr = (r >> 2) & 3
        ins += [I(f"v_bfe_u32 v{x + 2}, v{r_}, 2, 2", VALU, rd=vr(r_), wr=vr(x + 2)),
                I(f"v_xor_b32_e32 v{x + 3}, v{hh}, v{x + 2}", VALU, rd=vr(hh) + vr(x + 2), wr=vr(x + 3)),
                I(f"v_lshlrev_b32_e32 v{x + 4}, 6, v{r_}", VALU, rd=vr(r_), wr=vr(x + 4)),
                I(f"v_lshl_add_u32 v{V_RB0}, v{x + 3}, 4, v{x + 4}", VALU, rd=vr(x + 3) + vr(x + 4), wr=vr(V_RB0)),
                I(f"v_add_u32_e32 v{x + 3}, 2, v{hh}", VALU, rd=vr(hh), wr=vr(x + 3)),
                I(f"v_xor_b32_e32 v{x + 3}, v{x + 3}, v{x + 2}", VALU, rd=vr(x + 3) + vr(x + 2), wr=vr(x + 3)),
                I(f"v_lshl_add_u32 v{V_RB1}, v{x + 3}, 4, v{x + 4}", VALU, rd=vr(x + 3) + vr(x + 4), wr=vr(V_RB1))]
        ins += [I(f"v_and_b32_e32 v{x + 2}, 15, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(x + 2)),             # i
                I(f"v_lshrrev_b32_e32 v{x + 3}, 2, v{x + 2}", VALU, rd=vr(x + 2), wr=vr(x + 3)),            # q
                I(f"v_and_b32_e32 v{x + 4}, 3, v{x + 2}", VALU, rd=vr(x + 2), wr=vr(x + 4)),                # pp
                I(f"v_lshrrev_b32_e32 v{x + 5}, 4, v{r_}", VALU, rd=vr(r_), wr=vr(x + 5)),                  # r >> 4
                I(f"v_lshrrev_b32_e32 v{x + 6}, 1, v{x + 4}", VALU, rd=vr(x + 4), wr=vr(x + 6)),            # pp >> 1
                I(f"v_lshl_add_u32 v{x + 5}, v{x + 5}, 1, v{x + 6}", VALU, rd=vr(x + 5) + vr(x + 6), wr=vr(x + 5)),   # trc
                I(f"v_lshl_add_u32 v{x + 6}, v{hh}, 2, v{x + 3}", VALU, rd=vr(hh) + vr(x + 3), wr=vr(x + 6)),      # 4 hh + q
                I(f"v_lshlrev_b32_e32 v{x + 6}, 6, v{x + 6}", VALU, rd=vr(x + 6), wr=vr(x + 6)),
                I(f"v_and_b32_e32 v{x + 3}, 1, v{x + 4}", VALU, rd=vr(x + 4), wr=vr(x + 3)),
                I(f"v_lshl_add_u32 v{x + 6}, v{x + 3}, 3, v{x + 6}", VALU, rd=vr(x + 3) + vr(x + 6), wr=vr(x + 6)),
                I(f"v_xor_b32_e32 v{x + 3}, v{x + 5}, v{hh}", VALU, rd=vr(x + 5) + vr(hh), wr=vr(x + 3)),
                I(f"v_lshl_add_u32 v{V_TB0}, v{x + 3}, 4, v{x + 6}", VALU, rd=vr(x + 3) + vr(x + 6), wr=vr(V_TB0)),
                I(f"v_add_u32_e32 v{x + 3}, 2, v{hh}", VALU, rd=vr(hh), wr=vr(x + 3)),
                I(f"v_xor_b32_e32 v{x + 3}, v{x + 5}, v{x + 3}", VALU, rd=vr(x + 5) + vr(x + 3), wr=vr(x + 3)),
                I(f"v_lshl_add_u32 v{V_TB1}, v{x + 3}, 4, v{x + 6}", VALU, rd=vr(x + 3) + vr(x + 6), wr=vr(V_TB1))]
        # chain-start lane base: 16 hh; mask lane value: kw0 + r - 4 hh
        ins += [I(f"v_lshlrev_b32_e32 v{V_LB}, 4, v{hh}", VALU, rd=vr(hh), wr=vr(V_LB)),
                I(f"v_add_u32_e32 v{V_LANEK}, s{KW0}, v{r_}", VALU, rd=sr(KW0) + vr(r_), wr=vr(V_LANEK)),
                I(f"v_lshlrev_b32_e32 v{x + 2}, 2, v{hh}", VALU, rd=vr(hh), wr=vr(x + 2)),
                I(f"v_sub_u32_e32 v{V_LANEK}, v{V_LANEK}, v{x + 2}", VALU, rd=vr(V_LANEK) + vr(x + 2), wr=vr(V_LANEK)),
                I(f"v_mov_b32_e32 v{V_NINF}, 0xff800000", VALU, wr=vr(V_NINF))]
        # ---- sweep geometry ----
        QF = S_QF
        ins += [I(f"s_mov_b32 s{QF}, s{N0}", SALU, rd=sr(N0), wr=sr(QF)) if self.causal else I(f"s_mov_b32 s{QF}, 0", SALU, wr=sr(QF))]
        ROWS = T6   # rows from q_first, clamped at 0
        ins += [I(f"s_sub_i32 s{ROWS}, s{SQ}, s{QF}", SALU, rd=sr(SQ) + sr(QF), wr=sr(ROWS)),
                I(f"s_max_i32 s{ROWS}, s{ROWS}, 0", SALU, rd=sr(ROWS), wr=sr(ROWS)),
                I(f"s_add_u32 s{T0}, s{ROWS}, {SUB - 1}", SALU, rd=sr(ROWS), wr=sr(T0)),
                I(f"s_lshr_b32 s{T0}, s{T0}, 5", SALU, rd=sr(T0), wr=sr(T0)),                 # ns
                I(f"s_lshl_b32 s{S_LREC0}, s{T0}, 8", SALU, rd=sr(T0), wr=sr(S_LREC0)),       # LSE / D bytes
                I(f"s_add_u32 s{T0}, s{T0}, 1", SALU, rd=sr(T0), wr=sr(T0)),
                I(f"s_and_b32 s{S_NSP}, s{T0}, -2", SALU, rd=sr(T0), wr=sr(S_NSP))]            # ns rounded up to even
        # heads of the sweep: reduced GQA -> the group of kv head KVH, else head HX alone
        HB = S_STR
        ins += [I(f"s_mul_i32 s{T0}, s{KVH}, s{GRP}", SALU, rd=sr(KVH) + sr(GRP), wr=sr(T0)),
                I(f"s_bitcmp1_b32 s{FLG}, 1", SALU, rd=sr(FLG), wr=[("scc", 0)]),
                I(f"s_cselect_b32 s{HB}, s{T0}, s{HX}", SALU, rd=sr(T0) + sr(HX) + [("scc", 0)], wr=sr(HB)),
                I(f"s_cselect_b32 s{T1}, s{NHS}, 1", SALU, rd=sr(NHS) + [("scc", 0)], wr=sr(T1)),     # nh
                I(f"s_sub_u32 s{S_HLD}, s{T1}, 1", SALU, rd=sr(T1), wr=sr(S_HLD)),
                I(f"s_mov_b32 s{S_HLL}, s{S_HLD}", SALU, rd=sr(S_HLD), wr=sr(S_HLL)),
                I(f"s_mul_i32 s{T1}, s{T1}, s{S_NSP}", SALU, rd=sr(T1) + sr(S_NSP), wr=sr(T1)),   # N
                I(f"s_lshr_b32 s{T1}, s{T1}, 1", SALU, rd=sr(T1), wr=sr(T1)),                       # steps
                I(f"s_sub_i32 s{T2}, s{T1}, 1", SALU, rd=sr(T1), wr=sr(T2))]                        # last step
        # LSE / D cursor: lsed + ((bidb h + HB) ng + q_first / 32) * 256
        ins += [I(f"s_mul_i32 s{T0}, s{BIDB}, s{H}", SALU, rd=sr(BIDB) + sr(H), wr=sr(T0)),
                I(f"s_add_u32 s{T0}, s{T0}, s{HB}", SALU, rd=sr(T0) + sr(HB), wr=sr(T0)),
                I(f"s_mul_i32 s{T0}, s{T0}, s{NG}", SALU, rd=sr(T0) + sr(NG), wr=sr(T0)),
                I(f"s_lshr_b32 s{T1}, s{QF}, 5", SALU, rd=sr(QF), wr=sr(T1)),
                I(f"s_add_u32 s{T0}, s{T0}, s{T1}", SALU, rd=sr(T0) + sr(T1), wr=sr(T0)),
                I(f"s_lshr_b32 s{T1}, s{T0}, 24", SALU, rd=sr(T0), wr=sr(T1)),
                I(f"s_lshl_b32 s{T0}, s{T0}, 8", SALU, rd=sr(T0), wr=sr(T0)),
                I(f"s_add_u32 s{S_LH}, s{Pl}, s{T0}", SALU, rd=sr(Pl) + sr(T0), wr=sr(S_LH) + [("scc", 0)]),
                I(f"s_addc_u32 s{S_LH + 1}, s{Pl + 1}, s{T1}", SALU, rd=sr(Pl + 1) + sr(T1) + [("scc", 0)], wr=sr(S_LH + 1)),
                I(f"s_lshl_b32 s{S_LHS}, s{NG}, 8", SALU, rd=sr(NG), wr=sr(S_LHS)),
                I(f"s_mov_b32 s{S_LD}, s{S_LH}", SALU, rd=sr(S_LH), wr=sr(S_LD)),
                I(f"s_and_b32 s{S_LD + 1}, s{S_LH + 1}, 0xffff", SALU, rd=sr(S_LH + 1), wr=sr(S_LD + 1)),
                I(f"s_mov_b32 s{S_LD + 2}, s{S_LREC0}", SALU, rd=sr(S_LREC0), wr=sr(S_LD + 2)),
                I(f"s_mov_b32 s{S_LD + 3}, 0x20000", SALU, wr=sr(S_LD + 3))]
        # ---- Q / dO cursors at (head HB, row q_first) ----
        ins += desc_at(S_QD, Pq, QOFF, HB, Hq, QF, Rq, ROWS)
        ins += desc_at(S_OD, Pdo, DOOFF, HB, Hdo, QF, Rdo, ROWS)
        ins += [I(f"s_mov_b32 s{S_QREC0}, s{S_QD + 2}", SALU, rd=sr(S_QD + 2), wr=sr(S_QREC0)),
                I(f"s_mov_b32 s{S_OREC0}, s{S_OD + 2}", SALU, rd=sr(S_OD + 2), wr=sr(S_OREC0)),
                I(f"s_mov_b32 s{S_QH}, s{S_QD}", SALU, rd=sr(S_QD), wr=sr(S_QH)),
                I(f"s_mov_b32 s{S_QH + 1}, s{S_QD + 1}", SALU, rd=sr(S_QD + 1), wr=sr(S_QH + 1)),
                I(f"s_mov_b32 s{S_OH}, s{S_OD}", SALU, rd=sr(S_OD), wr=sr(S_OH)),
                I(f"s_mov_b32 s{S_OH + 1}, s{S_OD + 1}", SALU, rd=sr(S_OD + 1), wr=sr(S_OH + 1)),
                I(f"s_mov_b32 s{S_QHS}, s{Hq}", SALU, rd=sr(Hq), wr=sr(S_QHS)),
                I(f"s_mov_b32 s{S_OHS}, s{Hdo}", SALU, rd=sr(Hdo), wr=sr(S_OHS)),
                I(f"s_lshl_b32 s{S_Q32}, s{Rq}, 5", SALU, rd=sr(Rq), wr=sr(S_Q32)),
                I(f"s_lshl_b32 s{S_O32}, s{Rdo}, 5", SALU, rd=sr(Rdo), wr=sr(S_O32))]
        if cont:
            # keys and no rows: the caller stores zeros; else the record N
            ins += [I(f"s_lshl_b32 s{S_W2K}, s{S_WAVE}, 11", SALU, rd=sr(S_WAVE), wr=sr(S_W2K)),
                    I(f"s_cmp_lt_i32 s{T2}, 0", SALU, rd=sr(T2), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {l_epi}", BRANCH)]

            def put(f, x):
                return I(f"v_mov_b32_e32 v{V_N + f}, s{x}", VALU, rd=sr(x), wr=vr(V_N + f))
            ins += [put(N_QH, S_QH), put(N_QH + 1, S_QH + 1), put(N_OH, S_OH), put(N_OH + 1, S_OH + 1),
                    put(N_LH, S_LH), put(N_LH + 1, S_LH + 1), put(N_QREC, S_QREC0), put(N_OREC, S_OREC0),
                    put(N_LREC, S_LREC0), put(N_NSP, S_NSP), put(N_KD, KD), put(N_KD + 1, KD + 1), put(N_KD + 2, KD + 2),
                    put(N_VD, VD), put(N_VD + 1, VD + 1), put(N_VD + 2, VD + 2), put(N_QF, QF), put(N_NLAST, T2),
                    put(N_HL0, S_HLD),
                    I(f"v_mov_b32_e32 v{V_N + N_LANEK}, v{V_LANEK}", VALU, rd=vr(V_LANEK), wr=vr(V_N + N_LANEK))]
            return ins
        # ---- loop state ----
        ins += [I(f"s_lshl_b32 s{S_W2K}, s{S_WAVE}, 11", SALU, rd=sr(S_WAVE), wr=sr(S_W2K)),
                I(f"s_mov_b32 s{S_SDMA}, 0", SALU, wr=sr(S_SDMA)),
                I(f"s_mov_b32 s{S_LDMA}, {LBASE}", SALU, wr=sr(S_LDMA)),
                I(f"s_mov_b32 s{S_LOCD}, 0", SALU, wr=sr(S_LOCD)),
                I(f"s_mov_b32 s{S_LOCL}, 0", SALU, wr=sr(S_LOCL)),
                I(f"s_mov_b32 s{S_LOCV}, 0", SALU, wr=sr(S_LOCV)),
                I(f"s_mov_b32 s{S_Q0V}, s{QF}", SALU, rd=sr(QF), wr=sr(S_Q0V)),
                I(f"s_mov_b32 s{S_NLAST}, s{T2}", SALU, rd=sr(T2), wr=sr(S_NLAST)),
                I(f"s_mov_b32 s{S_N}, 0", SALU, wr=sr(S_N))]
        # zero dV^T, dK^T
        zero = [I(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i)) for i in range(128)]
        if OPT_ZLATE:   # (build() zeroes after the first DMAs; an empty item zeroes out of line)
            l_empty = self.lab("empty")
            self.ool.extend([label(l_empty), nop(15)] + zero + [I(f"s_branch {l_epi}", BRANCH)])
            l_epi = l_empty
        else:
            ins += zero
        # nothing to sweep: epilogue (zeros)
        ins += [I(f"s_cmp_lt_i32 s{S_NLAST}, 0", SALU, rd=sr(S_NLAST), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_epi}", BRANCH)]
        return ins

    def prologue_dma(self):
        """LSE / D of subtiles 0, 1, then three virtual steps (Q / dO of 0..5, LSE / D of 2..7), with
        the cursors' head wraps, in the steady state's issue order"""
        ins = self.dma_l_only() + self.dma_l_only() + self.wrap_check("l")
        for vs in range(3):
            ins += self.dma_subtile(True) + self.dma_subtile(True)
            ins += self.wrap_check("d") + self.wrap_check("l")
            if vs == 0 and OPT_ZLATE and not OPT_CONT:
                ins += [Inst(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i)) for i in range(128)]
        return ins

    def dma_l_only(self):
        I = Inst
        t = S_TMP
        ops = [I(f"s_mov_b32 m0, s{S_LDMA}", SALU, rd=sr(S_LDMA), wr=[("m0", 0)]),
               I(f"buffer_load_dword v{V_L4}, s[{S_LD}:{S_LD + 3}], 0 offen lds", DMA, rd=vr(V_L4) + sr(S_LD, 4) + [("m0", 0)]),
               I(f"s_add_u32 s{S_LD}, s{S_LD}, {LSLOT}", SALU, rd=sr(S_LD), wr=sr(S_LD) + [("scc", 0)]),
               I(f"s_addc_u32 s{S_LD + 1}, s{S_LD + 1}, 0", SALU, rd=sr(S_LD + 1) + [("scc", 0)], wr=sr(S_LD + 1)),
               I(f"s_sub_u32 s{t + 1}, s{S_LD + 2}, {LSLOT}", SALU, rd=sr(S_LD + 2), wr=sr(t + 1) + [("scc", 0)]),
               I(f"s_cselect_b32 s{S_LD + 2}, 0, s{t + 1}", SALU, rd=sr(t + 1) + [("scc", 0)], wr=sr(S_LD + 2)),
               I(f"s_add_u32 s{S_LOCL}, s{S_LOCL}, 1", SALU, rd=sr(S_LOCL), wr=sr(S_LOCL))]
        ops += self.lslot_advance(S_LDMA)
        return ops

    def epilogue(self, stash=V_ST, zero=False):
        """dV = (dV^T)^T, dK = scale (dK^T)^T in bf16 / f16, rows of keys < seqlen_k (range-checked);
        zero: store zeros (an item with keys and no rows, OPT_CONT) for the scalars at v[stash]"""
        I = Inst
        ins = []
        KW0v, HDv, DKO, DVO, PDK, PDV, RDK, RDV, HDK, HDV, SKv = (stash + i for i in (0, 1, 2, 4, 6, 8, 10, 11, 12, 13, 14))
        T0, T1, T2, T3, T4, T5, T6 = (S_TMP + i for i in range(7))

        def rf(v, s):
            return I(f"v_readfirstlane_b32 s{s}, v{v}", RFL, rd=vr(v), wr=sr(s))

        def sa(op, d, a, b, extra_rd=()):
            return I(f"{op} s{d}, s{a}, s{b}", SALU, rd=sr(a) + sr(b) + list(extra_rd), wr=sr(d) + [("scc", 0)])

        # the last steps' DMA (zero records past the sweep) must have landed before the workgroup's LDS
        # is released (moving this wait after the stores measured ±0 at C3 / C5, +0.3..1.8 % at C4)
        # (OPT_CONT: the DMA in flight is the next item's, into ring slots no wave reads now; the item
        # switch waits for it)
        if not OPT_CONT:
            ins += [I("s_waitcnt vmcnt(0)", WAIT)]
        elif OPT_KVAT == "epi" and not zero:
            ins += self.kv_next_ops()
        kvi = []
        if OPT_CONT and OPT_KVAT == "epii" and not zero:    # one load per store group, under the VALU work
            kvi = self.kv_next_ops()
            ins += kvi[:8]
            kvi = kvi[8:]
        ins += [rf(KW0v, T4), rf(HDv, T5), rf(SKv, T6)]
        d0, d1 = (S_EPD, S_EPD + 4) if OPT_CONT else (S_QD, S_OD)
        for dst, ptr, off, rowv, headv, acc, scale in ((d0, PDV, DVO, RDV, HDV, DV, False),
                                                        (d1, PDK, DKO, RDK, HDK, DK, True)):
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
                    # lane offset: r row + 16 hh (lane halves store alternate 8-column groups)
                    I(f"v_and_b32_e32 v{V_TMP}, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(V_TMP)),
                    I(f"v_mul_lo_u32 v{V_TMP}, v{V_TMP}, s{T2}", VALU, rd=vr(V_TMP) + sr(T2), wr=vr(V_TMP)),
                    I(f"v_lshrrev_b32_e32 v{V_TMP + 1}, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(V_TMP + 1)),
                    I(f"v_lshl_add_u32 v{V_TMP + 2}, v{V_TMP + 1}, 4, v{V_TMP}", VALU, rd=vr(V_TMP, 2), wr=vr(V_TMP + 2))]
            # per (d-tile, u pair): lane half 0 writes columns 8 u0 .. +7 (its 4 + its partner's 4),
            # half 1 writes 8 (u0 + 1) .. +7, one dwordx4 each (v_permlane32_swap joins the halves)
            x = 0
            for dt in range(NP):
                for u0 in (0, 2):
                    if kvi:
                        ins.append(kvi.pop(0))
                    if zero:
                        ins.append(I(f"buffer_store_dwordx4 v[{V_ZERO}:{V_ZERO + 3}], v{V_TMP + 2}, s[{dst}:{dst + 3}], 0 offen offset:{64 * dt + 16 * u0}",
                                     VSTORE, rd=vr(V_ZERO, 4) + vr(V_TMP + 2) + sr(dst, 4)))
                        continue
                    w = x + 8
                    for uu in range(2):
                        a = acc + 16 * dt + 4 * (u0 + uu)
                        xs = x + 4 * uu
                        ins += [I(f"v_accvgpr_read_b32 v{xs + k}, a{a + k}", ACCR, rd=ar(a + k), wr=vr(xs + k)) for k in range(4)]
                        if scale:
                            ins += [I(f"v_mul_f32_e32 v{xs + k}, s{S_SCALE}, v{xs + k}", VALU, rd=sr(S_SCALE) + vr(xs + k), wr=vr(xs + k))
                                    for k in range(4)]
                        ins += [self.cvt(w + 2 * uu, xs, xs + 1), self.cvt(w + 2 * uu + 1, xs + 2, xs + 3)]
                    ins += [I(f"v_permlane32_swap_b32_e32 v{w}, v{w + 2}", PERM, rd=vr(w) + vr(w + 2), wr=vr(w) + vr(w + 2)),
                            I(f"v_permlane32_swap_b32_e32 v{w + 1}, v{w + 3}", PERM, rd=vr(w + 1) + vr(w + 3), wr=vr(w + 1) + vr(w + 3))]
                    ins.append(I(f"buffer_store_dwordx4 v[{w}:{w + 3}], v{V_TMP + 2}, s[{dst}:{dst + 3}], 0 offen offset:{64 * dt + 16 * u0}",
                                 VSTORE, rd=vr(w, 4) + vr(V_TMP + 2) + sr(dst, 4)))
                    x = (x + 12) % 60
        # (no wait: the stores complete after the wave ends; the DMAs were drained before them)
        return ins

    # ------------------------------------------------------------------ whole kernel
    def build(self):
        self.lab_end = self.lab("end")
        self.lab_next = self.lab("next")
        self.ool = []         # out-of-line blocks (head wraps)
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
              Inst(f"v_mov_b32_e32 v{V_ROUND}, 0", VALU, wr=vr(V_ROUND))] +
             ([Inst(f"v_mov_b32_e32 v{V_SS + i}, 0", VALU) for i in range(16)] + self.stamp(None) if OPT_STEPSTAMP else []))
        # persistent item loop (fa_bwd_asm.cpp, knob 6): workgroup w runs items r G + (r odd ? rev(w) :
        # w); G = n_items runs one item per workgroup.  The barrier keeps every wave's LDS reads of
        # the previous item ahead of the DMA of this one.
        l_item = self.lab("item")
        code.append(label(l_item))
        T0, T1, T2, T3, T4 = (S_TMP + i for i in range(5))
        head = [Inst("s_barrier", BARRIER),
                Inst(f"s_load_dwordx2 s[{T1}:{T2}], s[0:1], {NITEMS_OFF}", SMEM),     # n_items, grid
                Inst(f"v_readfirstlane_b32 s{T0}, v{V_ROUND}", RFL),
                Inst("s_waitcnt lgkmcnt(0)", WAIT)]
        head += self.n_items_ops(T1)
        head += item_pos_ops(S_ITEM, T0, 2, T2, T3, T4)
        head += [Inst(f"s_cmp_ge_u32 s{S_ITEM}, s{T1}", SALU), Inst(f"s_cbranch_scc1 {self.lab_end}", BRANCH)]
        head += self.stamp(V_SS + 10)
        pro = head + self.prologue(l_epi) + self.stamp(V_SS + 13) + self.prologue_dma() + self.stamp(V_SS + 14)
        # wait: Q / dO(0) (phase -1), Q / dO(1) (its tail prefetches fragments of 1), LSE / D(0, 1)
        # landed; younger than Q / dO(1): L3, Q2, L4, Q3, L5, Q4, L6, Q5, L7 = 21
        pro += [Inst("s_waitcnt vmcnt(21)", WAIT), Inst("s_barrier", BARRIER)]
        pro += self.stamp(V_SS + 15)
        if OPT_STAMP:
            pro += [Inst(f"s_memtime s[{S_TMP + 1}:{S_TMP + 2}]", SMEM), Inst("s_waitcnt lgkmcnt(0)", WAIT),
                    Inst(f"v_mov_b32_e32 v{V_STAMP + 10}, s{S_TMP + 1}", VALU), Inst(f"v_mov_b32_e32 v{V_STAMP + 11}, s{S_TMP + 2}", VALU)]
        emit(pro, pre=[nop(15)])
        # phase -1: chain starts of subtiles 0 (-> buffers 0) and 1 (-> 1), S / dP(0)
        ph = [Inst(f"s_mov_b32 s{S_SROW}, 0", SALU, wr=sr(S_SROW)),
              Inst(f"s_mov_b32 s{S_STR}, {RING - 2 * SLOT}", SALU, wr=sr(S_STR)),   # slot of subtile -2
              Inst(f"s_mov_b32 s{S_LRD}, {LBASE}", SALU, wr=sr(S_LRD)),
              Inst(f"v_add_u32_e32 v{V_KB0}, 0, v{V_RB0}", VALU, rd=vr(V_RB0), wr=vr(V_KB0)),
              Inst(f"v_add_u32_e32 v{V_KB1}, 0, v{V_RB1}", VALU, rd=vr(V_RB1), wr=vr(V_KB1)),
              Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR))]
        ini0 = self.init_reads(0)
        for op in ini0:
            op.dl = 0            # S / dP(0) chains start from them
        ph += ini0
        ph += self.lslot_advance(S_LRD)
        ph += [Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR))]
        ph += self.init_reads(1)
        ph += self.lslot_advance(S_LRD)
        ph += [Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR))]
        mf = self.phase_mfmas(1, True, False)     # S / dP(0) -> buffers 0
        fill = []
        for m, (_, t, i) in enumerate(mf):
            fill += self.frag_reads(m, t, i, key=-100 + m, deadline=max(m - 2, 0))
        fill += self.slot_advance(S_SROW, key=400) + self.slot_advance(S_STR, key=400)
        fill += [Inst(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0), key=401),
                 Inst(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1), key=401),
                 Inst(f"v_add_u32_e32 v{V_VB0}, s{S_STR}, v{V_TB0}", VALU, rd=sr(S_STR) + vr(V_TB0), wr=vr(V_VB0), key=401),
                 Inst(f"v_add_u32_e32 v{V_VB1}, s{S_STR}, v{V_TB1}", VALU, rd=sr(S_STR) + vr(V_TB1), wr=vr(V_VB1), key=401)]
        nm = self.phase_mfmas(0, True, False)     # phase 0 of the first step: S / dP only
        for m in range(3):
            _, t, i = nm[m]
            fill += self.frag_reads(m, t, i, key=600 + m, earliest=m)
        sch = schedule([x[0] for x in mf], ph + fill)
        # step 0 reads Q / dO <= 3 and LSE / D <= 3: the same wait as at every step's end
        sch += [Inst(f"s_waitcnt vmcnt({VMCNT_STEP}) lgkmcnt(0)", WAIT), Inst("s_barrier", BARRIER)]
        sch += self.stamp(V_SS + 5)
        emit(sch, pre=[nop(15)])
        L = {}
        variants = [(f, l, m) for f in (True, False) for l in (True, False) for m in ((True, False) if self.causal else (False,))
                    if not (f and self.causal and not m)]
        for v in variants:
            L[v] = self.lab("step_" + ("".join(c for c, on in zip("FLM", v) if on) or "R"))
        l_tail = self.lab("tail")
        l_disp = self.lab("dispatch")
        l_notlast = self.lab("notlast")
        fm = self.causal
        code += [Inst(f"s_cmp_eq_u32 s{S_NLAST}, 0", SALU), Inst(f"s_cbranch_scc1 {L[(True, True, fm)]}", BRANCH),
                 Inst(f"s_branch {L[(True, False, fm)]}", BRANCH)]
        # dispatch of the next step: done? last? masked (the first 4 subtiles of a head's sweep)?
        code += [label(l_disp), Inst(f"s_cmp_gt_u32 s{S_N}, s{S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_tail}", BRANCH),
                 Inst(f"s_cmp_lt_u32 s{S_N}, s{S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_notlast}", BRANCH)]
        if self.causal:
            code += [Inst(f"s_cmp_lt_u32 s{S_LOCV}, 4", SALU), Inst(f"s_cbranch_scc1 {L[(False, True, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, True, False)]}", BRANCH), label(l_notlast)]
        if self.causal:
            code += [Inst(f"s_cmp_lt_u32 s{S_LOCV}, 4", SALU), Inst(f"s_cbranch_scc1 {L[(False, False, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, False, False)]}", BRANCH)]
        pad = [nop(15)]
        for v in variants:
            f, l, m = v
            code.append(label(L[v]))
            emit(self.step(f, l, m) + self.step_end(l), pre=pad)
            code.append(Inst(f"s_branch {l_disp}", BRANCH))
        code.append(label(l_tail))
        emit(self.tail(), pre=pad)
        code.append(label(l_epi))
        stamp_epi = []
        if OPT_STAMP:
            stamp_epi = [Inst(f"s_memtime s[{S_TMP + 1}:{S_TMP + 2}]", SMEM), Inst("s_waitcnt lgkmcnt(0)", WAIT),
                         Inst(f"v_mov_b32_e32 v{V_STAMP + 12}, s{S_TMP + 1}", VALU),
                         Inst(f"v_mov_b32_e32 v{V_STAMP + 13}, s{S_TMP + 2}", VALU)]
        emit([nop(15)] + stamp_epi + self.epilogue() + self.stamp(V_SS + 6, count=V_SS + 7), pre=pad)
        code.append(label(self.lab_next))
        code += [Inst(f"v_add_u32_e32 v{V_ROUND}, 1, v{V_ROUND}", VALU), Inst(f"s_branch {l_item}", BRANCH)]
        code.append(label(self.lab_end))
        if OPT_STEPSTAMP:
            I = Inst
            code.extend([I("s_waitcnt vmcnt(0)", WAIT), I("s_load_dwordx2 s[52:53], s[0:1], 0xd8", SMEM),
                         I("s_waitcnt lgkmcnt(0)", WAIT),
                         I("s_cmp_eq_u64 s[52:53], 0", SALU), I("s_cselect_b32 s54, 0, 0x7fffffff", SALU),
                         I("s_mov_b32 s55, 0x20000", SALU), I("s_and_b32 s53, s53, 0xffff", SALU),
                         I("s_lshl_b32 s50, s2, 2", SALU), I(f"s_add_u32 s50, s50, s{S_WAVE}", SALU),
                         I("s_lshl_b32 s50, s50, 6", SALU), I(f"v_mov_b32_e32 v{V_SS + 8}, 0", VALU), nop(4),
                         I(f"buffer_store_dwordx4 v[{V_SS}:{V_SS + 3}], v{V_SS + 8}, s[52:55], s50 offen", VSTORE),
                         I(f"buffer_store_dwordx4 v[{V_SS + 4}:{V_SS + 7}], v{V_SS + 8}, s[52:55], s50 offen offset:16", VSTORE),
                         I(f"buffer_store_dwordx4 v[{V_SS + 8}:{V_SS + 11}], v{V_SS + 8}, s[52:55], s50 offen offset:32", VSTORE),
                         I(f"buffer_store_dwordx4 v[{V_SS + 12}:{V_SS + 15}], v{V_SS + 8}, s[52:55], s50 offen offset:48", VSTORE),
                         I("s_waitcnt vmcnt(0)", WAIT)])
        if OPT_STAMP:
            I = Inst
            st = [I("s_waitcnt vmcnt(0)", WAIT),
                  I(f"s_memtime s[{S_TMP + 1}:{S_TMP + 2}]", SMEM), I("s_load_dwordx2 s[52:53], s[0:1], 0xd8", SMEM),
                  I("s_waitcnt lgkmcnt(0)", WAIT),
                  I(f"v_mov_b32_e32 v{V_STAMP + 5}, s{S_TMP + 1}", VALU), I(f"v_mov_b32_e32 v{V_STAMP + 6}, s{S_TMP + 2}", VALU),
                  I(f"v_mov_b32_e32 v{V_STAMP + 7}, s{S_WAVE}", VALU),
                  # a NULL buffer (stamps off) gets zero records: the stores are dropped
                  I("s_cmp_eq_u64 s[52:53], 0", SALU), I("s_cselect_b32 s54, 0, 0x7fffffff", SALU),
                  I("s_mov_b32 s55, 0x20000", SALU),
                  I("s_and_b32 s53, s53, 0xffff", SALU),
                  I(f"v_lshlrev_b32_e32 v{V_STAMP + 8}, 6, v{V_STAMP + 4}", VALU), nop(4),
                  I(f"buffer_store_dwordx4 v[{V_STAMP}:{V_STAMP + 3}], v{V_STAMP + 8}, s[52:55], 0 offen", VSTORE),
                  I(f"buffer_store_dwordx4 v[{V_STAMP + 4}:{V_STAMP + 7}], v{V_STAMP + 8}, s[52:55], 0 offen offset:16", VSTORE),
                  I(f"buffer_store_dwordx4 v[{V_STAMP + 10}:{V_STAMP + 13}], v{V_STAMP + 8}, s[52:55], 0 offen offset:32", VSTORE),
                  I("s_waitcnt vmcnt(0)", WAIT)]
            code.extend(st)
        code.append(Inst("s_endpgm", SOPP))
        code.extend(self.ool)
        return code

    def n_items_ops(self, dst):
        """s[dst] = the item count: kernarg n_items, or with a device-built work list (flags bit 2)
        its first dword (the host only knows an upper bound); uses s56..59"""
        I = Inst
        l = self.lab("nitems")
        return [I(f"s_load_dword s{dst}, s[0:1], {NITEMS_OFF}", SMEM, rd=sr(0, 2), wr=sr(dst)),
                I("s_load_dword s56, s[0:1], 0xd0", SMEM, rd=sr(0, 2), wr=sr(56)),
                I("s_load_dwordx2 s[58:59], s[0:1], 0x38", SMEM, rd=sr(0, 2), wr=sr(58, 2)),
                I("s_waitcnt lgkmcnt(0)", WAIT),
                I("s_bitcmp1_b32 s56, 2", SALU), I(f"s_cbranch_scc0 {l}", BRANCH),
                I(f"s_load_dword s{dst}, s[58:59], 0x0", SMEM, rd=sr(58, 2), wr=sr(dst)),
                I("s_waitcnt lgkmcnt(0)", WAIT), label(l)]

    # ------------------------------------------------------------------ the pipelined item loop
    def geometry_loop(self):
        """(OPT_CONT) the record N of the workgroup's next item with keys and rows, from round V_ROUND
        on; an item with keys and no rows stores zero dK / dV on the way; no item left: an empty
        record (NLAST -1, zero records: the cursors that switch to it DMA zeros)"""
        I = Inst
        T0, T1, T2, T3, T4 = (S_TMP + i for i in range(5))
        top, zero, none, done = self.lab("g_top"), self.lab("g_zero"), self.lab("g_none"), self.lab("g_done")
        ins = [label(top),
               I(f"s_load_dwordx2 s[{T1}:{T2}], s[0:1], {NITEMS_OFF}", SMEM, rd=sr(0, 2), wr=sr(T1, 2)),
               I(f"v_readfirstlane_b32 s{T0}, v{V_ROUND}", RFL, rd=vr(V_ROUND), wr=sr(T0)),
               I("s_waitcnt lgkmcnt(0)", WAIT)]
        ins += self.n_items_ops(T1)
        ins += item_pos_ops(S_ITEM, T0, 2, T2, T3, T4)
        ins += [I(f"s_cmp_ge_u32 s{S_ITEM}, s{T1}", SALU), I(f"s_cbranch_scc1 {none}", BRANCH),
                I(f"v_add_u32_e32 v{V_ROUND}, 1, v{V_ROUND}", VALU, rd=vr(V_ROUND), wr=vr(V_ROUND))]
        ins += self.prologue(zero, l_nokeys=top, cont=True)
        ins += [I(f"s_branch {done}", BRANCH), label(zero)]
        ins += self.epilogue(stash=V_N + N_ST, zero=True)
        ins += [I(f"s_branch {top}", BRANCH), label(none)]
        empty = {N_NLAST: -1, N_NSP: 2}
        ins += [I(f"v_mov_b32_e32 v{V_N + f}, {empty.get(f, 0)}", VALU, wr=vr(V_N + f)) for f in range(N_LEN)]
        ins += [label(done)]
        return ins

    def copy_record(self):
        """(OPT_CONT) C <- N"""
        return [Inst(f"v_mov_b32_e32 v{V_C + f}, v{V_N + f}", VALU, rd=vr(V_N + f), wr=vr(V_C + f)) for f in range(N_LEN)]

    def compute_from_c(self, first):
        """(OPT_CONT) the compute side of the item in C: sweep geometry, mask lane values, the
        epilogue's scalars, the ring read slots (first: from 0; else continuing: v99, v100)"""
        I = Inst
        T1, T2 = S_TMP + 1, S_TMP + 2

        def rf(s_, v):
            return I(f"v_readfirstlane_b32 s{s_}, v{v}", RFL, rd=vr(v), wr=sr(s_))
        ins = [rf(S_QF, V_C + N_QF), rf(S_NLAST, V_C + N_NLAST), rf(S_NSP, V_C + N_NSP),
               I(f"v_mov_b32_e32 v{V_LANEK}, v{V_C + N_LANEK}", VALU, rd=vr(V_C + N_LANEK), wr=vr(V_LANEK))]
        ins += [I(f"v_mov_b32_e32 v{V_ST + i}, v{V_C + N_ST + i}", VALU, rd=vr(V_C + N_ST + i), wr=vr(V_ST + i))
                for i in range(15)]
        ins += [I(f"s_mov_b32 s{S_Q0V}, s{S_QF}", SALU, rd=sr(S_QF), wr=sr(S_Q0V)),
                I(f"s_mov_b32 s{S_LOCV}, 0", SALU, wr=sr(S_LOCV)), I(f"s_mov_b32 s{S_N}, 0", SALU, wr=sr(S_N))]
        if first:
            ins += [I(f"s_mov_b32 s{S_SROW}, 0", SALU, wr=sr(S_SROW)),
                    I(f"s_mov_b32 s{S_STR}, {RING - 2 * SLOT}", SALU, wr=sr(S_STR)),
                    I(f"s_mov_b32 s{S_LRD}, {LBASE}", SALU, wr=sr(S_LRD))]
        else:
            ins += [rf(S_SROW, 99), rf(S_LRD, 100),
                    I(f"s_sub_u32 s{T1}, s{S_SROW}, {2 * SLOT}", SALU, rd=sr(S_SROW), wr=sr(T1)),
                    I(f"s_add_u32 s{T2}, s{T1}, {RING}", SALU, rd=sr(T1), wr=sr(T2)),
                    I(f"s_cmp_lt_i32 s{T1}, 0", SALU, rd=sr(T1), wr=[("scc", 0)]),
                    I(f"s_cselect_b32 s{S_STR}, s{T2}, s{T1}", SALU, rd=sr(T1) + sr(T2) + [("scc", 0)], wr=sr(S_STR))]
        return ins

    def reissue(self, name):
        """(OPT_CONT, at the item switch) the cursor `name` now runs on the compute's item; if it
        stalled at the end of that item, it moves to the next one (record N) and the subtiles it
        DMA'd as zeros are issued again, from the slot where it stalled"""
        I = Inst
        T3, T4 = S_TMP + 3, S_TMP + 4
        sw, stall, slot = (S_DSW, S_DSTALL, S_SDMA) if name == "d" else (S_LSW, S_LSTALL, S_LDMA)
        ok, loop = self.lab("re_ok" + name), self.lab("re_loop" + name)
        ins = [I(f"s_mov_b32 s{sw}, 0", SALU), I(f"s_cmp_eq_u32 s{stall}, -1", SALU), I(f"s_cbranch_scc1 {ok}", BRANCH),
               I(f"s_sub_u32 s{T3}, s{slot}, s{stall}", SALU)]
        if name == "d":
            assert SLOT == 1 << 14
            ins += [I(f"s_add_u32 s{T4}, s{T3}, {RING}", SALU), I(f"s_cmp_lt_i32 s{T3}, 0", SALU),
                    I(f"s_cselect_b32 s{T3}, s{T4}, s{T3}", SALU), I(f"s_lshr_b32 s{T3}, s{T3}, 14", SALU)]
        else:
            ins += [I(f"s_and_b32 s{T3}, s{T3}, {NLS * LSLOT - 1}", SALU), I(f"s_lshr_b32 s{T3}, s{T3}, 8", SALU)]
        ins += [I(f"s_mov_b32 s{slot}, s{stall}", SALU), I(f"s_mov_b32 s{stall}, -1", SALU)]
        ins += self.switch_ops(name)
        ins += [label(loop), I(f"s_cmp_eq_u32 s{T3}, 0", SALU), I(f"s_cbranch_scc1 {ok}", BRANCH)]
        if name == "d":
            ins += self.dma_subtile(False) + self.dma_subtile(False)
        else:
            ins += self.dma_l_only() + self.dma_l_only()
        ins += self.wrap_check(name)
        ins += [I(f"s_sub_u32 s{T3}, s{T3}, 2", SALU), I(f"s_branch {loop}", BRANCH), label(ok)]
        return ins

    def phase_m1(self):
        """phase -1: chain starts of subtiles 0 (-> buffers 0) and 1 (-> 1), S / dP(0); the ring read
        slots S_SROW, S_STR, S_LRD of subtiles 0, -2, 0 (set by the caller under OPT_CONT)"""
        if OPT_CONT:
            ph = [Inst(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0)),
                  Inst(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1))]
        else:
            ph = [Inst(f"s_mov_b32 s{S_SROW}, 0", SALU, wr=sr(S_SROW)),
                  Inst(f"s_mov_b32 s{S_STR}, {RING - 2 * SLOT}", SALU, wr=sr(S_STR)),   # slot of subtile -2
                  Inst(f"s_mov_b32 s{S_LRD}, {LBASE}", SALU, wr=sr(S_LRD)),
                  Inst(f"v_add_u32_e32 v{V_KB0}, 0, v{V_RB0}", VALU, rd=vr(V_RB0), wr=vr(V_KB0)),
                  Inst(f"v_add_u32_e32 v{V_KB1}, 0, v{V_RB1}", VALU, rd=vr(V_RB1), wr=vr(V_KB1))]
        ph += [Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR))]
        ini0 = self.init_reads(0)
        for op in ini0:
            op.dl = 0            # S / dP(0) chains start from them
        ph += ini0
        ph += self.lslot_advance(S_LRD)
        ph += [Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR))]
        ph += self.init_reads(1)
        ph += self.lslot_advance(S_LRD)
        ph += [Inst(f"v_add_u32_e32 v{V_LCUR}, s{S_LRD}, v{V_LB}", VALU, rd=sr(S_LRD) + vr(V_LB), wr=vr(V_LCUR))]
        mf = self.phase_mfmas(1, True, False)     # S / dP(0) -> buffers 0
        fill = []
        for m, (_, t, i) in enumerate(mf):
            fill += self.frag_reads(m, t, i, key=-100 + m, deadline=max(m - 2, 0))
        fill += self.slot_advance(S_SROW, key=400) + self.slot_advance(S_STR, key=400)
        fill += [Inst(f"v_add_u32_e32 v{V_KB0}, s{S_SROW}, v{V_RB0}", VALU, rd=sr(S_SROW) + vr(V_RB0), wr=vr(V_KB0), key=401),
                 Inst(f"v_add_u32_e32 v{V_KB1}, s{S_SROW}, v{V_RB1}", VALU, rd=sr(S_SROW) + vr(V_RB1), wr=vr(V_KB1), key=401),
                 Inst(f"v_add_u32_e32 v{V_VB0}, s{S_STR}, v{V_TB0}", VALU, rd=sr(S_STR) + vr(V_TB0), wr=vr(V_VB0), key=401),
                 Inst(f"v_add_u32_e32 v{V_VB1}, s{S_STR}, v{V_TB1}", VALU, rd=sr(S_STR) + vr(V_TB1), wr=vr(V_VB1), key=401)]
        nm = self.phase_mfmas(0, True, False)     # phase 0 of the first step: S / dP only
        for m in range(3):
            _, t, i = nm[m]
            fill += self.frag_reads(m, t, i, key=600 + m, earliest=m)
        sch = schedule([x[0] for x in mf], ph + fill)
        # step 0 reads Q / dO <= 3 and LSE / D <= 3: the same wait as at every step's end
        sch += [Inst(f"s_waitcnt vmcnt({VMCNT_STEP}) lgkmcnt(0)", WAIT), Inst("s_barrier", BARRIER)]
        sch += self.stamp(V_SS + 5)
        return sch

    def steps_code(self, emit, code):
        """the step dispatch, the step variants and the tail (control flow as build())"""
        L = {}
        variants = [(f, l, m) for f in (True, False) for l in (True, False) for m in ((True, False) if self.causal else (False,))
                    if not (f and self.causal and not m)]
        for v in variants:
            L[v] = self.lab("step_" + ("".join(c for c, on in zip("FLM", v) if on) or "R"))
        l_tail = self.lab("tail")
        l_disp = self.lab("dispatch")
        l_notlast = self.lab("notlast")
        fm = self.causal
        code += [Inst(f"s_cmp_eq_u32 s{S_NLAST}, 0", SALU), Inst(f"s_cbranch_scc1 {L[(True, True, fm)]}", BRANCH),
                 Inst(f"s_branch {L[(True, False, fm)]}", BRANCH)]
        code += [label(l_disp), Inst(f"s_cmp_gt_u32 s{S_N}, s{S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_tail}", BRANCH),
                 Inst(f"s_cmp_lt_u32 s{S_N}, s{S_NLAST}", SALU), Inst(f"s_cbranch_scc1 {l_notlast}", BRANCH)]
        if self.causal:
            code += [Inst(f"s_cmp_lt_u32 s{S_LOCV}, 4", SALU), Inst(f"s_cbranch_scc1 {L[(False, True, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, True, False)]}", BRANCH), label(l_notlast)]
        if self.causal:
            code += [Inst(f"s_cmp_lt_u32 s{S_LOCV}, 4", SALU), Inst(f"s_cbranch_scc1 {L[(False, False, True)]}", BRANCH)]
        code += [Inst(f"s_branch {L[(False, False, False)]}", BRANCH)]
        pad = [nop(15)]
        for v in variants:
            f, l, m = v
            code.append(label(L[v]))
            emit(self.step(f, l, m) + self.step_end(l), pre=pad)
            code.append(Inst(f"s_branch {l_disp}", BRANCH))
        code.append(label(l_tail))
        emit(self.tail(), pre=pad)

    def build_cont(self):
        """the kernel with the pipelined item loop (OPT_CONT): per workgroup
             N <- record(first item); C <- N; N <- record(next); DMA and K / V loads of C's first
             subtiles; then per item: phase -1, steps (the cursors run into N's subtiles at the end
             of C's sweep, the last step loads N's K / V), tail, epilogue; C <- N;
             N <- record(next) (the DMA side's registers saved across it); re-issue a stalled
             cursor; next item"""
        assert not OPT_STAMP, "the workgroup timeline build (FA_GBW_STAMP=1) is for the item-at-a-time loop"
        self.lab_end = self.lab("end")
        self.lab_next = None
        self.ool = []
        code = []
        I = Inst
        pad = [nop(15)]

        def emit(insts, pre=()):
            out, _ = add_waits(insts)
            out, _ = fix_hazards(out, pre=pre)
            code.extend(out)

        T0, T1 = S_TMP, S_TMP + 1
        l_common, l_switch, l_drain = self.lab("common"), self.lab("switch"), self.lab("drain")
        emit([I("v_lshrrev_b32_e32 v1, 6, v0", VALU, rd=vr(0), wr=vr(1)),
              I(f"v_readfirstlane_b32 s{S_WAVE}, v1", RFL, rd=vr(1), wr=sr(S_WAVE)),
              I(f"v_and_b32_e32 v{V_LANE}, 63, v0", VALU, rd=vr(0), wr=vr(V_LANE)),
              I(f"v_mov_b32_e32 v{V_ROUND}, 0", VALU, wr=vr(V_ROUND))] +
             [I(f"v_mov_b32_e32 v{V_ZERO + i}, 0", VALU, wr=vr(V_ZERO + i)) for i in range(4)] +
             ([I(f"v_mov_b32_e32 v{V_SS + i}, 0", VALU) for i in range(16)] + self.stamp(None) if OPT_STEPSTAMP else []))
        zero_acc = [I(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i)) for i in range(128)]
        no_item = [I(f"v_readfirstlane_b32 s{T0}, v{V_N + N_NLAST}", RFL, rd=vr(V_N + N_NLAST), wr=sr(T0)),
                   I(f"s_cmp_lt_i32 s{T0}, 0", SALU, rd=sr(T0), wr=[("scc", 0)]),
                   I(f"s_cbranch_scc1 {l_drain}", BRANCH)]
        # ---- the first item ----
        emit(self.geometry_loop(), pre=pad)
        save = [I(f"v_mov_b32_e32 v{V_SAVE + i}, s{r}", VALU, rd=sr(r), wr=vr(V_SAVE + i)) for i, r in enumerate(DMA_SIDE)]
        restore = [I(f"v_readfirstlane_b32 s{r}, v{V_SAVE + i}", RFL, rd=vr(V_SAVE + i), wr=sr(r)) for i, r in enumerate(DMA_SIDE)]
        emit(no_item + self.copy_record() + save, pre=pad)
        emit(self.geometry_loop(), pre=pad)
        start = restore + self.switch_ops("d", rec=V_C) + self.switch_ops("l", rec=V_C)
        start += [I(f"s_mov_b32 s{r}, {v}", SALU, wr=sr(r)) for r, v in
                  ((S_DSW, 0), (S_LSW, 0), (S_DSTALL, -1), (S_LSTALL, -1), (S_SDMA, 0), (S_LDMA, LBASE))]
        start += self.kv_next_ops(rec=V_C)
        start += self.prologue_dma()
        start += self.compute_from_c(first=True) + zero_acc
        # Q / dO(0), (1), LSE / D(0, 1) and K / V landed; younger than Q / dO(1): 21 (as build())
        start += [I("s_waitcnt vmcnt(21)", WAIT)]
        emit(start, pre=pad)
        code.append(I(f"s_branch {l_common}", BRANCH))
        # ---- the item switch (after the epilogue) ----
        code.append(label(l_switch))
        sw = list(no_item)
        # the continuing ring read slots of the next item's subtile 0 / LSE subtile 0
        sw += [I(f"s_sub_u32 s{T1}, s{S_SROW}, {SLOT}", SALU, rd=sr(S_SROW), wr=sr(T1)),
               I(f"s_add_u32 s{T0}, s{T1}, {RING}", SALU, rd=sr(T1), wr=sr(T0)),
               I(f"s_cmp_lt_i32 s{T1}, 0", SALU, rd=sr(T1), wr=[("scc", 0)]),
               I(f"s_cselect_b32 s{T1}, s{T0}, s{T1}", SALU, rd=sr(T0) + sr(T1) + [("scc", 0)], wr=sr(T1)),
               I(f"v_mov_b32_e32 v99, s{T1}", VALU, rd=sr(T1), wr=vr(99)),
               I(f"s_sub_u32 s{T1}, s{S_LRD}, {2 * LSLOT}", SALU, rd=sr(S_LRD), wr=sr(T1)),
               I(f"s_and_b32 s{T1}, s{T1}, {NLS * LSLOT - 1}", SALU, rd=sr(T1), wr=sr(T1)),
               I(f"s_or_b32 s{T1}, s{T1}, {LBASE}", SALU, rd=sr(T1), wr=sr(T1)),
               I(f"v_mov_b32_e32 v100, s{T1}", VALU, rd=sr(T1), wr=vr(100))]
        sw += self.copy_record() + save
        emit(sw, pre=pad)
        emit(self.geometry_loop(), pre=pad)
        rs = list(restore)
        rs += self.stamp(V_SS + 10)
        rs += zero_acc + [I("s_waitcnt vmcnt(0)", WAIT)]
        rs += self.stamp(V_SS + 11)
        rs += self.reissue("d") + self.reissue("l")
        rs += self.compute_from_c(first=False)
        emit(rs, pre=pad)
        # ---- one item ----
        code.append(label(l_common))
        emit(self.stamp(V_SS + 14) + [I("s_barrier", BARRIER)] + self.stamp(V_SS + 15) + self.phase_m1(), pre=pad)
        self.steps_code(emit, code)
        emit([nop(15)] + self.epilogue() + self.stamp(V_SS + 6, count=V_SS + 7), pre=pad)
        code.append(I(f"s_branch {l_switch}", BRANCH))
        code.append(label(l_drain))
        code.append(I("s_waitcnt vmcnt(0)", WAIT))
        code.append(label(self.lab_end))
        if OPT_STEPSTAMP:
            code.extend([I("s_waitcnt vmcnt(0)", WAIT), I("s_load_dwordx2 s[52:53], s[0:1], 0xd8", SMEM),
                         I("s_waitcnt lgkmcnt(0)", WAIT),
                         I("s_cmp_eq_u64 s[52:53], 0", SALU), I("s_cselect_b32 s54, 0, 0x7fffffff", SALU),
                         I("s_mov_b32 s55, 0x20000", SALU), I("s_and_b32 s53, s53, 0xffff", SALU),
                         I("s_lshl_b32 s50, s2, 2", SALU), I(f"s_add_u32 s50, s50, s{S_WAVE}", SALU),
                         I("s_lshl_b32 s50, s50, 6", SALU), I(f"v_mov_b32_e32 v{V_SS + 8}, 0", VALU), nop(4)] +
                        [I(f"buffer_store_dwordx4 v[{V_SS + 4 * j}:{V_SS + 4 * j + 3}], v{V_SS + 8}, s[52:55], s50 offen offset:{16 * j}", VSTORE)
                         for j in range(4)] + [I("s_waitcnt vmcnt(0)", WAIT)])
        code.append(Inst("s_endpgm", SOPP))
        code.extend(self.ool)
        return code

    def render(self):
        code = self.build_cont() if OPT_CONT else self.build()
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
    kernels = [K(bf, ca, u) for u in (False, True) for bf in (True, False) for ca in (True, False)]
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
