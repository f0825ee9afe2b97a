#!/usr/bin/env python3
"""Generates fa_fwd_asm.s: the gfx950 FlashAttention-2 forward for head dims 128 and 64 (kernels
fa_fwd_asm_d128_* and fa_fwd_asm_d64_*), written as hand-scheduled assembly (one wave per SIMD).

    python3 gen_fwd.py > fa_fwd_asm.s

Algorithm: the reference's compute_attn_1rowblock (csrc/flash_attn/src/flash_fwd_kernel.h:121-583):
per (query block, batch, head) stream K/V tiles, S = Q K^T, online softmax with running max / sum,
O += P V, epilogue O /= l, LSE = m * scale + ln l (+inf when l == 0 or NaN, :509-518), causal mask
top-left (key <= query, softmax.h:143-178).

MI355X structure (MI355X_MICROARCH.md "one wave per SIMD"; cdna_hip_programming.md "4-wave,
one-wave-per-SIMD" attention structure):
  * workgroup = 4 waves x 64 query rows = a 256-row query block; every wave owns two 32-row query
    blocks a (rows 64w..64w+31) and b (+32) and the whole 512-entry register file:
      a[0:127]   O^T accumulators (2 q-blocks x 4 d-tiles x 16)
      a[128:191] Q fragments (B operands of S^T = K Q^T), loaded once
      a[192:223] K fragment ring (8 x 4), a[224:255] V fragment ring (8 x 4)
      v[0:143]   S^T tiles (a: 32, b: 2 x 32) and packed P fragments (a: 2 x 16, b: 16)
  * K/V tiles of 64 keys arrive by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per instruction,
    range-checked descriptors zero-fill keys past seqlen_k) into a 5-deep ring of K and V slots
    (5 x 32 KiB = the whole 160 KiB LDS); tile n+4 is issued during step n, so every tile has about
    three steps to land.  One s_waitcnt vmcnt + s_barrier per step.
  * step n = two phases of 32 MFMAs (v_mfma_f32_32x32x16), each carrying one q-block's softmax in
    its gaps:  phase X: S(n+1, a), S(n+1, b) = K(n+1) Q^T  ||  P(n, b) = exp2(c S(n, b) - c m_b)
               phase Y: O_a, O_b += V(n)^T P(n)            ||  P(n+1, a)
    Each K fragment (ds_read_b128) and V fragment (2 x ds_read_b64_tr_b16) feeds two MFMAs (q-blocks
    a and b).  The filler instructions are placed into the MFMA gaps by isa.schedule (issue budget
    per 32-cycle gap), the wait states by isa.fix_hazards, the counted lgkmcnt waits by isa.add_waits.
  * max-free online softmax: P = exp2(c S - c m_run) against the running max of the first tile; a
    tile whose per-lane partial row sum exceeds 2^8 (or is NaN) is recomputed with the true max
    ("refit", out of line, rare); the deferred-max rule of fa_fwd.hip.
  * scale folded into Q (round 5, FA_GEN_FOLD): tile 0 rewrites the Q fragments as bf16/f16(c Q) and
    every S chain starts from the constant tile -c m_run, so the MFMA hands over c S - c m_run and
    P = exp2(acc) needs no v_fma (reference softmax.h:66-85 does scale * x - max_scaled per score).
  * tiles that need a mask (causal diagonal, ragged last tile) run a MASKED step variant that sets
    the masked scores to -inf before the exponent (per lane limit min(q, sk-1) - key base).
  * work order decoded in the kernel from the workgroup index and the round of the persistent loop
    (fa_params.h ItemDecode, isa.item_decode_ops): heaviest causal blocks first, heads fastest or
    grouped per XCD; varlen launches read a device-built list.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa import (ACCR, ACCW, BARRIER, BRANCH, DMA, LABEL, LDS, MFMA, NOP, PERM, RFL, SALU, SMEM, SOPP,  # noqa: E402
                 TRANS, VALU, VLOAD, VSTORE, WAIT, Counters, Inst, add_waits, ar, fix_hazards, label, nop,
                 item_decode_ops, rtxt, schedule, sr, vr)

import isa as _isa  # noqa: E402

# scheduling weights (round 4 A/B, profiles/r04/ab_sched_weights_r04.txt): an LDS read weighs 4 issue
# cycles in the gap budget (2 before), spreading the reads over more MFMA gaps; an LDS-DMA piece 24
# (round 5: 8 before; MI355X_MICROARCH.md prices one at 60-185 cycles beside MFMAs -- C3 forward
# -0.7 %, bitwise identical, profiles/r05/ab_dma24_r05b.txt)
_isa.apply_costs("LDS=4,DMA=24")
_isa.apply_costs(os.environ.get("FA_ISA_COST", ""))
_isa.apply_costs(os.environ.get("FA_GEN_COST", ""))
BN = 64               # keys per K/V tile
BM = 256              # query rows per workgroup
NSLOT = 5


def configure(d):
    """head dim of the kernels generated next (128 or 64): K/V tiles of 64 keys x d, D / 32 column
    blocks of 64 bytes per key row (one DMA piece each), AGPR layout O | Q | K ring | V ring"""
    global D, KS, NP, TILE, VBASE, LDS_BYTES, QB, KF, VF, NX, NY
    D = d
    KS = D // 16          # QK^T k-steps
    NP = D // 32          # d tiles of O = column blocks of a K/V tile
    TILE = BN * D * 2     # bytes per K (or V) tile
    VBASE = NSLOT * TILE
    LDS_BYTES = 2 * NSLOT * TILE
    assert LDS_BYTES <= 163840
    QB = 2 * NP * 16
    KF = QB + 2 * KS * 4
    VF = KF + 32
    NX = 2 * KS * 2       # phase X MFMAs: S(n+1) of 2 q-blocks, 2 key subtiles
    NY = NP * 8           # phase Y MFMAs: PV(n) of 2 q-blocks


configure(128)


# ---- AGPRs ----
def O_(j, dt):
    return 2 * NP * 8 * j + 16 * dt


def Q_(j, ks):
    return QB + KS * 4 * j + 4 * ks

# ---- VGPRs ----
SA = 0


def SB(p):
    return 32 + 32 * p


def PA(p):
    return 96 + 16 * p


PB = 128
V_RB0, V_RB1, V_TB0, V_TB1 = 144, 145, 146, 147        # lane LDS bases (no slot)
V_KB0, V_KB1, V_VB0, V_VB1 = 148, 149, 150, 151        # current K / V read bases
V_VOFF = 152                                             # 4 DMA voffsets (152..155)
V_NEGMC = (156, 157)                                     # -m*c per q-block
V_L = (158, 159)                                         # running row sums (this lane's keys)
V_PS = (160, 161)                                        # partial sums of the current tile
V_LB = (162, 163)                                        # mask limit bases
V_LM = (164, 165)                                        # mask limits of the current tile (st 0, 1)
V_NINF = 166
V_T = 167                                                # temps 167..183
V_QOFF = (184, 185)                                      # Q / O row offsets per q-block
V_LSEOFF = (186, 187)
V_LANE = 188
V_OOFF = (189, 190)
V_ROW = (192, 193)                                       # row of the lane in the block, per q-block
V_HH4 = 194                                              # 4 * (lane >> 5)
V_TRI = 196   # 196..211: causal diagonal chain start (-inf where key > query in a 32 x 32 S^T subtile)
V_NT = 212    # 212..227: all -inf chain start (a subtile wholly above the diagonal; not with the fold)
NVGPR = 228
# scale folded into Q (round 5 default; FA_GEN_FOLD=0 restores the per-score v_fma): the Q fragments
# hold bf16/f16(c Q) with c = scale * log2(e), every S chain starts from the constant tile -c m_run of
# its q-block (V_M[j], 16 registers of V_NEGMC[j]), so a score leaves the MFMA as c S - c m_run and
# P = v_exp_f32(acc) -- one VALU op per score instead of two.  Scores wholly above the causal
# diagonal are written as -inf (no chain), so the all -inf tile V_NT gives its registers to V_M.
OPT_FOLD = os.environ.get("FA_GEN_FOLD", "1") == "1"
NAME = "fa_fwd_asm"     # kernel name prefix (gen_fwdnf.py: the unfolded kernels, "fa_fwdnf_asm")
V_M = (212, 228)      # 212..227, 228..243
if OPT_FOLD:
    NVGPR = 244

# ---- SGPRs ----
S_KD, S_VD, S_QD, S_OD, S_LD = 4, 8, 12, 16, 20          # buffer descriptors
S_WARM = 3        # 1: the next item's K/V tiles 0..2 and its Q are in flight (set by the switch block)
S_ROUND = 24      # round r of the persistent item loop (item position: r G + (r odd ? G-1-w : w))
S_N = 25          # step n
S_N0 = 26         # 64 n
S_NF2 = 27        # nfast - 2
S_NL1 = 28        # nblk - 1
S_KOFF = 29       # K slot offset of the tile phase X reads
S_VOFF = 30       # V slot offset (incl. VBASE) of the tile phase Y reads
S_DOFF = 31       # K slot offset of the next DMA tile + wave * 1024
S_TB = 32         # tile bytes = 64 * kv_row
S_DT = 33         # index of the next DMA tile
S_NBLK = 34
S_WAVE = 35
S_TMP = 36        # 36..39 temps
S_KA = 40         # kernarg block 40..84 (84: grid)
S_C = S_KA + 41   # scale * log2(e) (kernarg)
S_NITEMS = S_KA + 43
S_GRID = S_KA + 44
# FA_GEN_DECBURST=1 (dev switch, off in the shipped build): the first item's ItemDecode comes with the
# kernargs (one scalar round trip less per workgroup; profiles/r06/ab_*_decburst_r06s3.txt), so the
# rng_state store descriptor moves off s[92:95]
OPT_DECBURST = os.environ.get("FA_GEN_DECBURST") == "1"
S_RNGD = S_KD if OPT_DECBURST else 92   # rng_state store descriptor, written once in entry(), before the geometry
# persistent item loop: the NEXT item's descriptors (its K/V tiles are DMA'd into the ring while the
# current item finishes, its Q is loaded in the current item's last step)
S_QD2 = 56        # over the rng / seed / offset kernargs (dead after the rng store)
S_DLIM = 60       # tiles of the item the DMA stream currently reads (S_DT counts the issued ones)
S_NXN = 61        # tiles of the next item (0: none / empty)
S_KD2, S_VD2 = 92, 96
S_SWT = 100       # switch-block temp
S_WD = 85         # wave + m0 / 64: a diagonal tile t is visible to this wave (u = S_WD - t >= 1),
                  # on its diagonal (u = 0) or above it (u < 0)
S_M0R = 101       # 256 m_block of the item being set up (prologue temp)
NSGPR = 102

KARG_SIZE = 224
DEC_OFF = 184    # fa_params.h ItemDecode (40 bytes) after FwdAsmArgs' 184

# dev A/B switches, read when the .s is generated (tools/asm_variant.sh)
OPT_NOZERO = os.environ.get("FA_GEN_NOZERO") == "1"          # never zero K/V record counts
OPT_NODIAG = os.environ.get("FA_GEN_NODIAG") == "1"          # causal diagonal: generic masked steps only
OPT_PLAIN_SNAKE = os.environ.get("FA_GEN_PLAIN_SNAKE") == "1"  # snake reversal over single workgroups
OPT_BUDGET = int(os.environ.get("FA_GEN_BUDGET", "24"))        # filler issue cycles per MFMA gap
# ... at head dim 64, where the softmax VALU outweighs the 16 MFMAs of a phase: a fuller gap (32)
# ran C2 -0.7 / -0.9 % in two one-process A/Bs, 40 +-0, 48 / 64 +3 / +5 % (profiles/r05/ab_b64*_c2_r05p.txt)
OPT_BUDGET64 = int(os.environ.get("FA_GEN_BUDGET64", "32"))
OPT_ZERO_NOP = int(os.environ.get("FA_GEN_ZERO_NOP", "0"))    # s_nop 15 x N before zeroing them
OPT_SHIFT = int(os.environ.get("FA_GEN_SHIFT", "0"))          # s_nop 0 x N at the kernel entry (code placement)
OPT_ALIGN = int(os.environ.get("FA_GEN_ALIGN", "0"))          # .p2align N before each step body (code placement)
# dev clock / cycle stamps: every wave stores {s_memtime, s_memrealtime} at its start and end, the
# tiles and items it ran, HW_ID, XCC_ID to the buffer passed as the `seed` kernarg (tools/fwd_stamps.py)
OPT_MFZERO = os.environ.get("FA_GEN_MFZERO") == "1"          # zero O with 2 NP MFMAs (zero operands)
OPT_EPI2 = os.environ.get("FA_GEN_EPI2") == "1"              # epilogue: groups interleaved stage by stage
OPT_LAST2 = os.environ.get("FA_GEN_LAST2") == "1"            # last step: PV(a) under softmax(b), then PV(b)
OPT_NOGUARD = os.environ.get("FA_GEN_NOGUARD") == "1"        # ablation (wrong on a refit): no guard branch
OPT_SM_ABL = os.environ.get("FA_GEN_SM_ABL", "").split(",")  # ablation (wrong results): nosum / noexp / nocvt
OPT_T0OV = os.environ.get("FA_GEN_T0OV") == "1"              # tile 0: QK(a), then QK(b) || max / softmax(a)
# guard: compare as soon as the partial sum is complete, branch on vcc later (round 4 default: the
# compare + s_cmp + branch in one place stalled the wave, 1.3 % at C3; FA_GEN_GUARD1=1 restores it)
OPT_GUARD2 = os.environ.get("FA_GEN_GUARD1") != "1"
# epilogue ablations (wrong results; with FA_GEN_STAMP=3 they split its cost): no O stores / only them
OPT_EPI_ABL = os.environ.get("FA_GEN_EPI_ABL", "")
# deferred epilogue stores: the epilogue leaves O (packed) and the LSE in registers that the next
# item's tile 0 does not touch, and its O / LSE stores issue in the gaps of that tile 0's MFMAs --
# after its s_waitcnt (vmcnt counts stores: stores queued ahead of the wait were waited for) and
# spread one per gap (a store of 32 rows x 32 bytes holds the wave's issue for ~76 cycles)
OPT_DEFER = os.environ.get("FA_GEN_DEFER") == "1"
# O zeroed by v_accvgpr_write in the gaps of tile 0's MFMAs instead of ahead of them (an empty item,
# which runs no tile 0, zeroes it on its own branch)
OPT_T0ZERO = os.environ.get("FA_GEN_T0ZERO") == "1"
# cache-policy modifiers of the epilogue's O stores (dev A/B), e.g. "nt"
OPT_OPOL = (" " + os.environ["FA_GEN_OPOL"]) if os.environ.get("FA_GEN_OPOL") else ""
# cold item start: the Q fragment loads are waited for by tile 0's vmcnt wait (they are older than
# the K / V DMA it waits for) instead of before the DMA issue -- one memory round trip less per cold
# item (round 6; FA_GEN_QWAIT=1 restores the wait, which an item with no tiles still takes)
OPT_QWAIT = os.environ.get("FA_GEN_QWAIT") == "1"
# O staged through LDS (the K/V slot of the item's last tile, free after the last step): each store
# then writes whole rows (4 rows of 256 B at d = 128) instead of 32 rows x 32 B (round 4 default:
# C3 -0.3 %, C4 -0.4 %, C2 ±0, bitwise identical; FA_GEN_OSTAGE=0 restores the direct stores)
OPT_OSTAGE = os.environ.get("FA_GEN_OSTAGE", "1") == "1"
V_LSEV = (191, 195)                   # LSE values of the finished item (deferred stores)
V_SAVE = (228, 229, 230, 231, 238, 239)   # its O / LSE descriptor words 0..2 across the warm start
S_ODD, S_LDD = 88, 36                 # ... restored here for tile 0 (geometry temps, free by then)


def PKR(j, dt, u):
    """(deferred stores) packed O of q-block j, d-tile dt, column half u: v64..95 and v112..143 (S(1)
    / P(1) / P(b): idle in tile 0)"""
    i = 32 * j + 4 * (2 * dt + u // 2)
    return 64 + i if i < 32 else 112 + (i - 32)
V_ZERO = 228      # 228..231: zeros (MFMA operands of the O zeroing)
OPT_STAMP = os.environ.get("FA_GEN_STAMP") in ("1", "2", "3", "4")
# FA_GEN_STAMP=2 also sums, per wave, the cycles of each step's compute, its vmcnt/lgkmcnt wait and
# its barrier wait (s_memtime around the step-end wait and barrier; perturbs the schedule a little)
OPT_STEPSTAMP = os.environ.get("FA_GEN_STAMP") in ("2", "3", "4")
# FA_GEN_STAMP=3: the tile-0 / item-start accumulators time the epilogue's parts instead (LSE of both
# q-blocks -> tile 0's slot, O of q-block a -> item start's slot, O of q-block b -> the epilogue's)
OPT_EPISTAMP = os.environ.get("FA_GEN_STAMP") == "3"
# FA_GEN_STAMP=4: the item start split -- geometry (epilogue end -> tile 0's wait) in the item-start
# slot, tile 0's vmcnt wait in the tile-0 slot, its barrier wait in V_SSUM + 5 (record offset 96)
OPT_T0STAMP = os.environ.get("FA_GEN_STAMP") == "4"
OPT_STAMP_NONFAST = os.environ.get("FA_GEN_STAMP_ONLY") == "nonfast"
V_SSUM = 174 if OPT_FOLD else 240   # +0..4: compute, wait, barrier sums, step count, last stamp;
                  # +6..9: item phases: tile 0, last step, epilogue, item start (geometry .. tile 0's barrier)
# latency-aware gap scheduling (isa.schedule lat=): "valu,trans,lds,mfma" result latencies in cycles
_lat = os.environ.get("FA_GEN_LAT")
OPT_LAT = None
if _lat:
    _v = [int(x) for x in _lat.split(",")]
    OPT_LAT = {VALU: _v[0], PERM: _v[0], TRANS: _v[1], LDS: _v[2], MFMA: _v[3]}
V_STAMP = 244 if OPT_FOLD else 232     # +0..5: start memtime lo / hi, realtime lo / hi, tiles, items
# dev options whose registers the fold's V_M tiles take, or that predate it
assert not (OPT_FOLD and (OPT_DEFER or OPT_MFZERO or OPT_T0OV or OPT_LAST2)), \
    "FA_GEN_DEFER / MFZERO / T0OV / LAST2 need FA_GEN_FOLD=0"
# debug: at the named point, workgroup 0 stores every register of each wave (and wave 0 the LDS) to
# the buffer whose address is passed as the `seed` kernarg, then ends (tools/asm_dump.py)
OPT_DUMP = os.environ.get("FA_GEN_DUMP")
DUMP_SLOTS = 512 + 128   # per wave: v0..v255, a0..a255, s0..s127 -- 256 bytes (64 lanes) each


class K:
    """one kernel variant"""

    def __init__(self, bf16, causal):
        self.bf16 = bf16
        self.causal = causal
        self.ty = "bf16" if bf16 else "f16"
        self.name = f"{NAME}_d{D}_{self.ty}_{'causal' if causal else 'full'}"
        self.lines = []
        self.uid = 0
        self.refit_regs = {}

    def lab(self, s):
        self.uid += 1
        return f".L{self.name}_{s}_{self.uid}"

    def stamp_point(self, acc):
        """(FA_GEN_STAMP=2) v[V_SSUM + acc] += now - last stamp; last stamp = now"""
        if not OPT_STEPSTAMP:
            return []
        t0 = V_T
        # (s[100:101]: dead at every stamp point; S_TMP may hold the deferred LSE descriptor)
        return [Inst(f"s_memtime s[{S_SWT}:{S_SWT + 1}]", SMEM), Inst("s_waitcnt lgkmcnt(0)", WAIT),
                Inst(f"v_mov_b32_e32 v{t0}, s{S_SWT}", VALU),
                Inst(f"v_sub_u32_e32 v{t0 + 1}, v{t0}, v{V_SSUM + 4}", VALU),
                Inst(f"v_add_u32_e32 v{V_SSUM + acc}, v{V_SSUM + acc}, v{t0 + 1}", VALU),
                Inst(f"v_mov_b32_e32 v{V_SSUM + 4}, v{t0}", VALU)]

    # ------------------------------------------------------------------ instruction builders
    def mfma_s(self, st_reg, kslot, j, ks, first, bias=None):
        """S^T chain step; the first step starts from 0 or from a bias tile (bias: VGPR base of a
        16-register chain start: a -inf / 0 mask tile, the causal mask folded into the chain start,
        and / or, with the fold, the -c m_run tile of the q-block)"""
        if first:
            c = "0" if bias is None else rtxt("v", bias, 16)
            rc = [] if bias is None else vr(bias, 16)
        else:
            c = rtxt("v", st_reg, 16)
            rc = vr(st_reg, 16)
        t = (f"v_mfma_f32_32x32x16_{self.ty} {rtxt('v', st_reg, 16)}, {rtxt('a', KF + 4 * kslot, 4)}, "
             f"{rtxt('a', Q_(j, ks), 4)}, {c}")
        rd = ar(KF + 4 * kslot, 4) + ar(Q_(j, ks), 4) + rc
        return Inst(t, MFMA, rd=rd, wr=vr(st_reg, 16), rd_c=rc)

    def mfma_o(self, j, dt, vslot, preg):
        o = O_(j, dt)
        t = (f"v_mfma_f32_32x32x16_{self.ty} {rtxt('a', o, 16)}, {rtxt('a', VF + 4 * vslot, 4)}, "
             f"{rtxt('v', preg, 4)}, {rtxt('a', o, 16)}")
        return Inst(t, MFMA, rd=ar(VF + 4 * vslot, 4) + vr(preg, 4) + ar(o, 16), wr=ar(o, 16), rd_c=ar(o, 16))

    def kread(self, f, kslot, **kw):
        st, ks = f // KS, f % KS
        base = V_KB0 if ks % 2 == 0 else V_KB1
        off = (ks // 2) * BN * 64 + st * 32 * 64
        return Inst(f"ds_read_b128 {rtxt('a', KF + 4 * kslot, 4)}, v{base} offset:{off}", LDS,
                    rd=vr(base), wr=ar(KF + 4 * kslot, 4), **kw)

    def vread(self, f, vslot, half, **kw):
        dt, kk = f // 4, f % 4
        base = V_VB0 if half == 0 else V_VB1
        off = dt * BN * 64 + kk * 16 * 64 + half * 8 * 64
        dst = VF + 4 * vslot + 2 * half
        return Inst(f"ds_read_b64_tr_b16 {rtxt('a', dst, 2)}, v{base} offset:{off}", LDS,
                    rd=vr(base), wr=ar(dst, 2), **kw)

    def cvt(self, dst, s0, s1, **kw):
        return Inst(f"v_cvt_pk_{self.ty}_f32 v{dst}, v{s0}, v{s1}", VALU, rd=vr(s0) + vr(s1), wr=vr(dst), **kw)

    # ------------------------------------------------------------------ softmax op lists
    def mask_ops(self, j, sreg, kbase_sgpr_add, lm, key0=0):
        """scores of q-block j at v[sreg..+31] whose key exceeds the lane limit become -inf.  The limit
        of subtile st (32 keys) is V_LB[j] - key base - 32 st, kept in v[lm[st]]; element g of a lane
        holds key base + acc_row(g, hh), masked iff (g & 3) + 8 (g >> 2) > V_LB - base (V_LB already
        holds min(q, sk - 1) - 4 hh).  kbase_sgpr_add: key base = sgpr + add."""
        ops = []
        sg, add = kbase_sgpr_add
        ops.append(Inst(f"v_subrev_u32 v{lm[0]}, s{sg}, v{V_LB[j]}", VALU, rd=sr(sg) + vr(V_LB[j]), wr=vr(lm[0]), key=key0))
        if add:
            ops.append(Inst(f"v_subrev_u32 v{lm[0]}, {add}, v{lm[0]}", VALU, rd=vr(lm[0]), wr=vr(lm[0]), key=key0))
        ops.append(Inst(f"v_subrev_u32 v{lm[1]}, 32, v{lm[0]}", VALU, rd=vr(lm[0]), wr=vr(lm[1]), key=key0))
        for e in range(32):
            st, g = e // 16, e % 16
            reg = sreg + e
            const = (g & 3) + 8 * (g >> 2)
            ops.append(Inst(f"v_cmp_gt_i32_e32 vcc, {const}, v{lm[st]}", VALU, rd=vr(lm[st]), wr=[("vcc", 0)], key=key0 + 4 * e))
            ops.append(Inst(f"v_cndmask_b32_e32 v{reg}, v{reg}, v{V_NINF}, vcc", VALU,
                            rd=vr(reg) + vr(V_NINF) + [("vcc", 0)], wr=vr(reg), key=key0 + 4 * e))
        return ops

    def softmax_ops(self, j, sreg, preg, masked, kbase_sgpr_add, key0, lm=None, fold_add=False):
        """ops of P = exp2(c S - c m) for q-block j on the 32 scores at v[sreg..+31] -> packed P at
        v[preg..+15]; partial row sum into V_PS[j] (masked: mask_ops first).  With the fold the
        scores already are c S - c m (chain start V_M[j]): P = exp2(score); fold_add: scores c S from
        a chain started at 0 (tile 0, refit), - c m added first.  Dependencies among the ops are
        derived from their registers by isa.schedule.  Returns (ops, last sum op)."""
        ops = self.mask_ops(j, sreg, kbase_sgpr_add, lm or V_LM, key0) if masked else []
        k = key0
        last_sum = None
        for e in range(32):
            st, g = e // 16, e % 16
            reg = sreg + e
            kk = 4 * e
            if not OPT_FOLD:
                ops.append(Inst(f"v_fma_f32 v{reg}, v{reg}, s{S_C}, v{V_NEGMC[j]}", VALU,
                                rd=vr(reg) + sr(S_C) + vr(V_NEGMC[j]), wr=vr(reg), key=k + kk + 1))
            elif fold_add:
                ops.append(Inst(f"v_add_f32_e32 v{reg}, v{V_NEGMC[j]}, v{reg}", VALU, rd=vr(reg) + vr(V_NEGMC[j]),
                                wr=vr(reg), key=k + kk + 1))
            if "noexp" not in OPT_SM_ABL:
                ops.append(Inst(f"v_exp_f32_e32 v{reg}, v{reg}", TRANS, rd=vr(reg), wr=vr(reg), key=k + kk + 2))
            if e > 1 and "nosum" in OPT_SM_ABL:
                pass
            elif e == 1:    # (p1 + p0: the first two terms in one add, no copy of p0)
                a = Inst(f"v_add_f32_e32 v{V_PS[j]}, v{reg}, v{reg - 1}", VALU, rd=vr(reg) + vr(reg - 1),
                         wr=vr(V_PS[j]), key=k + kk + 3)
            elif e > 1:
                a = Inst(f"v_add_f32_e32 v{V_PS[j]}, v{reg}, v{V_PS[j]}", VALU, rd=vr(reg) + vr(V_PS[j]),
                         wr=vr(V_PS[j]), key=k + kk + 3)
            if e == 1 or (e > 1 and "nosum" not in OPT_SM_ABL):
                last_sum = a
                ops.append(a)
            if e % 2 == 1 and "nocvt" not in OPT_SM_ABL:
                kkf = 2 * st + (g >> 3)
                w = (g & 7) >> 1
                ops.append(self.cvt(preg + 4 * kkf + w, reg - 1, reg, key=k + kk + 3))
        return ops, last_sum

    def touched(self, refit_label):
        """the registers the out-of-line refit block at refit_label writes (scc, vcc, S_TMP, V_T, its
        fragment ring, ...): its guard branch declares them as read and written, so the gap scheduler
        keeps every filler that uses one of them wholly before or wholly after the branch -- an
        s_cmp / s_cselect pair or an S_TMP temporary live across the branch would be clobbered when
        the refit runs (found in the emulator: a refit between a slot advance's s_sub and its
        s_cselect corrupted O)"""
        return sorted(self.refit_regs.get(refit_label, ()))

    def guard_ops(self, j, refit_label, key, deadline=None):
        """partial sum <= 2^8 on every lane (and not NaN), else refit; then l += partial.  The branch
        and its return label are one instruction so that nothing is scheduled between them."""
        add = Inst(f"v_add_f32_e32 v{V_L[j]}, v{V_L[j]}, v{V_PS[j]}", VALU, rd=vr(V_L[j]) + vr(V_PS[j]),
                   wr=vr(V_L[j]), key=key, deadline=deadline)
        if OPT_NOGUARD:
            return [Inst(f"{refit_label}_back:", LABEL, key=key), add]
        cmp = Inst(f"v_cmp_nge_f32_e32 vcc, 0x43800000, v{V_PS[j]}", VALU, rd=vr(V_PS[j]), wr=[("vcc", 0)],
                   key=key, deadline=deadline)
        sc = Inst("s_cmp_lg_u64 vcc, 0", SALU, rd=[("vcc", 0)], wr=[("scc", 0)], key=key, deadline=deadline)
        tch = self.touched(refit_label)
        br = Inst(f"s_cbranch_scc1 {refit_label}\n{refit_label}_back:", BRANCH, rd=[("scc", 0)] + tch, wr=tch,
                  key=key, deadline=deadline)
        add = Inst(f"v_add_f32_e32 v{V_L[j]}, v{V_L[j]}, v{V_PS[j]}", VALU, rd=vr(V_L[j]) + vr(V_PS[j]),
                   wr=vr(V_L[j]), key=key, deadline=deadline)
        return [cmp, sc, br, add]

    def guard_cmp(self, j, key):
        """(FA_GEN_GUARD2) the guard's compare alone: vcc = partial sum > 2^8 or NaN.  Scheduled as
        soon as the sum is complete; the branch reads vcc later, so the wave does not stall on it."""
        return Inst(f"v_cmp_nge_f32_e32 vcc, 0x43800000, v{V_PS[j]}", VALU, rd=vr(V_PS[j]), wr=[("vcc", 0)], key=key)

    def guard_br(self, j, refit_label, key, deadline=None, eg=None):
        """(FA_GEN_GUARD2) branch to the refit on vcc (all lanes are active), then l += partial"""
        tch = self.touched(refit_label)
        br = Inst(f"s_cbranch_vccnz {refit_label}\n{refit_label}_back:", BRANCH, rd=[("vcc", 0)] + tch, wr=tch,
                  key=key, deadline=deadline, earliest=eg)
        add = Inst(f"v_add_f32_e32 v{V_L[j]}, v{V_L[j]}, v{V_PS[j]}", VALU, rd=vr(V_L[j]) + vr(V_PS[j]),
                   wr=vr(V_L[j]), key=key, deadline=deadline, earliest=eg)
        return [br, add]

    # ------------------------------------------------------------------ the item's last step (no QK)
    def step_last2(self, p, tag):
        """the last step (tile n = the item's last, no QK(n+1)): phase X runs PV(n) of q-block a --
        whose P was made in the previous step -- with softmax(n, b) and its guard in the gaps; phase
        Y runs PV(n) of q-block b with the next item's Q loads.  (The plain last step runs softmax(n,
        b) with no MFMA beside it.)  V fragments: phase X reads all 4 NP; at d = 128 phase Y uses
        the 8 still in the ring first (d-tiles 2, 3) and re-reads those of d-tiles 0, 1."""
        refits = []
        nv = 4 * NP
        mx = [self.mfma_o(0, f // 4, f % 8, PA(p) + 4 * (f % 4)) for f in range(nv)]
        fx = [Inst(f"v_add_u32_e32 v{V_VB0}, s{S_VOFF}, v{V_TB0}", VALU, rd=sr(S_VOFF) + vr(V_TB0), wr=vr(V_VB0), key=-200),
              Inst(f"v_add_u32_e32 v{V_VB1}, s{S_VOFF}, v{V_TB1}", VALU, rd=sr(S_VOFF) + vr(V_TB1), wr=vr(V_VB1), key=-200)]
        for f in range(nv):
            for h in range(2):
                fx.append(self.vread(f, f % 8, h, key=-150 + 2 * f + h, earliest=(f - 8 + 1) if f >= 8 else None,
                                     deadline=max(f - 2, 0)))
        sm_b, _ = self.softmax_ops(1, SB(p), PB, True, (S_N0, 0), key0=0)
        fx += sm_b
        rl_b = self.lab(f"{tag}_refit_b")
        refits.append(self.refit(1, SB(p), PB, rl_b, tile_add=0, phase="Y"))
        fx += self.guard_ops(1, rl_b, key=600)
        xs = schedule(mx, fx, budget=(OPT_BUDGET64 if D == 64 else OPT_BUDGET))
        order = list(range(8, nv)) + list(range(min(8, nv)))
        my = [self.mfma_o(1, f // 4, f % 8, PB + 4 * (f % 4)) for f in order]
        fy = []
        if nv > 8:
            for f in range(8):
                for h in range(2):
                    fy.append(self.vread(f, f % 8, h, key=-150 + 2 * f + h, earliest=f + 1, deadline=8 + f - 2))
        # Q of the next item (persistent loop): no QK MFMA reads the Q registers from here on
        for j in range(2):
            for ks in range(KS):
                fy.append(Inst(f"buffer_load_dwordx4 {rtxt('a', Q_(j, ks), 4)}, v{V_QOFF[j]}, s[{S_QD2}:{S_QD2 + 3}], 0 offen offset:{32 * ks}",
                               VLOAD, rd=vr(V_QOFF[j]) + sr(S_QD2, 4), wr=ar(Q_(j, ks), 4), key=900 + 8 * j + ks))
        t = S_TMP
        fy += [Inst(f"s_add_u32 s{S_VOFF}, s{S_VOFF}, {TILE}", SALU, rd=sr(S_VOFF), wr=sr(S_VOFF) + [("scc", 0)], key=800),
               Inst(f"s_sub_u32 s{t + 2}, s{S_VOFF}, {NSLOT * TILE}", SALU, rd=sr(S_VOFF), wr=sr(t + 2) + [("scc", 0)], key=801),
               Inst(f"s_cmp_ge_u32 s{S_VOFF}, {VBASE + NSLOT * TILE}", SALU, rd=sr(S_VOFF), wr=[("scc", 0)], key=802),
               Inst(f"s_cselect_b32 s{S_VOFF}, s{t + 2}, s{S_VOFF}", SALU, rd=sr(t + 2) + sr(S_VOFF) + [("scc", 0)], wr=sr(S_VOFF), key=803)]
        ys = schedule(my, fy, budget=(OPT_BUDGET64 if D == 64 else OPT_BUDGET))
        return xs + ys, refits

    # ------------------------------------------------------------------ one pipelined step
    def step(self, p, variant, tag):
        """step n: phase X (QK(n+1) || softmax(n, b)), phase Y (PV(n) || softmax(n+1, a)).
        variant: 'fast', 'masked' or 'last', or (causal, a full diagonal tile n+1 that is not the
        item's last) 'diag' / 'dead': the fast step with the causal mask of S(n+1) folded into the
        chain starts -- on this wave's diagonal the 32 x 32 subtiles (q-block j, key subtile st) are
        the triangle (j == st), wholly visible (j > st) or wholly hidden (j < st); above it, all
        hidden.  Returns (instruction list, refit blocks)."""
        last = variant == "last"
        masked = variant in ("masked", "last")
        if last and OPT_LAST2:
            return self.step_last2(p, tag)

        # fold: the triangle's chain start V_TRI + (-c m) is built per diagonal step in PA(p ^ 1), which
        # is idle during phase X (P(n-1, a) was read by the previous step's PV, P(n+1, a) is written
        # in phase Y): q-block a's before MFMA 0, then q-block b's once MFMA 0 has read it
        tri = PA(p ^ 1)

        def bias(j, st):
            if OPT_FOLD:
                if variant == "diag" and j < st:
                    return None          # chain from 0, overwritten by -inf in phase Y
                if variant == "diag" and j == st:
                    return tri
                return V_M[j]
            if variant == "dead":
                return V_NT
            if variant == "diag":
                return V_TRI if j == st else (None if j > st else V_NT)
            return None
        refits = []
        # ---------------- phase X
        mx = []
        fold_dead = OPT_FOLD and variant == "dead"
        if not last and not fold_dead:
            for i in range(NX):
                st, ks, j = i // (2 * KS), (i % (2 * KS)) // 2, i % 2
                f = st * KS + ks
                sreg = (SA if j == 0 else SB(p ^ 1)) + 16 * st
                mx.append(self.mfma_s(sreg, f % 8, j, ks, ks == 0, bias=bias(j, st)))
        fx = []
        if OPT_FOLD and variant == "diag":
            i_b = 2 * KS + 1              # first MFMA of q-block b's triangle chain (st 1, ks 0)
            for j, (eg, dl) in enumerate(((None, 0), (1, i_b))):
                for g in range(16):
                    fx.append(Inst(f"v_add_f32_e32 v{tri + g}, v{V_NEGMC[j]}, v{V_TRI + g}", VALU,
                                   rd=vr(V_NEGMC[j]) + vr(V_TRI + g), wr=vr(tri + g), key=-300 + 20 * j + g,
                                   earliest=eg, deadline=dl))
        if fold_dead:
            # the whole tile n+1 lies above this wave's diagonal: S(n+1) = -inf, no QK
            for base in (SA, SB(p ^ 1)):
                for e in range(32):
                    fx.append(Inst(f"v_mov_b32_e32 v{base + e}, v{V_NINF}", VALU, rd=vr(V_NINF), wr=vr(base + e),
                                   key=50 + e))
        # V base of tile n (slot offset S_VOFF, already advanced at the end of the previous step)
        fx.append(Inst(f"v_add_u32_e32 v{V_VB0}, s{S_VOFF}, v{V_TB0}", VALU, rd=sr(S_VOFF) + vr(V_TB0), wr=vr(V_VB0), key=0))
        fx.append(Inst(f"v_add_u32_e32 v{V_VB1}, s{S_VOFF}, v{V_TB1}", VALU, rd=sr(S_VOFF) + vr(V_TB1), wr=vr(V_VB1), key=0))
        vb = fx[-2:]
        if not last:
            # K fragments 3..15 (0..2 were prefetched at the end of the previous step)
            for f in range(3, 2 * KS) if not fold_dead else ():
                eg = max(2 * (f - 3), 2 * (f - 8) + 3)
                fx.append(self.kread(f, f % 8, key=-100 + f, earliest=eg, deadline=2 * f - 1))
            # K DMA of tile n+4 (4 pieces)
            for jj in range(NP):
                m = Inst(f"s_add_u32 m0, s{S_DOFF}, {jj * 4096}", SALU, rd=sr(S_DOFF), wr=[("m0", 0)], key=-60 + 4 * jj,
                         earliest=3 + 7 * jj)
                d = Inst(f"buffer_load_dwordx4 v{V_VOFF + jj}, s[{S_KD}:{S_KD + 3}], 0 offen lds", DMA,
                         rd=vr(V_VOFF + jj) + sr(S_KD, 4) + [("m0", 0)], key=-60 + 4 * jj, earliest=3 + 7 * jj)
                fx += [m, d]
        # softmax (n, b)
        sm_b, sum_b = self.softmax_ops(1, SB(p), PB, masked, (S_N0, 0), key0=0)
        fx += sm_b
        if OPT_GUARD2:
            fx.append(self.guard_cmp(1, key=1))
        # V fragments of d-tiles 0 and 1 (8 frags) for phase Y
        for f in range(8):
            for h in range(2):
                fx.append(self.vread(f, f % 8, h, key=-80 + 2 * f + h, earliest=max(0, NX - 18 + 2 * f) if not last else None))
        xs = schedule(mx, fx, budget=(OPT_BUDGET64 if D == 64 else OPT_BUDGET), lat=OPT_LAT) if mx else schedule([], fx)
        # ---------------- phase Y
        my = []
        for i in range(NY):
            dt, w = i // 8, i % 8
            j, kk = w // 4, w % 4
            f = 4 * dt + kk
            preg = (PA(p) if j == 0 else PB) + 4 * kk
            my.append(self.mfma_o(j, dt, f % 8, preg))
        fy = []
        rl_b = self.lab(f"{tag}_refit_b")
        # (fold) a refit of q-block b moves its -c m: S(n+1, b), made in phase X from the old
        # chain start, moves with it
        refits.append(self.refit(1, SB(p), PB, rl_b, tile_add=0, phase="Y",
                                 nxt=SB(p ^ 1) if (OPT_FOLD and not last) else None))
        if OPT_GUARD2:
            fy += self.guard_br(1, rl_b, key=-200, deadline=4)
        else:
            fy += self.guard_ops(1, rl_b, key=-200, deadline=4)
        # V fragments of d-tiles 2, 3
        for f in range(8, 4 * NP):
            dt, kk = f // 4, f % 4
            eg = 8 * (dt - 2) + 4 + kk + 1
            dl = 8 * dt + kk - 2
            for h in range(2):
                fy.append(self.vread(f, f % 8, h, key=-150 + 2 * f + h, earliest=eg, deadline=dl))
        t = S_TMP
        if OPT_FOLD and variant == "diag":
            # q-block a's key subtile 1 lies above this wave's diagonal: -inf (its chain ran from 0)
            for e in range(16, 32):
                fy.append(Inst(f"v_mov_b32_e32 v{SA + e}, v{V_NINF}", VALU, rd=vr(V_NINF), wr=vr(SA + e), key=-10))
        if not last:
            # softmax (n+1, a)
            sm_a, sum_a = self.softmax_ops(0, SA, PA(p ^ 1), masked, (S_N0, 64), key0=0)
            fy += sm_a
            # V DMA of tile n+4, then advance the DMA offsets / slot / record counts
            for jj in range(NP):
                fy.append(Inst(f"s_add_u32 m0, s{S_DOFF}, {VBASE + jj * 4096}", SALU, rd=sr(S_DOFF), wr=[("m0", 0)],
                               key=-60 + 4 * jj, earliest=2 + 6 * jj))
                fy.append(Inst(f"buffer_load_dwordx4 v{V_VOFF + jj}, s[{S_VD}:{S_VD + 3}], 0 offen lds", DMA,
                               rd=vr(V_VOFF + jj) + sr(S_VD, 4) + [("m0", 0)], key=-60 + 4 * jj, earliest=2 + 6 * jj))
                fy.append(Inst(f"v_add_u32_e32 v{V_VOFF + jj}, s{S_TB}, v{V_VOFF + jj}", VALU,
                               rd=sr(S_TB) + vr(V_VOFF + jj), wr=vr(V_VOFF + jj), key=-58 + 4 * jj))
            # next DMA slot / tile, zero the record counts once the tile index passes the end
            fy += [
                Inst(f"s_add_u32 s{S_DOFF}, s{S_DOFF}, {TILE}", SALU, rd=sr(S_DOFF), wr=sr(S_DOFF) + [("scc", 0)], key=-30),
                Inst(f"s_sub_u32 s{t}, s{S_DOFF}, {NSLOT * TILE}", SALU, rd=sr(S_DOFF), wr=sr(t) + [("scc", 0)], key=-30),
                Inst(f"s_cmp_ge_u32 s{S_DOFF}, {NSLOT * TILE}", SALU, rd=sr(S_DOFF), wr=[("scc", 0)], key=-30),
                Inst(f"s_cselect_b32 s{S_DOFF}, s{t}, s{S_DOFF}", SALU, rd=sr(t) + sr(S_DOFF) + [("scc", 0)], wr=sr(S_DOFF), key=-30),
            ]
            # the DMA stream passed the end of its item: switch to the next item (out of line, once)
            fy += self.dma_count_ops(self.lab(f"{tag}_sw"), key=-30)
            # K read base of tile n+2 and prefetch of its first three fragments (next phase X)
            fy += [
                Inst(f"s_add_u32 s{S_KOFF}, s{S_KOFF}, {TILE}", SALU, rd=sr(S_KOFF), wr=sr(S_KOFF) + [("scc", 0)], key=-20, earliest=NY - 14),
                Inst(f"s_sub_u32 s{t + 1}, s{S_KOFF}, {NSLOT * TILE}", SALU, rd=sr(S_KOFF), wr=sr(t + 1) + [("scc", 0)], key=-20),
                Inst(f"s_cmp_ge_u32 s{S_KOFF}, {NSLOT * TILE}", SALU, rd=sr(S_KOFF), wr=[("scc", 0)], key=-20),
                Inst(f"s_cselect_b32 s{S_KOFF}, s{t + 1}, s{S_KOFF}", SALU, rd=sr(t + 1) + sr(S_KOFF) + [("scc", 0)], wr=sr(S_KOFF), key=-20),
                Inst(f"v_add_u32_e32 v{V_KB0}, s{S_KOFF}, v{V_RB0}", VALU, rd=sr(S_KOFF) + vr(V_RB0), wr=vr(V_KB0), key=-20),
                Inst(f"v_add_u32_e32 v{V_KB1}, s{S_KOFF}, v{V_RB1}", VALU, rd=sr(S_KOFF) + vr(V_RB1), wr=vr(V_KB1), key=-20),
            ]
            for f in range(3):
                fy.append(self.kread(f, f % 8, key=-19 + f, earliest=NY - 10 + 2 * f))
            rl_a = self.lab(f"{tag}_refit_a")
            refits.append(self.refit(0, SA, PA(p ^ 1), rl_a, tile_add=64, phase="end"))
            # after the phase's LAST MFMA: refit_a borrows the V fragment ring as scratch and rescales
            # O_a, so no PV MFMA may still be pending (placed earlier, it corrupted the d-tile 3 MFMAs)
            if OPT_GUARD2:
                fy += [self.guard_cmp(0, key=700)] + self.guard_br(0, rl_a, key=700, eg=NY - 1)
            else:
                ga = self.guard_ops(0, rl_a, key=700)
                for op in ga:
                    op.eg = NY - 1
                fy += ga
        if last:
            # Q of the next item (persistent loop): the Q registers are idle from here on (no QK MFMA
            # in the last step; the refit of q-block b, which reads them, returns before MFMA 4)
            for j in range(2):
                for ks in range(KS):
                    fy.append(Inst(f"buffer_load_dwordx4 {rtxt('a', Q_(j, ks), 4)}, v{V_QOFF[j]}, s[{S_QD2}:{S_QD2 + 3}], 0 offen offset:{32 * ks}",
                                   VLOAD, rd=vr(V_QOFF[j]) + sr(S_QD2, 4), wr=ar(Q_(j, ks), 4), key=900 + 8 * j + ks, earliest=8))
        # V read slot of the next tile
        fy += [Inst(f"s_add_u32 s{S_VOFF}, s{S_VOFF}, {TILE}", SALU, rd=sr(S_VOFF), wr=sr(S_VOFF) + [("scc", 0)], key=800, earliest=NY - 4),
               Inst(f"s_sub_u32 s{t + 2}, s{S_VOFF}, {NSLOT * TILE}", SALU, rd=sr(S_VOFF), wr=sr(t + 2) + [("scc", 0)], key=801),
               Inst(f"s_cmp_ge_u32 s{S_VOFF}, {VBASE + NSLOT * TILE}", SALU, rd=sr(S_VOFF), wr=[("scc", 0)], key=802),
               Inst(f"s_cselect_b32 s{S_VOFF}, s{t + 2}, s{S_VOFF}", SALU, rd=sr(t + 2) + sr(S_VOFF) + [("scc", 0)], wr=sr(S_VOFF), key=803)]
        ys = schedule(my, fy, budget=(OPT_BUDGET64 if D == 64 else OPT_BUDGET), lat=OPT_LAT)
        body = xs + ys
        if not last and OPT_STEPSTAMP and OPT_STAMP_NONFAST and variant == "fast":
            # (FA_GEN_STAMP_ONLY=nonfast: the fast steps only move the last stamp, so the sums and the
            # count are those of the masked / diagonal / dead steps alone)
            A, t0 = S_TMP, V_T
            body += [Inst(f"s_add_u32 s{S_N}, s{S_N}, 1", SALU, rd=sr(S_N), wr=sr(S_N) + [("scc", 0)]),
                     Inst(f"s_add_u32 s{S_N0}, s{S_N0}, {BN}", SALU, rd=sr(S_N0), wr=sr(S_N0) + [("scc", 0)]),
                     Inst(f"s_waitcnt vmcnt({2 * NP}) lgkmcnt(0)", WAIT),
                     Inst("s_barrier", BARRIER),
                     Inst(f"s_memtime s[{A}:{A + 1}]", SMEM),
                     Inst("s_waitcnt lgkmcnt(0)", WAIT),
                     Inst(f"v_mov_b32_e32 v{V_SSUM + 4}, s{A}", VALU)]
        elif not last and OPT_STEPSTAMP:
            A, B, t0 = S_TMP, S_TMP + 2, V_T
            body += [Inst(f"s_add_u32 s{S_N}, s{S_N}, 1", SALU, rd=sr(S_N), wr=sr(S_N) + [("scc", 0)]),
                     Inst(f"s_add_u32 s{S_N0}, s{S_N0}, {BN}", SALU, rd=sr(S_N0), wr=sr(S_N0) + [("scc", 0)]),
                     Inst(f"s_memtime s[{A}:{A + 1}]", SMEM),
                     Inst(f"s_waitcnt vmcnt({2 * NP}) lgkmcnt(0)", WAIT),
                     Inst(f"s_memtime s[{B}:{B + 1}]", SMEM),
                     Inst(f"v_mov_b32_e32 v{t0}, s{A}", VALU),
                     Inst("s_waitcnt lgkmcnt(0)", WAIT),
                     Inst(f"v_mov_b32_e32 v{t0 + 1}, s{B}", VALU),
                     Inst("s_barrier", BARRIER),
                     Inst(f"s_memtime s[{A}:{A + 1}]", SMEM),
                     Inst("s_waitcnt lgkmcnt(0)", WAIT),
                     Inst(f"v_mov_b32_e32 v{t0 + 2}, s{A}", VALU),
                     Inst(f"v_sub_u32_e32 v{t0 + 3}, v{t0}, v{V_SSUM + 4}", VALU),
                     Inst(f"v_add_u32_e32 v{V_SSUM}, v{V_SSUM}, v{t0 + 3}", VALU),
                     Inst(f"v_sub_u32_e32 v{t0 + 3}, v{t0 + 1}, v{t0}", VALU),
                     Inst(f"v_add_u32_e32 v{V_SSUM + 1}, v{V_SSUM + 1}, v{t0 + 3}", VALU),
                     Inst(f"v_sub_u32_e32 v{t0 + 3}, v{t0 + 2}, v{t0 + 1}", VALU),
                     Inst(f"v_add_u32_e32 v{V_SSUM + 2}, v{V_SSUM + 2}, v{t0 + 3}", VALU),
                     Inst(f"v_add_u32_e32 v{V_SSUM + 3}, 1, v{V_SSUM + 3}", VALU),
                     Inst(f"v_mov_b32_e32 v{V_SSUM + 4}, v{t0 + 2}", VALU)]
        elif not last:
            # tiles <= n+3 landed in every wave (K(n+3) is prefetched in the next step's phase Y)
            body += [Inst(f"s_add_u32 s{S_N}, s{S_N}, 1", SALU, rd=sr(S_N), wr=sr(S_N) + [("scc", 0)]),
                     Inst(f"s_add_u32 s{S_N0}, s{S_N0}, {BN}", SALU, rd=sr(S_N0), wr=sr(S_N0) + [("scc", 0)]),
                     Inst(f"s_waitcnt vmcnt({2 * NP}) lgkmcnt(0)", WAIT),
                     Inst("s_barrier", BARRIER)]
        return body, refits

    # ------------------------------------------------------------------ DMA stream across items
    def dma_count_ops(self, lab, key=0):
        """after one tile's K and V pieces are issued: count it; when the stream reaches the end of
        its item, branch to the (out-of-line) switch block.  The branch is one instruction with its
        return label, and it carries the registers the block touches so that the scheduler keeps
        every V_VOFF update / DMA of this tile before it."""
        self.switches.append(self.switch_block(lab))
        touched = vr(V_VOFF, NP) + sr(S_KD, 4) + sr(S_VD, 4) + sr(S_DT) + sr(S_DLIM) + sr(S_WARM)
        return [Inst(f"s_add_u32 s{S_DT}, s{S_DT}, 1", SALU, rd=sr(S_DT), wr=sr(S_DT) + [("scc", 0)], key=key),
                Inst(f"s_cmp_eq_u32 s{S_DT}, s{S_DLIM}", SALU, rd=sr(S_DT) + sr(S_DLIM), wr=[("scc", 0)], key=key),
                Inst(f"s_cbranch_scc1 {lab}\n{lab}_back:", BRANCH, rd=[("scc", 0)] + touched, wr=touched, key=key)]

    def switch_block(self, lab):
        """The DMA stream issued the last tile of its item.  If the next item has >= 4 tiles, the
        following DMAs read it: K/V descriptors <- the next item's, per-lane offsets back to tile 0,
        S_DT = 0, S_DLIM = its tile count, S_WARM = 1 (its tiles 0..2 get issued before the current
        item ends, so it starts warm).  Otherwise the records are zeroed (the DMAs past the end
        zero-fill their slots) and the next item starts cold."""
        I = Inst
        lz = lab + "_z"
        ins = [label(lab),
               I(f"s_cmp_lt_u32 s{S_NXN}, 4", SALU), I(f"s_cbranch_scc1 {lz}", BRANCH)]
        ins += [I(f"s_mov_b32 s{S_KD + i}, s{S_KD2 + i}", SALU) for i in range(4)]
        ins += [I(f"s_mov_b32 s{S_VD + i}, s{S_VD2 + i}", SALU) for i in range(4)]
        ins += [I(f"s_mul_i32 s{S_SWT}, s{S_DT}, s{S_TB}", SALU)]
        ins += [I(f"v_subrev_u32_e32 v{V_VOFF + jj}, s{S_SWT}, v{V_VOFF + jj}", VALU) for jj in range(NP)]
        ins += [I(f"s_mov_b32 s{S_DT}, 0", SALU), I(f"s_mov_b32 s{S_DLIM}, s{S_NXN}", SALU),
                I(f"s_mov_b32 s{S_WARM}, 1", SALU), nop(4), I(f"s_branch {lab}_back", BRANCH),
                label(lz),
                I(f"s_mov_b32 s{S_KD + 2}, 0", SALU), I(f"s_mov_b32 s{S_VD + 2}, 0", SALU), nop(4),
                I(f"s_branch {lab}_back", BRANCH)]
        return ins

    def dma_tile_ops(self, tag):
        """one whole tile (K then V pieces) into the slot at S_DOFF, then the stream bookkeeping
        (prologue use: not scheduled)"""
        I = Inst
        ins = []
        for jj in range(NP):
            ins += [I(f"s_add_u32 m0, s{S_DOFF}, {jj * 4096}", SALU, rd=sr(S_DOFF), wr=[("m0", 0)]),
                    I(f"buffer_load_dwordx4 v{V_VOFF + jj}, s[{S_KD}:{S_KD + 3}], 0 offen lds", DMA,
                      rd=vr(V_VOFF + jj) + sr(S_KD, 4) + [("m0", 0)])]
        for jj in range(NP):
            ins += [I(f"s_add_u32 m0, s{S_DOFF}, {VBASE + jj * 4096}", SALU, rd=sr(S_DOFF), wr=[("m0", 0)]),
                    I(f"buffer_load_dwordx4 v{V_VOFF + jj}, s[{S_VD}:{S_VD + 3}], 0 offen lds", DMA,
                      rd=vr(V_VOFF + jj) + sr(S_VD, 4) + [("m0", 0)])]
        for jj in range(NP):
            ins.append(I(f"v_add_u32_e32 v{V_VOFF + jj}, s{S_TB}, v{V_VOFF + jj}", VALU, rd=sr(S_TB) + vr(V_VOFF + jj), wr=vr(V_VOFF + jj)))
        ins += [I(f"s_add_u32 s{S_DOFF}, s{S_DOFF}, {TILE}", SALU, rd=sr(S_DOFF), wr=sr(S_DOFF)),
                I(f"s_sub_u32 s{S_SWT}, s{S_DOFF}, {NSLOT * TILE}", SALU, rd=sr(S_DOFF), wr=sr(S_SWT)),
                I(f"s_cmp_ge_u32 s{S_DOFF}, {NSLOT * TILE}", SALU, rd=sr(S_DOFF), wr=[("scc", 0)]),
                I(f"s_cselect_b32 s{S_DOFF}, s{S_SWT}, s{S_DOFF}", SALU, rd=sr(S_SWT) + sr(S_DOFF), wr=sr(S_DOFF))]
        ins += self.dma_count_ops(self.lab(f"{tag}_sw"))
        return ins

    # ------------------------------------------------------------------ refit (rare, out of line)
    def refit(self, j, sreg, preg, lab, tile_add, phase, nxt=None):
        """Out-of-line slow path (rare): recompute S of q-block j for its tile from the K slot that
        still holds it, mask it, take the true row max, rescale O_j / l_j to it and redo P and the
        partial sum.  phase 'Y' (tile n, checked before its first PV MFMA): S_KOFF still addresses
        tile n+1; phase 'end' (tile n+1, checked at the end of phase Y): S_KOFF was advanced to tile
        n+2.  Either way the tile's K slot is S_KOFF - TILE (mod the ring).  With the fold the
        recomputed scores are c S (chain from 0; Q holds c Q), the new -c m also goes into the
        chain-start tile V_M[j], and nxt (the q-block's next S tile, already computed from the old
        chain start) is moved by the change of -c m."""
        ins = [label(lab), nop(15), Inst("s_waitcnt lgkmcnt(0)", WAIT)]
        t = V_T
        s0 = S_TMP + 3
        ins += [Inst(f"s_sub_u32 s{s0}, s{S_KOFF}, {TILE}", SALU, rd=sr(S_KOFF), wr=sr(s0)),
                Inst(f"s_add_u32 s{S_TMP}, s{s0}, {NSLOT * TILE}", SALU, rd=sr(s0), wr=sr(S_TMP)),
                Inst(f"s_cmp_lt_i32 s{s0}, 0", SALU, rd=sr(s0), wr=[("scc", 0)]),
                Inst(f"s_cselect_b32 s{s0}, s{S_TMP}, s{s0}", SALU, rd=sr(S_TMP) + sr(s0), wr=sr(s0)),
                Inst(f"v_add_u32_e32 v{t}, s{s0}, v{V_RB0}", VALU, rd=sr(s0) + vr(V_RB0), wr=vr(t)),
                Inst(f"v_add_u32_e32 v{t + 1}, s{s0}, v{V_RB1}", VALU, rd=sr(s0) + vr(V_RB1), wr=vr(t + 1))]
        # K fragment ring to use: phase Y -> the K ring (idle), end -> the V ring (the K ring holds
        # the next phase X's prefetch)
        ring = KF if phase == "Y" else VF
        for st in range(2):
            for ks in range(KS):
                base = t if ks % 2 == 0 else t + 1
                off = (ks // 2) * BN * 64 + st * 32 * 64
                ins.append(Inst(f"ds_read_b128 {rtxt('a', ring + 4 * ks, 4)}, v{base} offset:{off}", LDS,
                                rd=vr(base), wr=ar(ring + 4 * ks, 4)))
            for ks in range(KS):
                sreg_st = sreg + 16 * st
                c = "0" if ks == 0 else rtxt("v", sreg_st, 16)
                ins.append(Inst(f"v_mfma_f32_32x32x16_{self.ty} {rtxt('v', sreg_st, 16)}, {rtxt('a', ring + 4 * ks, 4)}, "
                                f"{rtxt('a', Q_(j, ks), 4)}, {c}", MFMA,
                                rd=ar(ring + 4 * ks, 4) + ar(Q_(j, ks), 4) + ([] if ks == 0 else vr(sreg_st, 16)),
                                wr=vr(sreg_st, 16), rd_c=[] if ks == 0 else vr(sreg_st, 16)))
        ins.append(nop(15))
        # mask with the tile's limits (own limit registers: the interrupted stream may hold V_LM)
        ins += self.mask_ops(j, sreg, (S_N0, tile_add), (t + 5, t + 6))
        # row max -> v[t+2]
        mx = t + 2
        ins.append(Inst(f"v_max3_f32 v{mx}, v{sreg}, v{sreg + 1}, v{sreg + 2}", VALU, rd=vr(sreg, 3), wr=vr(mx)))
        for e in range(3, 32, 2):
            if e + 1 < 32:
                ins.append(Inst(f"v_max3_f32 v{mx}, v{mx}, v{sreg + e}, v{sreg + e + 1}", VALU, rd=vr(mx) + vr(sreg + e, 2), wr=vr(mx)))
            else:
                ins.append(Inst(f"v_max_f32_e32 v{mx}, v{mx}, v{sreg + e}", VALU, rd=vr(mx) + vr(sreg + e), wr=vr(mx)))
        ins += self.half_max(mx, t + 3)
        # mnc = max(mc_old, mt * c); alpha = exp2(mc_old - mnc)   (fold: the scores are c S already)
        if not OPT_FOLD:
            ins += [Inst(f"v_mul_f32_e32 v{mx}, s{S_C}, v{mx}", VALU, rd=sr(S_C) + vr(mx), wr=vr(mx))]
        ins += [Inst(f"v_max_f32_e64 v{mx}, -v{V_NEGMC[j]}, v{mx}", VALU, rd=vr(V_NEGMC[j]) + vr(mx), wr=vr(mx)),
                Inst(f"v_add_f32_e32 v{t + 3}, v{V_NEGMC[j]}, v{mx}", VALU, rd=vr(V_NEGMC[j]) + vr(mx), wr=vr(t + 3))]
        if nxt is not None:
            # next tile: c S + (-c m_old) -> c S + (-c m_new) = score - (mc_new - mc_old)
            ins += [Inst(f"v_sub_f32_e32 v{nxt + e}, v{nxt + e}, v{t + 3}", VALU, rd=vr(nxt + e) + vr(t + 3),
                         wr=vr(nxt + e)) for e in range(32)]
        ins += [Inst(f"v_exp_f32_e64 v{t + 3}, -v{t + 3}", TRANS, rd=vr(t + 3), wr=vr(t + 3)),
                Inst(f"v_sub_f32_e32 v{V_NEGMC[j]}, 0, v{mx}", VALU, rd=vr(mx), wr=vr(V_NEGMC[j])),
                Inst(f"v_mul_f32_e32 v{V_L[j]}, v{V_L[j]}, v{t + 3}", VALU, rd=vr(V_L[j]) + vr(t + 3), wr=vr(V_L[j]))]
        if OPT_FOLD:
            ins += self.m_tile_ops(j)
        for dt in range(NP):
            for g in range(16):
                a = O_(j, dt) + g
                ins += [Inst(f"v_accvgpr_read_b32 v{t + 4}, a{a}", ACCR, rd=ar(a), wr=vr(t + 4)),
                        Inst(f"v_mul_f32_e32 v{t + 4}, v{t + 4}, v{t + 3}", VALU, rd=vr(t + 4, 1) + vr(t + 3), wr=vr(t + 4)),
                        Inst(f"v_accvgpr_write_b32 a{a}, v{t + 4}", ACCW, rd=vr(t + 4), wr=ar(a))]
        sm, _ = self.softmax_ops(j, sreg, preg, False, None, key0=0, fold_add=OPT_FOLD)
        ins += sm
        ins.append(nop(7))
        ins.append(Inst(f"s_branch {lab}_back", BRANCH))
        out, _ = add_waits(ins)
        out, _ = fix_hazards(out)
        self.refit_regs[lab] = set().union(*(i.wr for i in out))
        return out

    def m_tile_ops(self, j, key=0):
        """(fold) the chain-start tile of q-block j: 16 copies of its -c m"""
        return [Inst(f"v_mov_b32_e32 v{V_M[j] + g}, v{V_NEGMC[j]}", VALU, rd=vr(V_NEGMC[j]), wr=vr(V_M[j] + g), key=key)
                for g in range(16)]

    def q_scale_ops(self, j, X, LO, key=0, deadline=None):
        """(fold) q-block j's Q fragments (AGPRs, as loaded) -> bf16/f16(c Q), round to nearest even,
        through v[X..X+4KS) and v[LO..LO+4KS): lo half into LO, hi half in place, the pack into LO"""
        I = Inst
        n = 4 * KS
        q0 = Q_(j, 0)
        kw = dict(key=key, deadline=deadline)
        ops = [I(f"v_accvgpr_read_b32 v{X + i}, a{q0 + i}", ACCR, rd=ar(q0 + i), wr=vr(X + i), **kw) for i in range(n)]
        if self.bf16:
            ops += [I(f"v_lshlrev_b32_e32 v{LO + i}, 16, v{X + i}", VALU, rd=vr(X + i), wr=vr(LO + i), **kw) for i in range(n)]
            ops += [I(f"v_and_b32_e32 v{X + i}, 0xffff0000, v{X + i}", VALU, rd=vr(X + i), wr=vr(X + i), **kw) for i in range(n)]
        else:
            ops += [I(f"v_cvt_f32_f16_e32 v{LO + i}, v{X + i}", VALU, rd=vr(X + i), wr=vr(LO + i), **kw) for i in range(n)]
            ops += [I(f"v_lshrrev_b32_e32 v{X + i}, 16, v{X + i}", VALU, rd=vr(X + i), wr=vr(X + i), **kw) for i in range(n)]
            ops += [I(f"v_cvt_f32_f16_e32 v{X + i}, v{X + i}", VALU, rd=vr(X + i), wr=vr(X + i), **kw) for i in range(n)]
        for R in (LO, X):
            ops += [I(f"v_mul_f32_e32 v{R + i}, s{S_C}, v{R + i}", VALU, rd=sr(S_C) + vr(R + i), wr=vr(R + i), **kw)
                    for i in range(n)]
        ops += [self.cvt(LO + i, LO + i, X + i, **kw) for i in range(n)]
        ops += [I(f"v_accvgpr_write_b32 a{q0 + i}, v{LO + i}", ACCW, rd=vr(LO + i), wr=ar(q0 + i), **kw) for i in range(n)]
        return ops

    def tile0_fold(self, l_entry_last, l_entry_fast, l_entry_masked):
        """(fold) tile 0 with the Q conversion overlapped: q-block a's Q is converted first, then
        S(0, a) runs its MFMAs while q-block b's Q is converted in their gaps, and S(0, b) runs while
        a's mask, row max, -c m and P(0, a) fill its gaps (at d = 128 the K fragments are read again
        for b: the 8-slot ring does not hold all 16).  S(0, b) then gets its own max, its -c m added
        (the first step's softmax takes scores from a V_M-started chain) and both V_M tiles are set."""
        I = Inst
        if OPT_T0STAMP:
            ins = (self.stamp_point(9) + [I(f"s_waitcnt vmcnt({2 * NP})", WAIT)] + self.stamp_point(6) +
                   [I("s_barrier", BARRIER)] + self.stamp_point(5))
        else:
            ins = [I(f"s_waitcnt vmcnt({2 * NP})", WAIT), I("s_barrier", BARRIER)]
            ins += [] if OPT_EPISTAMP else self.stamp_point(9)
        ins += self.dump("pro_lds")
        ins += self.q_scale_ops(0, 0, 32)
        ins += [I(f"v_add_u32_e32 v{V_KB0}, s{S_KOFF}, v{V_RB0}", VALU, rd=sr(S_KOFF) + vr(V_RB0), wr=vr(V_KB0)),
                I(f"v_add_u32_e32 v{V_KB1}, s{S_KOFF}, v{V_RB1}", VALU, rd=sr(S_KOFF) + vr(V_RB1), wr=vr(V_KB1))]
        n2 = 2 * KS
        mfm = []
        for j in range(2):
            for f in range(n2):
                st, ks = f // KS, f % KS
                mfm.append(self.mfma_s((SA if j == 0 else SB(0)) + 16 * st, f % 8, j, ks, ks == 0))
        fill = []
        for f in range(n2):
            fill.append(self.kread(f, f % 8, key=-100 + f, earliest=(f - 8) if f >= 8 else None, deadline=max(f - 2, 0)))
        if n2 > 8:
            for f in range(n2):
                fill.append(self.kread(f, f % 8, key=-60 + f, earliest=f + 8, deadline=n2 + f - 2))
        # q-block b's Q (temporaries: S(b) buffer 1 and the P(a) packs, idle in tile 0)
        fill += self.q_scale_ops(1, SB(1), PA(0), key=0, deadline=n2)
        if OPT_T0ZERO:
            fill += self.o_zero_ops(key=100)
        tail = self.tile0_maxops(0, SA, key=400)
        tail += self.softmax_ops(0, SA, PA(0), False, None, key0=600, fold_add=True)[0]
        tail += [Inst(f"v_mov_b32_e32 v{V_L[0]}, v{V_PS[0]}", VALU, rd=vr(V_PS[0]), wr=vr(V_L[0]), key=900)]
        for op in tail:
            op.eg = n2 - 1     # after S(0, a)'s last MFMA
        fill += tail
        ins += schedule(mfm, fill) + [nop(15)]
        ins += self.dump("pro_qk")
        ins += self.tile0_maxops(1, SB(0), key=0)
        ins += [Inst(f"v_add_f32_e32 v{SB(0) + e}, v{V_NEGMC[1]}, v{SB(0) + e}", VALU,
                     rd=vr(V_NEGMC[1]) + vr(SB(0) + e), wr=vr(SB(0) + e)) for e in range(32)]
        ins += self.m_tile_ops(0) + self.m_tile_ops(1)
        ins += self.dump("pro_end")
        ins += [] if (OPT_EPISTAMP or OPT_T0STAMP) else self.stamp_point(6)
        ins += self.tile0_exit(l_entry_last, l_entry_fast, l_entry_masked)
        return ins

    def dump(self, point):
        """register / LDS dump of workgroup 0 at `point` (OPT_DUMP), then s_endpgm"""
        if OPT_DUMP != point:
            return []
        I = Inst
        D, SO, SW = 96, 90, 91
        ins = [Inst("s_waitcnt vmcnt(0) lgkmcnt(0)", WAIT), nop(15), nop(15),
               # the seed kernarg SGPRs are S_QD2 by now: reload the dump address from the kernarg segment
               I(f"s_load_dwordx2 s[{D}:{D + 1}], s[0:1], 0x48", SMEM), Inst("s_waitcnt lgkmcnt(0)", WAIT),
               I(f"s_and_b32 s{D + 1}, s{D + 1}, 0xffff", SALU),
               I(f"s_cmp_eq_u32 s2, 0", SALU), I(f"s_cselect_b32 s{D + 2}, 0x7fffffff, 0", SALU),
               I(f"s_mov_b32 s{D + 3}, 0x20000", SALU),
               I(f"s_mul_i32 s{SW}, s{S_WAVE}, {DUMP_SLOTS * 256}", SALU),
               I(f"v_lshlrev_b32_e32 v255, 2, v{V_LANE}", VALU), nop(4)]
        # SGPRs first (their copies go through v254)
        for i in range(128):
            if i >= NSGPR and i not in (D, D + 1, D + 2, D + 3):
                continue
            src = f"s{i}" if i < 102 else None
            if src is None:
                continue
            ins += [I(f"v_mov_b32_e32 v254, {src}", VALU), I(f"s_add_u32 s{SO}, s{SW}, {(512 + i) * 256}", SALU), nop(1),
                    I(f"buffer_store_dword v254, v255, s[{D}:{D + 3}], s{SO} offen", VSTORE), nop(1)]
        for i in range(254):
            ins += [I(f"s_add_u32 s{SO}, s{SW}, {i * 256}", SALU), nop(1),
                    I(f"buffer_store_dword v{i}, v255, s[{D}:{D + 3}], s{SO} offen", VSTORE)]
        for i in range(256):
            ins += [I(f"v_accvgpr_read_b32 v254, a{i}", ACCR), I(f"s_add_u32 s{SO}, s{SW}, {(256 + i) * 256}", SALU), nop(1),
                    I(f"buffer_store_dword v254, v255, s[{D}:{D + 3}], s{SO} offen", VSTORE), nop(1)]
        # LDS (wave 0): 160 KiB after the 4 waves' register slots
        l_skip = self.lab("dumpskip")
        ins += [I(f"s_cmp_lg_u32 s{S_WAVE}, 0", SALU), I(f"s_cbranch_scc1 {l_skip}", BRANCH),
                I("v_lshlrev_b32_e32 v253, 4, v{0}".format(V_LANE), VALU), nop(4)]
        for blk in range(LDS_BYTES // 1024):
            if blk % 64 == 0 and blk:
                ins += [I("v_add_u32_e32 v253, 0x10000, v253", VALU), nop(4)]
            ins += [I(f"ds_read_b128 v[0:3], v253 offset:{(blk % 64) * 1024}", LDS), Inst("s_waitcnt lgkmcnt(0)", WAIT),
                    I(f"s_mov_b32 s{SO}, {4 * DUMP_SLOTS * 256 + blk * 1024}", SALU),
                    I(f"v_lshlrev_b32_e32 v252, 4, v{V_LANE}", VALU), nop(1),
                    I(f"buffer_store_dwordx4 v[0:3], v252, s[{D}:{D + 3}], s{SO} offen", VSTORE), nop(2)]
        ins += [label(l_skip), Inst("s_waitcnt vmcnt(0)", WAIT), I("s_endpgm", SOPP)]
        return ins

    def half_max(self, x, tmp):
        """x = max over the two lane halves (lanes l, l^32 hold the same query)"""
        return [Inst(f"v_mov_b32_e32 v{tmp}, v{x}", VALU, rd=vr(x), wr=vr(tmp)),
                Inst(f"v_permlane32_swap_b32_e32 v{x}, v{tmp}", PERM, rd=vr(x) + vr(tmp), wr=vr(x) + vr(tmp)),
                Inst(f"v_max_f32_e32 v{x}, v{x}, v{tmp}", VALU, rd=vr(x) + vr(tmp), wr=vr(x))]

    def half_sum(self, x, tmp):
        return [Inst(f"v_mov_b32_e32 v{tmp}, v{x}", VALU, rd=vr(x), wr=vr(tmp)),
                Inst(f"v_permlane32_swap_b32_e32 v{x}, v{tmp}", PERM, rd=vr(x) + vr(tmp), wr=vr(x) + vr(tmp)),
                Inst(f"v_add_f32_e32 v{x}, v{x}, v{tmp}", VALU, rd=vr(x) + vr(tmp), wr=vr(x))]

    # ------------------------------------------------------------------ prologue (persistent item loop)
    # kernargs: 40..55 pointers (q k v o lse sched cuq cuk); 56..63 rng seed offset q_batch;
    # 64..79 k_batch v_batch o_batch q_row kv_row o_row q_head k_head v_head o_head sq sk lse_pitch;
    # 80..84 h c flags n_items grid
    def kargs(self):
        ka = S_KA
        return dict(Pq=ka, Pk=ka + 2, Pv=ka + 4, Po=ka + 6, Pl=ka + 8, Psch=ka + 10, Pcq=ka + 12, Pck=ka + 14,
                    Prng=ka + 16, Pseed=ka + 18, Poff=ka + 20, Bq=ka + 22, Bk=ka + 24, Bv=ka + 26, Bo=ka + 28,
                    Rq=ka + 30, Rkv=ka + 31, Ro=ka + 32, Hq=ka + 33, Hk=ka + 34, Hv=ka + 35, Ho=ka + 36,
                    SQ=ka + 37, SK=ka + 38, LP=ka + 39, NH=ka + 40, CC=ka + 41, FL=ka + 42)

    def entry(self):
        """once per workgroup: kernargs, lane constants, rng_state; falls into the cold item start"""
        I = Inst
        ins = []
        ka = S_KA
        A = self.kargs()
        ins += [I(f"s_load_dwordx16 s[{ka}:{ka + 15}], s[0:1], 0x0", SMEM, rd=sr(0, 2), wr=sr(ka, 16)),
                I(f"s_load_dwordx8 s[{ka + 16}:{ka + 23}], s[0:1], 0x40", SMEM, rd=sr(0, 2), wr=sr(ka + 16, 8)),
                I(f"s_load_dwordx16 s[{ka + 24}:{ka + 39}], s[0:1], 0x60", SMEM, rd=sr(0, 2), wr=sr(ka + 24, 16)),
                I(f"s_load_dwordx4 s[{ka + 40}:{ka + 43}], s[0:1], 0xa0", SMEM, rd=sr(0, 2), wr=sr(ka + 40, 4)),
                I(f"s_load_dword s{S_GRID}, s[0:1], 0xb0", SMEM, rd=sr(0, 2), wr=sr(S_GRID))]
        if OPT_DECBURST:
            # the first item's work order (fa_params.h ItemDecode) in the same scalar-memory round
            # trip: s[88:97] hold it until that item's geometry (item_geom skips its reload in
            # round 0; later items reload it, the geometry reuses the registers)
            ins += [I(f"s_load_dwordx8 s[88:95], s[0:1], {DEC_OFF}", SMEM, rd=sr(0, 2), wr=sr(88, 8)),
                    I(f"s_load_dwordx2 s[96:97], s[0:1], {DEC_OFF + 32}", SMEM, rd=sr(0, 2), wr=sr(96, 2))]
        ins += [I("s_waitcnt lgkmcnt(0)", WAIT)]
        T0 = S_TMP
        # varlen work list built on the device (flags bit 1): the item count is its first dword and
        # the entries start 8 bytes in
        l_cnt, l_cnt_done = self.lab("cnt"), self.lab("cntdone")
        Psch = A["Psch"]
        ins += [I(f"s_bitcmp1_b32 s{A['FL']}, 1", SALU), I(f"s_cbranch_scc1 {l_cnt}", BRANCH),
                I(f"s_branch {l_cnt_done}", BRANCH), label(l_cnt),
                I(f"s_load_dword s{S_NITEMS}, s[{Psch}:{Psch + 1}], 0x0", SMEM),
                I(f"s_add_u32 s{Psch}, s{Psch}, 8", SALU), I(f"s_addc_u32 s{Psch + 1}, s{Psch + 1}, 0", SALU),
                I("s_waitcnt lgkmcnt(0)", WAIT), label(l_cnt_done)]
        # wave index, lane values
        ins += [I("v_lshrrev_b32_e32 v1, 6, v0", VALU, rd=vr(0), wr=vr(1)),
                I(f"v_readfirstlane_b32 s{S_WAVE}, v1", RFL, rd=vr(1), wr=sr(S_WAVE)),
                I(f"v_and_b32_e32 v{V_LANE}, 63, v0", VALU, rd=vr(0), wr=vr(V_LANE))]
        if OPT_STAMP:
            ins += [I(f"s_memtime s[{T0}:{T0 + 1}]", SMEM, wr=sr(T0, 2)),
                    I(f"s_memrealtime s[{T0 + 2}:{T0 + 3}]", SMEM, wr=sr(T0 + 2, 2)),
                    I("s_waitcnt lgkmcnt(0)", WAIT)]
            ins += [I(f"v_mov_b32_e32 v{V_STAMP + i}, s{T0 + i}", VALU, rd=sr(T0 + i), wr=vr(V_STAMP + i)) for i in range(4)]
            ins += [I(f"v_mov_b32_e32 v{V_STAMP + 4}, 0", VALU, wr=vr(V_STAMP + 4)),
                    I(f"v_mov_b32_e32 v{V_STAMP + 5}, 0", VALU, wr=vr(V_STAMP + 5))]
            ins += [I(f"v_mov_b32_e32 v{V_SSUM + i}, 0", VALU) for i in (0, 1, 2, 3, 5, 6, 7, 8, 9)]
            ins += [I(f"v_mov_b32_e32 v{V_SSUM + 4}, s{T0}", VALU)]
        # rng_state (block 0, wave 0): {seed, offset}; lanes >= 1 fall outside the 16-byte record
        l_norng = self.lab("norng")
        Prng, Pseed, Poff = A["Prng"], A["Pseed"], A["Poff"]
        ins += [I(f"s_or_b32 s{T0}, s2, s{S_WAVE}", SALU, rd=sr(2) + sr(S_WAVE), wr=sr(T0)),
                I(f"s_cmp_lg_u32 s{T0}, 0", SALU, rd=sr(T0), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_norng}", BRANCH),
                I(f"s_cmp_eq_u64 s[{Prng}:{Prng + 1}], 0", SALU, rd=sr(Prng, 2), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_norng}", BRANCH),
                I(f"s_mov_b32 s{S_RNGD}, s{Prng}", SALU, rd=sr(Prng), wr=sr(S_RNGD)),
                I(f"s_and_b32 s{S_RNGD + 1}, s{Prng + 1}, 0xffff", SALU, rd=sr(Prng + 1), wr=sr(S_RNGD + 1)),
                I(f"s_mov_b32 s{S_RNGD + 2}, 16", SALU, wr=sr(S_RNGD + 2)),
                I(f"s_mov_b32 s{S_RNGD + 3}, 0x20000", SALU, wr=sr(S_RNGD + 3)),
                I(f"v_lshlrev_b32_e32 v2, 4, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(2)),
                I(f"v_mov_b32_e32 v4, s{Pseed}", VALU, rd=sr(Pseed), wr=vr(4)),
                I(f"v_mov_b32_e32 v5, s{Pseed + 1}", VALU, rd=sr(Pseed + 1), wr=vr(5)),
                I(f"v_mov_b32_e32 v6, s{Poff}", VALU, rd=sr(Poff), wr=vr(6)),
                I(f"v_mov_b32_e32 v7, s{Poff + 1}", VALU, rd=sr(Poff + 1), wr=vr(7)),
                I(f"buffer_store_dwordx4 v[4:7], v2, s[{S_RNGD}:{S_RNGD + 3}], 0 offen", VSTORE, rd=vr(4, 4) + vr(2) + sr(S_RNGD, 4)),
                label(l_norng)]
        Rq, Rkv, Ro = A["Rq"], A["Rkv"], A["Ro"]
        # ---- per-lane values (v1 = wave, V_LANE = lane) ----
        ins += [I(f"v_and_b32_e32 v2, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(2)),
                I(f"v_lshrrev_b32_e32 v3, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(3)),
                I(f"v_lshlrev_b32_e32 v{V_HH4}, 2, v3", VALU, rd=vr(3), wr=vr(V_HH4))]
        # Q / O row offsets: row (in the block) = 64 wave + 32 j + r
        for j in range(2):
            ins += [I(f"v_lshl_add_u32 v{V_ROW[j]}, v1, 6, v2", VALU, rd=vr(1) + vr(2), wr=vr(V_ROW[j])),
                    I(f"v_add_u32_e32 v{V_ROW[j]}, {32 * j}, v{V_ROW[j]}", VALU, rd=vr(V_ROW[j]), wr=vr(V_ROW[j])),
                    I(f"v_mul_lo_u32 v{V_QOFF[j]}, v{V_ROW[j]}, s{Rq}", VALU, rd=vr(V_ROW[j]) + sr(Rq), wr=vr(V_QOFF[j])),
                    I(f"v_lshl_add_u32 v{V_QOFF[j]}, v3, 4, v{V_QOFF[j]}", VALU, rd=vr(3) + vr(V_QOFF[j]), wr=vr(V_QOFF[j])),
                    I(f"v_lshlrev_b32_e32 v{V_LSEOFF[j]}, 2, v{V_ROW[j]}", VALU, rd=vr(V_ROW[j]), wr=vr(V_LSEOFF[j])),
                    I(f"v_mul_lo_u32 v{V_OOFF[j]}, v{V_ROW[j]}, s{Ro}", VALU, rd=vr(V_ROW[j]) + sr(Ro), wr=vr(V_OOFF[j])),
                    I(f"v_lshl_add_u32 v{V_OOFF[j]}, v3, 4, v{V_OOFF[j]}", VALU, rd=vr(3) + vr(V_OOFF[j]), wr=vr(V_OOFF[j]))]
        # LDS lane bases (fa_common.h LdsBases): rb = r*64 + ((c ^ xr) << 4), c = hh / 2+hh, xr = (r>>2)&3
        ins += [I("v_bfe_u32 v4, v2, 2, 2", VALU, rd=vr(2), wr=vr(4)),                      # xr
                I("v_xor_b32_e32 v5, v3, v4", VALU, rd=vr(3) + vr(4), wr=vr(5)),
                I("v_lshlrev_b32_e32 v6, 6, v2", VALU, rd=vr(2), wr=vr(6)),
                I(f"v_lshl_add_u32 v{V_RB0}, v5, 4, v6", VALU, rd=vr(5) + vr(6), wr=vr(V_RB0)),
                I("v_add_u32_e32 v5, 2, v3", VALU, rd=vr(3), wr=vr(5)),
                I("v_xor_b32_e32 v5, v5, v4", VALU, rd=vr(5) + vr(4), wr=vr(5)),
                I(f"v_lshl_add_u32 v{V_RB1}, v5, 4, v6", VALU, rd=vr(5) + vr(6), wr=vr(V_RB1))]
        # tb: i = lane & 15, q = i >> 2, pp = i & 3, trc = 2 (r >> 4) + (pp >> 1)
        #     tb0 = (4 hh + q) 64 + ((trc ^ hh) << 4) + (pp & 1) 8 ; tb1 = ... ((trc ^ (2 + hh)) << 4) ...
        ins += [I(f"v_and_b32_e32 v4, 15, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(4)),        # i
                I("v_lshrrev_b32_e32 v5, 2, v4", VALU, rd=vr(4), wr=vr(5)),                  # q
                I("v_and_b32_e32 v6, 3, v4", VALU, rd=vr(4), wr=vr(6)),                      # pp
                I("v_lshrrev_b32_e32 v7, 4, v2", VALU, rd=vr(2), wr=vr(7)),                  # r >> 4
                I("v_lshrrev_b32_e32 v8, 1, v6", VALU, rd=vr(6), wr=vr(8)),                  # pp >> 1
                I("v_lshl_add_u32 v7, v7, 1, v8", VALU, rd=vr(7) + vr(8), wr=vr(7)),          # trc
                I("v_lshl_add_u32 v8, v3, 2, v5", VALU, rd=vr(3) + vr(5), wr=vr(8)),          # 4 hh + q
                I("v_lshlrev_b32_e32 v8, 6, v8", VALU, rd=vr(8), wr=vr(8)),
                I("v_and_b32_e32 v9, 1, v6", VALU, rd=vr(6), wr=vr(9)),
                I("v_lshl_add_u32 v8, v9, 3, v8", VALU, rd=vr(9) + vr(8), wr=vr(8)),          # + (pp & 1) 8
                I("v_xor_b32_e32 v9, v7, v3", VALU, rd=vr(7) + vr(3), wr=vr(9)),
                I(f"v_lshl_add_u32 v{V_TB0}, v9, 4, v8", VALU, rd=vr(9) + vr(8), wr=vr(V_TB0)),
                I("v_add_u32_e32 v9, 2, v3", VALU, rd=vr(3), wr=vr(9)),
                I("v_xor_b32_e32 v9, v7, v9", VALU, rd=vr(7) + vr(9), wr=vr(9)),
                I(f"v_lshl_add_u32 v{V_TB1}, v9, 4, v8", VALU, rd=vr(9) + vr(8), wr=vr(V_TB1))]
        # DMA voffsets (tile 0): row = 16 wave + lane / 4, chunk = (lane & 3) ^ ((row >> 2) & 3);
        # voff_j = row * kv_row + 64 j + 16 chunk
        ins += [I(f"v_lshrrev_b32_e32 v4, 2, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(4)),
                I("v_lshl_add_u32 v4, v1, 4, v4", VALU, rd=vr(1) + vr(4), wr=vr(4)),              # row
                I("v_bfe_u32 v5, v4, 2, 2", VALU, rd=vr(4), wr=vr(5)),
                I(f"v_and_b32_e32 v6, 3, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(6)),
                I("v_xor_b32_e32 v5, v5, v6", VALU, rd=vr(5) + vr(6), wr=vr(5)),                   # chunk
                I(f"v_mul_lo_u32 v4, v4, s{Rkv}", VALU, rd=vr(4) + sr(Rkv), wr=vr(4)),
                I(f"v_lshl_add_u32 v{V_VOFF}, v5, 4, v4", VALU, rd=vr(5) + vr(4), wr=vr(V_VOFF))]
        for jj in range(1, NP):
            ins.append(I(f"v_add_u32_e32 v{V_VOFF + jj}, {64 * jj}, v{V_VOFF}", VALU, rd=vr(V_VOFF), wr=vr(V_VOFF + jj)))
        ins += [I(f"v_mov_b32_e32 v{V_NINF}, 0xff800000", VALU, wr=vr(V_NINF))]
        if OPT_MFZERO:
            ins += [I(f"v_mov_b32_e32 v{V_ZERO + i}, 0", VALU, wr=vr(V_ZERO + i)) for i in range(4)]
        if self.causal:
            # diagonal mask tiles: element g of a lane holds key (g & 3) + 8 (g >> 2) + 4 hh of the
            # subtile, query r = lane & 31 (v2)
            for g in range(16):
                kr = (g & 3) + 8 * (g >> 2)
                ins += [I(f"v_add_u32_e32 v4, {kr}, v{V_HH4}", VALU, rd=vr(V_HH4), wr=vr(4)),
                        I("v_cmp_gt_u32_e32 vcc, v4, v2", VALU, rd=vr(4) + vr(2), wr=[("vcc", 0)]),
                        I(f"v_cndmask_b32_e64 v{V_TRI + g}, 0, v{V_NINF}, vcc", VALU,
                          rd=vr(V_NINF) + [("vcc", 0)], wr=vr(V_TRI + g))]
                if not OPT_FOLD:
                    ins += [I(f"v_mov_b32_e32 v{V_NT + g}, v{V_NINF}", VALU, rd=vr(V_NINF), wr=vr(V_NT + g))]
        ins += [I(f"s_lshl_b32 s{S_TB}, s{Rkv}, 6", SALU, rd=sr(Rkv), wr=sr(S_TB)),
                I(f"s_mov_b32 s{S_ROUND}, 0", SALU, wr=sr(S_ROUND)),
                I(f"s_mov_b32 s{S_WARM}, 0", SALU, wr=sr(S_WARM)),
                I(f"s_mov_b32 s{S_DT}, 0", SALU, wr=sr(S_DT)),
                # the rng_state store has read its descriptor before anything rewrites s92..95
                I("s_waitcnt vmcnt(0)", WAIT)]
        return ins

    def item_pos(self, dst, plus):
        """dst = r G + (r odd ? rev(w) : w), r = S_ROUND + plus: snake order over the sorted items.
        rev(w) = G - 8 - (w & ~7) + (w & 7) when G % 8 == 0 -- the reversal runs over groups of 8
        workgroups, so workgroup w stays on the items of the XCD it runs on (w mod 8; the heads of a
        level are fastest in the list, so a head keeps its XCD and its K/V stay in that L2) -- else
        G - 1 - w."""
        I = Inst
        T, R, U = S_TMP, S_TMP + 1, S_TMP + 2
        return [I(f"s_add_u32 s{R}, s{S_ROUND}, {plus}", SALU),
                I(f"s_mul_i32 s{dst}, s{R}, s{S_GRID}", SALU),
                I(f"s_and_b32 s{U}, s2, {0 if OPT_PLAIN_SNAKE else 7}", SALU),
                I(f"s_lshl_b32 s{U}, s{U}, 1", SALU),
                I(f"s_sub_u32 s{T}, s{S_GRID}, {1 if OPT_PLAIN_SNAKE else 8}", SALU),
                I(f"s_sub_u32 s{T}, s{T}, s2", SALU),
                I(f"s_add_u32 s{T}, s{T}, s{U}", SALU),
                I(f"s_sub_u32 s{U}, s{S_GRID}, 1", SALU),
                I(f"s_sub_u32 s{U}, s{U}, s2", SALU),
                I(f"s_and_b32 s{R + 0}, s{R}, 1", SALU),          # keep r's parity only (dst holds r G)
                I(f"s_bitcmp1_b32 s{S_GRID}, 0", SALU),
                I(f"s_cselect_b32 s{T}, s{U}, s{T}", SALU),
                I(f"s_bitcmp1_b32 s{S_GRID}, 1", SALU),
                I(f"s_cselect_b32 s{T}, s{U}, s{T}", SALU),
                I(f"s_bitcmp1_b32 s{S_GRID}, 2", SALU),
                I(f"s_cselect_b32 s{T}, s{U}, s{T}", SALU),
                I(f"s_bitcmp1_b32 s{R}, 0", SALU),
                I(f"s_cselect_b32 s{T}, s{T}, s2", SALU),
                I(f"s_add_u32 s{dst}, s{dst}, s{T}", SALU)]

    def item_geom(self, kind, l_skip):
        """Geometry of the item at list position S_SWT.  kind 'cold' / 'warm': the current item --
        Q (cold) / O / LSE (and K / V when cold) descriptors, m0 in S_M0R, tile counts; 'next': the
        next item's Q / K / V descriptors (S_QD2 / S_KD2 / S_VD2) and tile count S_NXN (0 when it
        does not exist or is empty).  The table entry is (bidb | head << 16, kvh | m_block << 16)."""
        I = Inst
        A = self.kargs()
        T0, T1, T2, T3 = S_TMP, S_TMP + 1, S_TMP + 2, S_TMP + 3
        nxt = kind == "next"
        ins = []
        l_none = self.lab("none") if nxt else None
        l_done = self.lab("gdone") if nxt else None
        if nxt:
            ins += self.item_pos(S_SWT, 1)
            ins += [I(f"s_cmp_ge_u32 s{S_SWT}, s{S_NITEMS}", SALU), I(f"s_cbranch_scc1 {l_none}", BRANCH)]
        Psch = A["Psch"]
        # scalars: bidb (T2), head (T3), kvh (S_N), m_block (S_N0) -- temporarily
        BIDB, HEAD, KVH, MB = T2, T3, S_N, S_N0
        # fixed length: computed from the item index (fa_params.h ItemDecode, dwords at DEC_OFF into
        # s[88:97], free until the geometry below); varlen with a device-built list (flags bit 1): its
        # entry (bidb | head << 16, kvh | m_block << 16)
        l_tab, l_dec = self.lab("tab"), self.lab("dec")
        ins += [I(f"s_bitcmp1_b32 s{A['FL']}, 1", SALU), I(f"s_cbranch_scc1 {l_tab}", BRANCH)]
        if kind == "cold" and OPT_DECBURST:
            # round 0 (the workgroup's first item, entered from entry()): s[88:97] already hold it
            l_have = self.lab("decin")
            ins += [I(f"s_cmp_eq_u32 s{S_ROUND}, 0", SALU), I(f"s_cbranch_scc1 {l_have}", BRANCH)]
        ins += [I(f"s_load_dwordx8 s[88:95], s[0:1], {DEC_OFF}", SMEM),
                I(f"s_load_dwordx2 s[96:97], s[0:1], {DEC_OFF + 32}", SMEM),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        if kind == "cold" and OPT_DECBURST:
            ins += [label(l_have)]
        ins += item_decode_ops(L=S_SWT, M=88, pa=T0, pb=T2, t=S_N, u=S_M0R, o_blk=MB, reverse=True)
        ins += [I(f"s_mov_b32 s{HEAD}, s{S_M0R}", SALU), I(f"s_mov_b32 s{KVH}, s{T0}", SALU),
                I(f"s_branch {l_dec}", BRANCH), label(l_tab)]
        ins += [I(f"s_lshl_b32 s{T0}, s{S_SWT}, 3", SALU, rd=sr(S_SWT), wr=sr(T0)),
                I(f"s_load_dwordx2 s[{T0}:{T1}], s[{Psch}:{Psch + 1}], s{T0}", SMEM, rd=sr(Psch, 2) + sr(T0), wr=sr(T0, 2)),
                I("s_waitcnt lgkmcnt(0)", WAIT)]
        ins += [I(f"s_and_b32 s{BIDB}, s{T0}, 0xffff", SALU, rd=sr(T0), wr=sr(BIDB)),
                I(f"s_lshr_b32 s{HEAD}, s{T0}, 16", SALU, rd=sr(T0), wr=sr(HEAD)),
                I(f"s_and_b32 s{KVH}, s{T1}, 0xffff", SALU, rd=sr(T1), wr=sr(KVH)),
                I(f"s_lshr_b32 s{MB}, s{T1}, 16", SALU, rd=sr(T1), wr=sr(MB)), label(l_dec)]
        # varlen geometry (BlockInfo, block_info.h:14-31): 64-bit byte offsets (lo, hi) of row 0 of
        # this sequence in Q, O and K/V; seqlens in SQ / SK (overwritten in place)
        QOFF, OOFF, KOFF = (86, 87), (88, 89), (90, 91)
        SQ, SK = A["SQ"], A["SK"]

        def mul64(dst, a32, b32):
            return [I(f"s_mul_i32 s{dst[0]}, s{a32}, s{b32}", SALU, rd=sr(a32) + sr(b32), wr=sr(dst[0])),
                    I(f"s_mul_hi_u32 s{dst[1]}, s{a32}, s{b32}", SALU, rd=sr(a32) + sr(b32), wr=sr(dst[1]))]

        def mul64_i64(dst, a32, b64):   # a32 * (b64 lo, hi) -> dst (lo, hi)
            return [I(f"s_mul_i32 s{dst[0]}, s{a32}, s{b64}", SALU, rd=sr(a32) + sr(b64), wr=sr(dst[0])),
                    I(f"s_mul_hi_u32 s{dst[1]}, s{a32}, s{b64}", SALU, rd=sr(a32) + sr(b64), wr=sr(dst[1])),
                    I(f"s_mul_i32 s{T0}, s{a32}, s{b64 + 1}", SALU, rd=sr(a32) + sr(b64 + 1), wr=sr(T0)),
                    I(f"s_add_u32 s{dst[1]}, s{dst[1]}, s{T0}", SALU, rd=sr(dst[1]) + sr(T0), wr=sr(dst[1]))]

        parts = [(A["Pcq"], A["Bq"], A["Rq"], QOFF, SQ)]
        if not nxt:
            parts.append((A["Pcq"], A["Bo"], A["Ro"], OOFF, None))
        parts.append((A["Pck"], A["Bk"], A["Rkv"], KOFF, SK))
        # varlen: the cu_seqlens loads of every part are issued together and waited for once (one
        # scalar-memory round trip per item start instead of one per part)
        ins += [I(f"s_lshl_b32 s{T1}, s{BIDB}, 2", SALU, rd=sr(BIDB), wr=sr(T1))]
        for cu, bstride, rstride, off, seq in parts:
            lf = self.lab("nold")
            ins += [I(f"s_cmp_eq_u64 s[{cu}:{cu + 1}], 0", SALU, rd=sr(cu, 2), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH),
                    I(f"s_load_dwordx2 s[{off[0]}:{off[1]}], s[{cu}:{cu + 1}], s{T1}", SMEM, rd=sr(cu, 2) + sr(T1), wr=sr(off[0], 2)),
                    label(lf)]
        ins += [I("s_waitcnt lgkmcnt(0)", WAIT)]
        for cu, bstride, rstride, off, seq in parts:
            lf, ld = self.lab("fixed"), self.lab("vdone")
            ins += [I(f"s_cmp_eq_u64 s[{cu}:{cu + 1}], 0", SALU, rd=sr(cu, 2), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH)]
            if seq is not None:
                ins += [I(f"s_sub_u32 s{seq}, s{off[1]}, s{off[0]}", SALU, rd=sr(off[0], 2), wr=sr(seq))]
            ins += [I(f"s_bitcmp1_b32 s{A['FL']}, 0", SALU, rd=sr(A["FL"]), wr=[("scc", 0)]),
                    I(f"s_cbranch_scc1 {lf}", BRANCH),
                    I(f"s_mov_b32 s{T1}, s{off[0]}", SALU, rd=sr(off[0]), wr=sr(T1))]
            ins += mul64(off, T1, rstride)
            ins += [I(f"s_branch {ld}", BRANCH), label(lf)]
            ins += mul64_i64(off, BIDB, bstride)
            ins += [label(ld)]
        # m0 = 256 m_block; an item past its sequence is skipped (cur) / counts as absent (next)
        M0R = S_M0R
        ins += [I(f"s_lshl_b32 s{M0R}, s{MB}, 8", SALU, rd=sr(MB), wr=sr(M0R)),
                I(f"s_cmp_ge_i32 s{M0R}, s{SQ}", SALU, rd=sr(M0R) + sr(SQ), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_none if nxt else l_skip}", BRANCH)]
        # rows of this item: nrow = min(sq - m0, 256)
        NROW = S_SWT if nxt else S_NBLK
        ins += [I(f"s_sub_u32 s{NROW}, s{SQ}, s{M0R}", SALU, rd=sr(SQ) + sr(M0R), wr=sr(NROW)),
                I(f"s_min_u32 s{NROW}, s{NROW}, {BM}", SALU, rd=sr(NROW), wr=sr(NROW))]

        def addr(dst4, ptr, off64, head, hstride, rows=None, rstride=None, nrec=None):
            """descriptor at ptr + off64 + head * hstride (+ rows * rstride)"""
            o = []
            o += [I(f"s_mul_i32 s{T0}, s{head}, s{hstride}", SALU, rd=sr(head) + sr(hstride), wr=sr(T0)),
                  I(f"s_mul_hi_u32 s{T1}, s{head}, s{hstride}", SALU, rd=sr(head) + sr(hstride), wr=sr(T1)),
                  I(f"s_add_u32 s{dst4}, s{ptr}, s{T0}", SALU, rd=sr(ptr) + sr(T0), wr=sr(dst4) + [("scc", 0)]),
                  I(f"s_addc_u32 s{dst4 + 1}, s{ptr + 1}, s{T1}", SALU, rd=sr(ptr + 1) + sr(T1) + [("scc", 0)], wr=sr(dst4 + 1) + [("scc", 0)]),
                  I(f"s_add_u32 s{dst4}, s{dst4}, s{off64[0]}", SALU, rd=sr(dst4) + sr(off64[0]), wr=sr(dst4) + [("scc", 0)]),
                  I(f"s_addc_u32 s{dst4 + 1}, s{dst4 + 1}, s{off64[1]}", SALU, rd=sr(dst4 + 1) + sr(off64[1]) + [("scc", 0)], wr=sr(dst4 + 1))]
            if rows is not None:
                o += [I(f"s_mul_i32 s{T0}, s{rows}, s{rstride}", SALU, rd=sr(rows) + sr(rstride), wr=sr(T0)),
                      I(f"s_mul_hi_u32 s{T1}, s{rows}, s{rstride}", SALU, rd=sr(rows) + sr(rstride), wr=sr(T1)),
                      I(f"s_add_u32 s{dst4}, s{dst4}, s{T0}", SALU, rd=sr(dst4) + sr(T0), wr=sr(dst4) + [("scc", 0)]),
                      I(f"s_addc_u32 s{dst4 + 1}, s{dst4 + 1}, s{T1}", SALU, rd=sr(dst4 + 1) + sr(T1), wr=sr(dst4 + 1))]
            o += [I(f"s_and_b32 s{dst4 + 1}, s{dst4 + 1}, 0xffff", SALU, rd=sr(dst4 + 1), wr=sr(dst4 + 1))]
            o += nrec
            o += [I(f"s_mov_b32 s{dst4 + 3}, 0x20000", SALU, wr=sr(dst4 + 3))]
            return o

        Rq, Rkv, Ro = A["Rq"], A["Rkv"], A["Ro"]
        qd = S_QD2 if nxt else S_QD
        kd, vd = (S_KD2, S_VD2) if nxt else (S_KD, S_VD)
        if kind != "warm":
            ins += addr(qd, A["Pq"], QOFF, HEAD, A["Hq"], rows=M0R, rstride=Rq,
                        nrec=[I(f"s_mul_i32 s{qd + 2}, s{NROW}, s{Rq}", SALU, rd=sr(NROW) + sr(Rq), wr=sr(qd + 2))])
        if not nxt:
            ins += addr(S_OD, A["Po"], OOFF, HEAD, A["Ho"], rows=M0R, rstride=Ro,
                        nrec=[I(f"s_mul_i32 s{S_OD + 2}, s{NROW}, s{Ro}", SALU, rd=sr(NROW) + sr(Ro), wr=sr(S_OD + 2))])
        # K / V descriptors: every key of this sequence and kv head (host checks sk * kv_row < 2^31)
        if kind != "warm":
            ins += addr(kd, A["Pk"], KOFF, KVH, A["Hk"],
                        nrec=[I(f"s_mul_i32 s{kd + 2}, s{SK}, s{Rkv}", SALU, rd=sr(SK) + sr(Rkv), wr=sr(kd + 2))])
            ins += addr(vd, A["Pv"], KOFF, KVH, A["Hv"],
                        nrec=[I(f"s_mul_i32 s{vd + 2}, s{SK}, s{Rkv}", SALU, rd=sr(SK) + sr(Rkv), wr=sr(vd + 2))])
        if not nxt:
            # LSE descriptor: lse + ((bidb * h + head) * lse_pitch + m0) * 4
            ins += [I(f"s_mul_i32 s{T0}, s{BIDB}, s{A['NH']}", SALU, rd=sr(BIDB) + sr(A["NH"]), wr=sr(T0)),
                    I(f"s_add_u32 s{T0}, s{T0}, s{HEAD}", SALU, rd=sr(T0) + sr(HEAD), wr=sr(T0)),
                    I(f"s_mul_i32 s{S_LD + 2}, s{T0}, s{A['LP']}", SALU, rd=sr(T0) + sr(A["LP"]), wr=sr(S_LD + 2)),
                    I(f"s_mul_hi_u32 s{S_LD + 3}, s{T0}, s{A['LP']}", SALU, rd=sr(T0) + sr(A["LP"]), wr=sr(S_LD + 3)),
                    I(f"s_add_u32 s{S_LD + 2}, s{S_LD + 2}, s{M0R}", SALU, rd=sr(S_LD + 2) + sr(M0R), wr=sr(S_LD + 2) + [("scc", 0)]),
                    I(f"s_addc_u32 s{S_LD + 3}, s{S_LD + 3}, 0", SALU, rd=sr(S_LD + 3), wr=sr(S_LD + 3)),
                    I(f"s_lshl_b64 s[{S_LD + 2}:{S_LD + 3}], s[{S_LD + 2}:{S_LD + 3}], 2", SALU, rd=sr(S_LD + 2, 2), wr=sr(S_LD + 2, 2)),
                    I(f"s_add_u32 s{S_LD}, s{A['Pl']}, s{S_LD + 2}", SALU, rd=sr(A["Pl"]) + sr(S_LD + 2), wr=sr(S_LD) + [("scc", 0)]),
                    I(f"s_addc_u32 s{S_LD + 1}, s{A['Pl'] + 1}, s{S_LD + 3}", SALU, rd=sr(A["Pl"] + 1) + sr(S_LD + 3), wr=sr(S_LD + 1)),
                    I(f"s_and_b32 s{S_LD + 1}, s{S_LD + 1}, 0xffff", SALU, rd=sr(S_LD + 1), wr=sr(S_LD + 1)),
                    I(f"s_lshl_b32 s{S_LD + 2}, s{NROW}, 2", SALU, rd=sr(NROW), wr=sr(S_LD + 2)),
                    I(f"s_mov_b32 s{S_LD + 3}, 0x20000", SALU, wr=sr(S_LD + 3))]
        # tile counts: n_end = causal ? min(sk, m0 + 256) : sk; nblk = ceil(n_end / 64);
        # nfast = min(nblk, (causal ? min(sk, m0 + 1) : sk) / 64)
        if self.causal:
            ins += [I(f"s_add_u32 s{T0}, s{M0R}, {BM}", SALU, rd=sr(M0R), wr=sr(T0)),
                    I(f"s_min_i32 s{T0}, s{T0}, s{SK}", SALU, rd=sr(T0) + sr(SK), wr=sr(T0)),
                    I(f"s_add_u32 s{T1}, s{M0R}, 1", SALU, rd=sr(M0R), wr=sr(T1)),
                    I(f"s_min_i32 s{T1}, s{T1}, s{SK}", SALU, rd=sr(T1) + sr(SK), wr=sr(T1))]
        else:
            ins += [I(f"s_mov_b32 s{T0}, s{SK}", SALU, rd=sr(SK), wr=sr(T0)),
                    I(f"s_mov_b32 s{T1}, s{SK}", SALU, rd=sr(SK), wr=sr(T1))]
        nb = S_NXN if nxt else S_NBLK
        ins += [I(f"s_max_i32 s{T0}, s{T0}, 0", SALU, rd=sr(T0), wr=sr(T0)),
                I(f"s_add_u32 s{T0}, s{T0}, {BN - 1}", SALU, rd=sr(T0), wr=sr(T0)),
                I(f"s_lshr_b32 s{nb}, s{T0}, 6", SALU, rd=sr(T0), wr=sr(nb))]
        if not nxt and OPT_STAMP:
            ins += [I(f"v_add_u32_e32 v{V_STAMP + 4}, s{S_NBLK}, v{V_STAMP + 4}", VALU),
                    I(f"v_add_u32_e32 v{V_STAMP + 5}, 1, v{V_STAMP + 5}", VALU)]
        if not nxt:
            ins += [I(f"s_lshr_b32 s{S_WD}, s{M0R}, 6", SALU, rd=sr(M0R), wr=sr(S_WD)),
                    I(f"s_add_u32 s{S_WD}, s{S_WD}, s{S_WAVE}", SALU, rd=sr(S_WD) + sr(S_WAVE), wr=sr(S_WD)),
                    I(f"s_max_i32 s{T1}, s{T1}, 0", SALU, rd=sr(T1), wr=sr(T1)),
                    I(f"s_lshr_b32 s{T1}, s{T1}, 6", SALU, rd=sr(T1), wr=sr(T1)),
                    I(f"s_min_u32 s{T1}, s{T1}, s{S_NBLK}", SALU, rd=sr(T1) + sr(S_NBLK), wr=sr(T1)),
                    I(f"s_sub_i32 s{S_NF2}, s{T1}, 2", SALU, rd=sr(T1), wr=sr(S_NF2)),
                    I(f"s_sub_i32 s{S_NL1}, s{S_NBLK}, 1", SALU, rd=sr(S_NBLK), wr=sr(S_NL1))]
            # per-lane mask limit base: (causal ? min(m0 + row, sk - 1) : sk - 1) - 4 hh
            ins += [I(f"s_sub_i32 s{T0}, s{SK}, 1", SALU, rd=sr(SK), wr=sr(T0))]
            for j in range(2):
                if self.causal:
                    ins += [I(f"v_add_u32_e32 v{V_LB[j]}, s{M0R}, v{V_ROW[j]}", VALU, rd=sr(M0R) + vr(V_ROW[j]), wr=vr(V_LB[j])),
                            I(f"v_min_i32_e32 v{V_LB[j]}, s{T0}, v{V_LB[j]}", VALU, rd=sr(T0) + vr(V_LB[j]), wr=vr(V_LB[j]))]
                else:
                    ins += [I(f"v_mov_b32_e32 v{V_LB[j]}, s{T0}", VALU, rd=sr(T0), wr=vr(V_LB[j]))]
                ins += [I(f"v_sub_u32_e32 v{V_LB[j]}, v{V_LB[j]}, v{V_HH4}", VALU, rd=vr(V_LB[j]) + vr(V_HH4), wr=vr(V_LB[j]))]
        else:
            ins += [I(f"s_branch {l_done}", BRANCH), label(l_none),
                    I(f"s_mov_b32 s{S_NXN}, 0", SALU)]
            ins += [I(f"s_mov_b32 s{S_QD2 + i}, s{S_QD + i}", SALU) for i in range(4)]
            ins += [I(f"s_mov_b32 s{S_QD2 + 2}, 0", SALU), label(l_done)]
        return ins

    def item_start(self, l_cold, l_cold_wait, l_warm, l_skip, l_tile0, l_epi, l_end):
        """cold start (first item; after an item whose successor could not be prefetched) and warm
        start (the next item's K/V tiles 0..2 and Q already issued by the previous item)"""
        I = Inst
        ins = []
        # ---- cold
        ins += [label(l_cold_wait)]
        if OPT_DEFER:
            ins += self.defer_stores(S_OD, S_LD)
        ins += [Inst("s_waitcnt vmcnt(0) lgkmcnt(0)", WAIT), Inst("s_barrier", BARRIER),
                label(l_cold)]
        ins += self.item_pos(S_SWT, 0)
        ins += [I(f"s_cmp_ge_u32 s{S_SWT}, s{S_NITEMS}", SALU), I(f"s_cbranch_scc1 {l_end}", BRANCH)]
        ins += self.item_geom("cold", l_skip)
        # DMA offsets back to tile 0 of the fresh descriptors
        ins += [I(f"s_mul_i32 s{S_SWT}, s{S_DT}, s{S_TB}", SALU)]
        ins += [I(f"v_subrev_u32_e32 v{V_VOFF + jj}, s{S_SWT}, v{V_VOFF + jj}", VALU) for jj in range(NP)]
        ins += [I(f"s_mov_b32 s{S_DT}, 0", SALU), I(f"s_mov_b32 s{S_DLIM}, s{S_NBLK}", SALU)]
        # Q fragments into the accumulator file: lane holds Q[row][16 ks + 8 hh .. +7]
        for j in range(2):
            for ks in range(KS):
                ins.append(I(f"buffer_load_dwordx4 {rtxt('a', Q_(j, ks), 4)}, v{V_QOFF[j]}, s[{S_QD}:{S_QD + 3}], 0 offen offset:{32 * ks}",
                             VLOAD, rd=vr(V_QOFF[j]) + sr(S_QD, 4), wr=ar(Q_(j, ks), 4)))
        ins += self.item_geom("next", None)
        ins += [I(f"s_mov_b32 s{S_WARM}, 0", SALU),
                I(f"s_mov_b32 s{S_KOFF}, 0", SALU),
                I(f"s_lshl_b32 s{S_DOFF}, s{S_WAVE}, 10", SALU)]
        ins += self.item_zero(o=False)
        # no tiles at all: epilogue (O = 0, LSE = +inf)
        l_nt = self.lab("notiles")
        ins += [I(f"s_cmp_eq_u32 s{S_NBLK}, 0", SALU, rd=sr(S_NBLK), wr=[("scc", 0)])]
        ins += [I("s_waitcnt vmcnt(0)", WAIT)] if OPT_QWAIT else []
        ins += [I(f"s_cbranch_scc1 {l_nt}", BRANCH)]
        for tile in range(4):
            ins += self.dma_tile_ops(f"c{tile}")
        ins += [I(f"s_branch {l_tile0}", BRANCH)]
        # an item with rows but no keys (a varlen sequence of length 0 in cu_seqlens_k): no tile 0 sets
        # the ring position, so the staged epilogue's region (the last tile's slot) is pinned to slot 0
        ins += [label(l_nt), I("s_waitcnt vmcnt(0)", WAIT), I(f"s_mov_b32 s{S_VOFF}, {VBASE + TILE}", SALU, wr=sr(S_VOFF)),
                I(f"s_branch {self.l_empty if OPT_T0ZERO else l_epi}", BRANCH)]
        ins += [label(l_skip), I(f"s_add_u32 s{S_ROUND}, s{S_ROUND}, 1", SALU), I(f"s_branch {l_cold}", BRANCH)]
        if OPT_T0ZERO:   # an item with no tiles: O = 0 for its epilogue (no tile 0 zeroes it)
            ins += [label(self.l_empty)] + self.o_zero_ops() + [I(f"s_branch {l_epi}", BRANCH)]
        # ---- warm
        ins += [label(l_warm)]
        ins += self.item_pos(S_SWT, 0)
        ins += [I(f"s_mov_b32 s{S_QD + i}, s{S_QD2 + i}", SALU) for i in range(4)]
        restore = []
        l_skip_w = l_skip
        if OPT_DEFER:
            assert not OPT_MFZERO
            ins += [I(f"v_mov_b32_e32 v{V_SAVE[i]}, s{S_OD + i}", VALU, rd=sr(S_OD + i), wr=vr(V_SAVE[i])) for i in range(3)]
            ins += [I(f"v_mov_b32_e32 v{V_SAVE[3 + i]}, s{S_LD + i}", VALU, rd=sr(S_LD + i), wr=vr(V_SAVE[3 + i])) for i in range(3)]
            restore = []
            for i in range(6):
                sd = S_ODD + i if i < 3 else S_LDD + i - 3
                restore += [nop(0), I(f"v_readfirstlane_b32 s{sd}, v{V_SAVE[i]}", RFL, rd=vr(V_SAVE[i]), wr=sr(sd))]
            restore += [I(f"s_mov_b32 s{S_ODD + 3}, 0x20000", SALU, wr=sr(S_ODD + 3)),
                        I(f"s_mov_b32 s{S_LDD + 3}, 0x20000", SALU, wr=sr(S_LDD + 3))]
            l_skip_w = self.lab("skipw")
        ins += self.item_geom("warm", l_skip_w)
        ins += self.item_geom("next", None)
        ins += [I(f"s_mov_b32 s{S_WARM}, 0", SALU),
                I(f"s_sub_u32 s{S_KOFF}, s{S_VOFF}, {VBASE}", SALU)]
        ins += self.item_zero(o=False)
        ins += restore
        ins += self.dma_tile_ops("w3")
        if OPT_DEFER:
            ins += [nop(5), I(f"s_branch {self.l_tile0w}", BRANCH),
                    label(l_skip_w)] + restore + [nop(5)] + self.defer_stores(S_ODD, S_LDD) + [I(f"s_branch {l_skip}", BRANCH)]
        return ins

    def o_zero_ops(self, key=0):
        return [Inst(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i), key=key + i) for i in range(2 * NP * 16)]

    def item_zero(self, o=True):
        I = Inst
        ins = [I(f"s_mov_b32 s{S_N}, 0", SALU, wr=sr(S_N)),
               I(f"s_mov_b32 s{S_N0}, 0", SALU, wr=sr(S_N0))]
        if OPT_T0ZERO and not o:
            pass
        elif OPT_MFZERO:   # O = 0 x 0 + 0: one MFMA per 16 accumulators instead of 16 v_accvgpr_write
            ins += [I(f"v_mfma_f32_32x32x16_{self.ty} {rtxt('a', 16 * i, 16)}, {rtxt('v', V_ZERO, 4)}, {rtxt('v', V_ZERO, 4)}, 0",
                      MFMA, rd=vr(V_ZERO, 4), wr=ar(16 * i, 16)) for i in range(2 * NP)]
        else:
            ins += [I(f"v_accvgpr_write_b32 a{i}, 0", ACCW, wr=ar(i)) for i in range(2 * NP * 16)]
        ins += [I(f"v_mov_b32_e32 v{V_L[0]}, 0", VALU, wr=vr(V_L[0])),
                I(f"v_mov_b32_e32 v{V_L[1]}, 0", VALU, wr=vr(V_L[1])),
                I(f"v_mov_b32_e32 v{V_NEGMC[0]}, 0", VALU, wr=vr(V_NEGMC[0])),
                I(f"v_mov_b32_e32 v{V_NEGMC[1]}, 0", VALU, wr=vr(V_NEGMC[1]))]
        return ins

    def tile0(self, l_entry_last, l_entry_fast, l_entry_masked, stores=False):
        """Q + tiles 0, 1, 2 landed (tile 3 in flight); tile 0: S(0, a), S(0, b) -> masked, explicit
        row max, P(0, a); then into the step loop"""
        if OPT_FOLD:
            return self.tile0_fold(l_entry_last, l_entry_fast, l_entry_masked)
        I = Inst
        if OPT_T0STAMP:
            ins = (self.stamp_point(9) + [I(f"s_waitcnt vmcnt({2 * NP})", WAIT)] + self.stamp_point(6) +
                   [I("s_barrier", BARRIER)] + self.stamp_point(5))
        else:
            ins = [I(f"s_waitcnt vmcnt({2 * NP})", WAIT), I("s_barrier", BARRIER)]
            ins += [] if OPT_EPISTAMP else self.stamp_point(9)
        ins += self.dump("pro_lds")
        ins += [I(f"v_add_u32_e32 v{V_KB0}, s{S_KOFF}, v{V_RB0}", VALU, rd=sr(S_KOFF) + vr(V_RB0), wr=vr(V_KB0)),
                I(f"v_add_u32_e32 v{V_KB1}, s{S_KOFF}, v{V_RB1}", VALU, rd=sr(S_KOFF) + vr(V_RB1), wr=vr(V_KB1))]
        mfm = []
        for i in range(NX):
            st, ks, j = i // (2 * KS), (i % (2 * KS)) // 2, i % 2
            f = st * KS + ks
            sreg = (SA if j == 0 else SB(0)) + 16 * st
            mfm.append(self.mfma_s(sreg, f % 8, j, ks, ks == 0))
        reads = []
        for f in range(2 * KS):
            reads.append(self.kread(f, f % 8, key=f, earliest=max(2 * (f - 3), 2 * (f - 8) + 3) if f >= 3 else None,
                                    deadline=2 * f - 1 if f >= 3 else 0))
        if stores:
            reads += self.defer_stores(S_ODD, S_LDD, spread=NX)
        if OPT_T0ZERO:
            reads += self.o_zero_ops(key=100)
        if OPT_T0OV:
            assert not stores
            ins += self.tile0_overlapped()
        else:
            body = schedule(mfm, reads)
            ins += body
            ins.append(nop(15))
        ins += self.dump("pro_qk")
        for j, sreg in ((((1, SB(0)),) if OPT_T0OV else ((0, SA), (1, SB(0))))):
            ins += self.mask_ops(j, sreg, (S_N0, 0), V_LM)
            mx = V_T + 2
            ins.append(Inst(f"v_max3_f32 v{mx}, v{sreg}, v{sreg + 1}, v{sreg + 2}", VALU, rd=vr(sreg, 3), wr=vr(mx)))
            for e in range(3, 32, 2):
                if e + 1 < 32:
                    ins.append(Inst(f"v_max3_f32 v{mx}, v{mx}, v{sreg + e}, v{sreg + e + 1}", VALU, rd=vr(mx) + vr(sreg + e, 2), wr=vr(mx)))
                else:
                    ins.append(Inst(f"v_max_f32_e32 v{mx}, v{mx}, v{sreg + e}", VALU, rd=vr(mx) + vr(sreg + e), wr=vr(mx)))
            ins += self.half_max(mx, V_T + 3)
            # negmc = m == -inf ? 0 : -m c
            ins += [Inst(f"v_mul_f32_e32 v{V_T + 4}, s{S_C}, v{mx}", VALU, rd=sr(S_C) + vr(mx), wr=vr(V_T + 4)),
                    Inst(f"v_sub_f32_e32 v{V_NEGMC[j]}, 0, v{V_T + 4}", VALU, rd=vr(V_T + 4), wr=vr(V_NEGMC[j])),
                    Inst(f"v_cmp_eq_f32_e32 vcc, v{V_NINF}, v{mx}", VALU, rd=vr(V_NINF) + vr(mx), wr=[("vcc", 0)]),
                    Inst(f"v_cndmask_b32_e64 v{V_NEGMC[j]}, v{V_NEGMC[j]}, 0, vcc", VALU,
                         rd=vr(V_NEGMC[j]) + [("vcc", 0)], wr=vr(V_NEGMC[j]))]
        if not OPT_T0OV:
            sm, _ = self.softmax_ops(0, SA, PA(0), False, None, key0=0)
            ins += sm
            ins += [Inst(f"v_mov_b32_e32 v{V_L[0]}, v{V_PS[0]}", VALU, rd=vr(V_PS[0]), wr=vr(V_L[0]))]
        ins += self.dump("pro_end")
        ins += [] if (OPT_EPISTAMP or OPT_T0STAMP) else self.stamp_point(6)
        ins += self.tile0_exit(l_entry_last, l_entry_fast, l_entry_masked)
        return ins

    def tile0_exit(self, l_entry_last, l_entry_fast, l_entry_masked):
        """end of tile 0: V read slot, K(1) base and its first fragments, into the step loop"""
        I = Inst
        ins = []
        # V reads tile 0 (slot S_KOFF); S_KOFF -> tile 1 (the LAST step's refit takes S_KOFF - TILE)
        ins += [I(f"s_add_u32 s{S_VOFF}, s{S_KOFF}, {VBASE}", SALU),
                I(f"s_add_u32 s{S_KOFF}, s{S_KOFF}, {TILE}", SALU),
                I(f"s_sub_u32 s{S_SWT}, s{S_KOFF}, {NSLOT * TILE}", SALU),
                I(f"s_cmp_ge_u32 s{S_KOFF}, {NSLOT * TILE}", SALU),
                I(f"s_cselect_b32 s{S_KOFF}, s{S_SWT}, s{S_KOFF}", SALU),
                I(f"s_cmp_eq_u32 s{S_NBLK}, 1", SALU, rd=sr(S_NBLK), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_entry_last}", BRANCH)]
        # K(1) base + prefetch of its first three fragments
        ins += [I(f"v_add_u32_e32 v{V_KB0}, s{S_KOFF}, v{V_RB0}", VALU, rd=sr(S_KOFF) + vr(V_RB0), wr=vr(V_KB0)),
                I(f"v_add_u32_e32 v{V_KB1}, s{S_KOFF}, v{V_RB1}", VALU, rd=sr(S_KOFF) + vr(V_RB1), wr=vr(V_KB1))]
        for f in range(3):
            ins.append(self.kread(f, f % 8))
        ins += [I("s_waitcnt lgkmcnt(0)", WAIT),
                I(f"s_cmp_ge_i32 s{S_NF2}, 0", SALU, rd=sr(S_NF2), wr=[("scc", 0)]),
                I(f"s_cbranch_scc1 {l_entry_fast}", BRANCH),
                I(f"s_branch {l_entry_masked}", BRANCH)]
        return ins

    def tile0_maxops(self, j, sreg, key):
        """mask, explicit row max and -m c of q-block j's first tile (tile 0)"""
        ops = self.mask_ops(j, sreg, (S_N0, 0), V_LM, key0=key)
        mx = V_T + 2
        ops.append(Inst(f"v_max3_f32 v{mx}, v{sreg}, v{sreg + 1}, v{sreg + 2}", VALU, rd=vr(sreg, 3), wr=vr(mx), key=key + 200))
        for e in range(3, 32, 2):
            if e + 1 < 32:
                ops.append(Inst(f"v_max3_f32 v{mx}, v{mx}, v{sreg + e}, v{sreg + e + 1}", VALU, rd=vr(mx) + vr(sreg + e, 2),
                                wr=vr(mx), key=key + 200))
            else:
                ops.append(Inst(f"v_max_f32_e32 v{mx}, v{mx}, v{sreg + e}", VALU, rd=vr(mx) + vr(sreg + e), wr=vr(mx), key=key + 200))
        for op in self.half_max(mx, V_T + 3):
            op.key = key + 200
            ops.append(op)
        if OPT_FOLD:   # (the scores are c S already)
            ops += [Inst(f"v_sub_f32_e32 v{V_NEGMC[j]}, 0, v{mx}", VALU, rd=vr(mx), wr=vr(V_NEGMC[j]), key=key + 200)]
        else:
            ops += [Inst(f"v_mul_f32_e32 v{V_T + 4}, s{S_C}, v{mx}", VALU, rd=sr(S_C) + vr(mx), wr=vr(V_T + 4), key=key + 200),
                    Inst(f"v_sub_f32_e32 v{V_NEGMC[j]}, 0, v{V_T + 4}", VALU, rd=vr(V_T + 4), wr=vr(V_NEGMC[j]), key=key + 200)]
        ops += [Inst(f"v_cmp_eq_f32_e32 vcc, v{V_NINF}, v{mx}", VALU, rd=vr(V_NINF) + vr(mx), wr=[("vcc", 0)], key=key + 200),
                Inst(f"v_cndmask_b32_e64 v{V_NEGMC[j]}, v{V_NEGMC[j]}, 0, vcc", VALU,
                     rd=vr(V_NEGMC[j]) + [("vcc", 0)], wr=vr(V_NEGMC[j]), key=key + 200)]
        return ops

    def tile0_overlapped(self):
        """tile 0's QK with q-block a's MFMAs first: a's mask, max and softmax run in the gaps of b's
        MFMAs (K fragments re-read for b at d = 128, where the 8-slot ring cannot hold all 16)"""
        mfm = []
        for j in range(2):
            for st in range(2):
                for ks in range(KS):
                    f = st * KS + ks
                    sreg = (SA if j == 0 else SB(0)) + 16 * st
                    mfm.append(self.mfma_s(sreg, f % 8, j, ks, ks == 0))
        n2 = 2 * KS
        fill = []
        for f in range(n2):
            fill.append(self.kread(f, f % 8, key=-100 + f, earliest=(f - 8) if f >= 8 else None, deadline=max(f - 2, 0)))
        if n2 > 8:
            for f in range(n2):
                fill.append(self.kread(f, f % 8, key=-60 + f, earliest=f + 8, deadline=n2 + f - 2))
        fill += self.tile0_maxops(0, SA, key=0)
        sm, _ = self.softmax_ops(0, SA, PA(0), False, None, key0=400)
        fill += sm
        fill += [Inst(f"v_mov_b32_e32 v{V_L[0]}, v{V_PS[0]}", VALU, rd=vr(V_PS[0]), wr=vr(V_L[0]), key=700)]
        return schedule(mfm, fill) + [nop(15)]

    # ------------------------------------------------------------------ epilogue
    def defer_stores(self, od, ld, spread=0):
        """(FA_GEN_DEFER) the finished item's LSE and O stores from V_LSEV / PKR with descriptors
        s[od:od+3], s[ld:ld+3]; spread > 0: store i not before MFMA gap i * spread / count"""
        out = []
        for j in range(2):
            out.append(Inst(f"buffer_store_dword v{V_LSEV[j]}, v{V_LSEOFF[j]}, s[{ld}:{ld + 3}], 0 offen", VSTORE,
                            rd=vr(V_LSEV[j]) + vr(V_LSEOFF[j]) + sr(ld, 4)))
            for dt in range(NP):
                for u in (0, 2):
                    w = PKR(j, dt, u)
                    out.append(Inst(f"buffer_store_dwordx4 v[{w}:{w + 3}], v{V_OOFF[j]}, s[{od}:{od + 3}], 0 offen offset:{64 * dt + 16 * u}",
                                    VSTORE, rd=vr(w, 4) + vr(V_OOFF[j]) + sr(od, 4)))
        for i, op in enumerate(out):
            op.key = 300 + i
            if spread:
                op.eg = i * spread // len(out)
        return out

    def lse_ops(self, j, inv, lse, t2, t3):
        """1 / l -> v[inv], LSE -> v[lse] of q-block j (bad l: inv = 1, LSE = +inf)"""
        l = V_L[j]
        ins = self.half_sum(l, t2)
        ins += [Inst(f"v_rcp_f32_e32 v{inv}, v{l}", TRANS, rd=vr(l), wr=vr(inv)),
                Inst(f"v_log_f32_e32 v{lse}, v{l}", TRANS, rd=vr(l), wr=vr(lse)),
                Inst(f"v_sub_f32_e32 v{lse}, v{lse}, v{V_NEGMC[j]}", VALU, rd=vr(lse) + vr(V_NEGMC[j]), wr=vr(lse)),
                Inst(f"v_mul_f32_e32 v{lse}, 0x3f317218, v{lse}", VALU, rd=vr(lse), wr=vr(lse)),
                Inst(f"v_cmp_neq_f32_e32 vcc, 0, v{l}", VALU, rd=vr(l), wr=[("vcc", 0)]),
                Inst(f"v_cmp_eq_f32_e64 s[{S_TMP}:{S_TMP + 1}], v{l}, v{l}", VALU, rd=vr(l), wr=sr(S_TMP, 2)),
                Inst(f"s_and_b64 vcc, vcc, s[{S_TMP}:{S_TMP + 1}]", SALU, rd=sr(S_TMP, 2) + [("vcc", 0)], wr=[("vcc", 0)]),
                Inst(f"v_cndmask_b32_e64 v{inv}, 1.0, v{inv}, vcc", VALU, rd=vr(inv) + [("vcc", 0)], wr=vr(inv)),
                Inst(f"v_mov_b32_e32 v{t3}, 0x7f800000", VALU, wr=vr(t3)),
                Inst(f"v_cndmask_b32_e32 v{lse}, v{t3}, v{lse}, vcc", VALU, rd=vr(lse) + vr(t3) + [("vcc", 0)], wr=vr(lse))]
        return ins

    def epilogue_staged(self):
        """(FA_GEN_OSTAGE) O normalised, packed and written to LDS in row-major order (XOR-swizzled
        16-byte chunks), read back 16 bytes per lane with lpr lanes per row and stored as whole rows.
        The staging area is the K/V slot of the item's last tile: its K part was last read in the
        previous step (before that step's barrier), its V part in the last step -- hence the barrier
        first (a refit of the last step re-reads the K part too).  Wave w stages one q-block at a time
        in 32 rows x 2D bytes: waves 0, 1 in the K part, 2, 3 in the V part."""
        I = Inst
        Ro = self.kargs()["Ro"]
        RB = 2 * D                      # bytes per staged row
        NCH = RB // 16                  # 16-byte chunks per row
        lpr = NCH                       # lanes per row when reading back
        rpi = 64 // lpr                 # rows per read / store instruction
        nrd = 32 // rpi
        sh = 0 if D == 128 else 1       # swizzle key = (row >> sh) & (NCH - 1): conflict-free writes
        R = S_M0R                       # region base (SGPR)
        T = S_TMP + 2
        ins = [I("s_barrier", BARRIER)]
        # region: K slot of the last tile = S_VOFF - VBASE - TILE (mod the ring), + wave part
        ins += [I(f"s_sub_i32 s{R}, s{S_VOFF}, {VBASE + TILE}", SALU, rd=sr(S_VOFF), wr=sr(R)),
                I(f"s_add_u32 s{T}, s{R}, {NSLOT * TILE}", SALU, rd=sr(R), wr=sr(T)),
                I(f"s_cmp_lt_i32 s{R}, 0", SALU, rd=sr(R), wr=[("scc", 0)]),
                I(f"s_cselect_b32 s{R}, s{T}, s{R}", SALU, rd=sr(T) + sr(R) + [("scc", 0)], wr=sr(R)),
                I(f"s_and_b32 s{T}, s{S_WAVE}, 1", SALU, rd=sr(S_WAVE), wr=sr(T)),
                I(f"s_mul_i32 s{T}, s{T}, {32 * RB}", SALU, rd=sr(T), wr=sr(T)),
                I(f"s_add_u32 s{R}, s{R}, s{T}", SALU, rd=sr(R) + sr(T), wr=sr(R)),
                I(f"s_cmp_ge_u32 s{S_WAVE}, 2", SALU, rd=sr(S_WAVE), wr=[("scc", 0)]),
                I(f"s_cselect_b32 s{T}, {VBASE}, 0", SALU, rd=[("scc", 0)], wr=sr(T)),
                I(f"s_add_u32 s{R}, s{R}, s{T}", SALU, rd=sr(R) + sr(T), wr=sr(R))]
        # per-lane constants (v4..): q = lane & 31, hh = lane >> 5
        VQ, VH, VB, VK, VBR, VLR = 4, 5, 6, 7, 80, 88
        VA = 8                          # write addresses of the NCH chunks: v8 ..
        ins += [I(f"v_and_b32_e32 v{VQ}, 31, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(VQ)),
                I(f"v_lshrrev_b32_e32 v{VH}, 5, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(VH)),
                I(f"v_lshrrev_b32_e32 v{VK}, {sh}, v{VQ}", VALU, rd=vr(VQ), wr=vr(VK)),
                I(f"v_and_b32_e32 v{VK}, {NCH - 1}, v{VK}", VALU, rd=vr(VK), wr=vr(VK)),
                I(f"v_lshlrev_b32_e32 v{VK}, 4, v{VK}", VALU, rd=vr(VK), wr=vr(VK)),
                I(f"v_mul_u32_u24_e32 v{VB}, {RB}, v{VQ}", VALU, rd=vr(VQ), wr=vr(VB)),
                I(f"v_add_u32_e32 v{VB}, s{R}, v{VB}", VALU, rd=sr(R) + vr(VB), wr=vr(VB)),
                I(f"v_or_b32_e32 v{VB}, v{VB}, v{VK}", VALU, rd=vr(VB) + vr(VK), wr=vr(VB)),
                I(f"v_lshl_or_b32 v{VB}, v{VH}, 3, v{VB}", VALU, rd=vr(VH) + vr(VB), wr=vr(VB))]
        for c in range(NCH):
            ins.append(I(f"v_xor_b32_e32 v{VA + c}, {16 * c}, v{VB}", VALU, rd=vr(VB), wr=vr(VA + c)))
        # read-back: lane row lr = lane / lpr, chunk cc = lane % lpr; physical chunk = cc ^ key(row)
        # key(rpi i + lr) = key_i ^ (lr >> sh)  (disjoint bits), key_i = ((rpi i) >> sh) & (NCH - 1)
        lg = lpr.bit_length() - 1
        ins += [I(f"v_lshrrev_b32_e32 v{VLR}, {lg}, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(VLR)),            # lr
                I(f"v_and_b32_e32 v{VLR + 1}, {lpr - 1}, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(VLR + 1)),   # cc
                I(f"v_lshrrev_b32_e32 v{VLR + 2}, {sh}, v{VLR}", VALU, rd=vr(VLR), wr=vr(VLR + 2)),
                I(f"v_xor_b32_e32 v{VLR + 2}, v{VLR + 2}, v{VLR + 1}", VALU, rd=vr(VLR + 1, 2), wr=vr(VLR + 2)),
                I(f"v_mul_u32_u24_e32 v{VLR + 3}, {RB}, v{VLR}", VALU, rd=vr(VLR), wr=vr(VLR + 3)),
                I(f"v_add_u32_e32 v{VLR + 3}, s{R}, v{VLR + 3}", VALU, rd=sr(R) + vr(VLR + 3), wr=vr(VLR + 3)),
                I(f"v_lshl_or_b32 v{VLR + 3}, v{VLR + 2}, 4, v{VLR + 3}", VALU, rd=vr(VLR + 2, 2), wr=vr(VLR + 3))]
        keys = sorted({((rpi * i) >> sh) & (NCH - 1) for i in range(nrd)})
        kreg = {}
        for n, k in enumerate(keys):
            kreg[k] = VBR + n
            ins.append(I(f"v_xor_b32_e32 v{VBR + n}, {16 * k}, v{VLR + 3}", VALU, rd=vr(VLR + 3), wr=vr(VBR + n)))
        # global row offsets of the read-back rows: (64 wave + 32 j + lr) Ro + 16 cc
        VS = (VLR + 4, VLR + 5)
        ins += [I(f"v_lshlrev_b32_e32 v{VLR + 6}, 4, v{VLR + 1}", VALU, rd=vr(VLR + 1), wr=vr(VLR + 6))]
        for j in range(2):
            ins += [I(f"s_lshl_b32 s{T}, s{S_WAVE}, 6", SALU, rd=sr(S_WAVE), wr=sr(T)),
                    I(f"s_add_u32 s{T}, s{T}, {32 * j}", SALU, rd=sr(T), wr=sr(T)),
                    I(f"v_add_u32_e32 v{VS[j]}, s{T}, v{VLR}", VALU, rd=sr(T) + vr(VLR), wr=vr(VS[j])),
                    I(f"v_mul_lo_u32 v{VS[j]}, v{VS[j]}, s{Ro}", VALU, rd=vr(VS[j]) + sr(Ro), wr=vr(VS[j])),
                    I(f"v_add_u32_e32 v{VS[j]}, v{VS[j]}, v{VLR + 6}", VALU, rd=vr(VS[j]) + vr(VLR + 6), wr=vr(VS[j]))]
        RD = 48                          # read-back data v48 .. v79
        XT, PKT = 24, 40                 # 4 sets of 4 temps, 4 pairs
        for j in range(2):
            inv, lse = 0, 1
            ins += self.lse_ops(j, inv, lse, 2, 3)
            ins.append(I(f"buffer_store_dword v{lse}, v{V_LSEOFF[j]}, s[{S_LD}:{S_LD + 3}], 0 offen", VSTORE,
                         rd=vr(lse) + vr(V_LSEOFF[j]) + sr(S_LD, 4)))
            n = 0
            for dt in range(NP):
                for k4 in range(4):
                    x, pk = XT + 4 * (n % 4), PKT + 2 * (n % 4)
                    o = O_(j, dt) + 4 * k4
                    ins += [I(f"v_accvgpr_read_b32 v{x + k}, a{o + k}", ACCR, rd=ar(o + k), wr=vr(x + k)) for k in range(4)]
                    ins += [I(f"v_mul_f32_e32 v{x + k}, v{x + k}, v{inv}", VALU, rd=vr(x + k) + vr(inv), wr=vr(x + k)) for k in range(4)]
                    ins += [self.cvt(pk, x, x + 1), self.cvt(pk + 1, x + 2, x + 3)]
                    c = 4 * dt + k4
                    ins.append(I(f"ds_write_b64 v{VA + c}, v[{pk}:{pk + 1}]", LDS, rd=vr(VA + c) + vr(pk, 2)))
                    n += 1
            ins.append(I("s_waitcnt lgkmcnt(0)", WAIT))
            for i in range(nrd):
                k = ((rpi * i) >> sh) & (NCH - 1)
                ins.append(I(f"ds_read_b128 v[{RD + 4 * i}:{RD + 4 * i + 3}], v{kreg[k]} offset:{rpi * i * RB}", LDS,
                             rd=vr(kreg[k]), wr=vr(RD + 4 * i, 4)))
            ins.append(I("s_waitcnt lgkmcnt(0)", WAIT))
            for i in range(nrd):
                ins += [I(f"s_mul_i32 s{T}, s{Ro}, {rpi * i}", SALU, rd=sr(Ro), wr=sr(T)),
                        I(f"buffer_store_dwordx4 v[{RD + 4 * i}:{RD + 4 * i + 3}], v{VS[j]}, s[{S_OD}:{S_OD + 3}], s{T} offen",
                          VSTORE, rd=vr(RD + 4 * i, 4) + vr(VS[j]) + sr(S_OD, 4) + sr(T))]
        return ins

    def epilogue(self):
        if OPT_EPI2:
            return self.epilogue2()
        if OPT_OSTAGE:
            return self.epilogue_staged()
        ins = []
        t = 0   # the score registers are free after the last step
        for j in range(2):
            l, inv, lse = V_L[j], t, t + 1
            ins += self.half_sum(l, t + 2)
            # bad = l == 0 || l != l  -> inv = 1, lse = +inf
            ins += [Inst(f"v_rcp_f32_e32 v{inv}, v{l}", TRANS, rd=vr(l), wr=vr(inv)),
                    Inst(f"v_log_f32_e32 v{lse}, v{l}", TRANS, rd=vr(l), wr=vr(lse)),
                    Inst(f"v_sub_f32_e32 v{lse}, v{lse}, v{V_NEGMC[j]}", VALU, rd=vr(lse) + vr(V_NEGMC[j]), wr=vr(lse)),
                    Inst(f"v_mul_f32_e32 v{lse}, 0x3f317218, v{lse}", VALU, rd=vr(lse), wr=vr(lse)),
                    Inst(f"v_cmp_neq_f32_e32 vcc, 0, v{l}", VALU, rd=vr(l), wr=[("vcc", 0)]),
                    Inst(f"v_cmp_eq_f32_e64 s[{S_TMP}:{S_TMP + 1}], v{l}, v{l}", VALU, rd=vr(l), wr=sr(S_TMP, 2)),
                    Inst(f"s_and_b64 vcc, vcc, s[{S_TMP}:{S_TMP + 1}]", SALU, rd=sr(S_TMP, 2) + [("vcc", 0)], wr=[("vcc", 0)]),
                    Inst(f"v_cndmask_b32_e64 v{inv}, 1.0, v{inv}, vcc", VALU, rd=vr(inv) + [("vcc", 0)], wr=vr(inv)),
                    Inst(f"v_mov_b32_e32 v{t + 3}, 0x7f800000", VALU, wr=vr(t + 3)),
                    Inst(f"v_cndmask_b32_e32 v{lse}, v{t + 3}, v{lse}, vcc", VALU, rd=vr(lse) + vr(t + 3) + [("vcc", 0)], wr=vr(lse))]
            if OPT_DEFER:
                ins.append(Inst(f"v_mov_b32_e32 v{V_LSEV[j]}, v{lse}", VALU, rd=vr(lse), wr=vr(V_LSEV[j])))
            else:
                ins.append(Inst(f"buffer_store_dword v{lse}, v{V_LSEOFF[j]}, s[{S_LD}:{S_LD + 3}], 0 offen", VSTORE,
                                rd=vr(lse) + vr(V_LSEOFF[j]) + sr(S_LD, 4)))
            if OPT_EPISTAMP:
                ins += self.stamp_point(6)
            for dt in range(NP):
                for u in (0, 2):
                    w = PKR(j, dt, u) if OPT_DEFER else t + 4 + 4 * ((dt * 2 + u // 2) % 4)
                    o = O_(j, dt) + 4 * u
                    x = t + 20
                    if OPT_EPI_ABL != "storeonly":
                        ins += [Inst(f"v_accvgpr_read_b32 v{x + k}, a{o + k}", ACCR, rd=ar(o + k), wr=vr(x + k)) for k in range(8)]
                        ins += [Inst(f"v_mul_f32_e32 v{x + k}, v{x + k}, v{inv}", VALU, rd=vr(x + k) + vr(inv), wr=vr(x + k)) for k in range(8)]
                        ins += [self.cvt(w + 0, x + 0, x + 1), self.cvt(w + 1, x + 2, x + 3),
                                self.cvt(w + 2, x + 4, x + 5), self.cvt(w + 3, x + 6, x + 7)]
                        ins += [Inst(f"v_permlane32_swap_b32_e32 v{w}, v{w + 2}", PERM, rd=vr(w) + vr(w + 2), wr=vr(w) + vr(w + 2)),
                                Inst(f"v_permlane32_swap_b32_e32 v{w + 1}, v{w + 3}", PERM, rd=vr(w + 1) + vr(w + 3), wr=vr(w + 1) + vr(w + 3))]
                    if OPT_EPI_ABL == "orows":   # timing ablation (wrong placement): 4 whole rows per store
                        Ro = self.kargs()["Ro"]
                        i = 2 * dt + u // 2
                        if i == 0:
                            ins += [Inst(f"v_and_b32_e32 v28, 0xffffffe0, v{V_ROW[j]}", VALU, rd=vr(V_ROW[j]), wr=vr(28)),
                                    Inst(f"v_lshrrev_b32_e32 v29, 4, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(29)),
                                    Inst("v_add_u32_e32 v28, v28, v29", VALU, rd=vr(28) + vr(29), wr=vr(28)),
                                    Inst(f"v_mul_lo_u32 v28, v28, s{Ro}", VALU, rd=vr(28) + sr(Ro), wr=vr(28)),
                                    Inst(f"v_and_b32_e32 v29, 15, v{V_LANE}", VALU, rd=vr(V_LANE), wr=vr(29)),
                                    Inst("v_lshl_add_u32 v28, v29, 4, v28", VALU, rd=vr(28) + vr(29), wr=vr(28))]
                        ins += [Inst(f"s_mul_i32 s{S_TMP + 2}, s{Ro}, {4 * i}", SALU, rd=sr(Ro), wr=sr(S_TMP + 2)),
                                Inst(f"v_add_u32_e32 v30, s{S_TMP + 2}, v28", VALU, rd=sr(S_TMP + 2) + vr(28), wr=vr(30)),
                                Inst(f"buffer_store_dwordx4 v[{w}:{w + 3}], v30, s[{S_OD}:{S_OD + 3}], 0 offen",
                                     VSTORE, rd=vr(w, 4) + vr(30) + sr(S_OD, 4))]
                    elif OPT_EPI_ABL != "nostore" and not OPT_DEFER:
                        ins.append(Inst(f"buffer_store_dwordx4 v[{w}:{w + 3}], v{V_OOFF[j]}, s[{S_OD}:{S_OD + 3}], 0 offen offset:{64 * dt + 16 * u}{OPT_OPOL}",
                                        VSTORE, rd=vr(w, 4) + vr(V_OOFF[j]) + sr(S_OD, 4)))
            if OPT_EPISTAMP and j == 0:
                ins += self.stamp_point(9)
        return ins

    def epilogue2(self):
        """the epilogue with its 2 NP x 2 groups (q-block, d-tile, column half) in two batches whose
        stages (AGPR reads, 1 / l scaling, packs, lane-half swaps, stores) are interleaved across the
        groups, so no instruction waits on its predecessor (registers: the score / pack VGPRs, free
        after the last step)"""
        ins = []
        inv = (140, 141)       # 1 / l per q-block (the LSE math uses 142.. as temporaries)
        for j in range(2):
            l, lse, tt = V_L[j], 142, 143
            ins += self.half_sum(l, tt)
            ins += [Inst(f"v_rcp_f32_e32 v{inv[j]}, v{l}", TRANS, rd=vr(l), wr=vr(inv[j])),
                    Inst(f"v_log_f32_e32 v{lse}, v{l}", TRANS, rd=vr(l), wr=vr(lse)),
                    Inst(f"v_sub_f32_e32 v{lse}, v{lse}, v{V_NEGMC[j]}", VALU, rd=vr(lse) + vr(V_NEGMC[j]), wr=vr(lse)),
                    Inst(f"v_mul_f32_e32 v{lse}, 0x3f317218, v{lse}", VALU, rd=vr(lse), wr=vr(lse)),
                    Inst(f"v_cmp_neq_f32_e32 vcc, 0, v{l}", VALU, rd=vr(l), wr=[("vcc", 0)]),
                    Inst(f"v_cmp_eq_f32_e64 s[{S_TMP}:{S_TMP + 1}], v{l}, v{l}", VALU, rd=vr(l), wr=sr(S_TMP, 2)),
                    Inst(f"s_and_b64 vcc, vcc, s[{S_TMP}:{S_TMP + 1}]", SALU, rd=sr(S_TMP, 2) + [("vcc", 0)], wr=[("vcc", 0)]),
                    Inst(f"v_cndmask_b32_e64 v{inv[j]}, 1.0, v{inv[j]}, vcc", VALU, rd=vr(inv[j]) + [("vcc", 0)], wr=vr(inv[j])),
                    Inst(f"v_mov_b32_e32 v{tt}, 0x7f800000", VALU, wr=vr(tt)),
                    Inst(f"v_cndmask_b32_e32 v{lse}, v{tt}, v{lse}, vcc", VALU, rd=vr(lse) + vr(tt) + [("vcc", 0)], wr=vr(lse)),
                    Inst(f"buffer_store_dword v{lse}, v{V_LSEOFF[j]}, s[{S_LD}:{S_LD + 3}], 0 offen", VSTORE,
                         rd=vr(lse) + vr(V_LSEOFF[j]) + sr(S_LD, 4))]
        groups = [(j, dt, u) for j in range(2) for dt in range(NP) for u in (0, 2)]
        nb = 8
        for b0 in range(0, len(groups), nb):
            stage = {k: [] for k in range(5)}
            for gi, (j, dt, u) in enumerate(groups[b0:b0 + nb]):
                x, w = 12 * gi, 12 * gi + 8
                o = O_(j, dt) + 4 * u
                stage[0] += [Inst(f"v_accvgpr_read_b32 v{x + k}, a{o + k}", ACCR, rd=ar(o + k), wr=vr(x + k)) for k in range(8)]
                stage[1] += [Inst(f"v_mul_f32_e32 v{x + k}, v{x + k}, v{inv[j]}", VALU, rd=vr(x + k) + vr(inv[j]), wr=vr(x + k))
                             for k in range(8)]
                stage[2] += [self.cvt(w + 0, x + 0, x + 1), self.cvt(w + 1, x + 2, x + 3),
                             self.cvt(w + 2, x + 4, x + 5), self.cvt(w + 3, x + 6, x + 7)]
                stage[3] += [Inst(f"v_permlane32_swap_b32_e32 v{w}, v{w + 2}", PERM, rd=vr(w) + vr(w + 2), wr=vr(w) + vr(w + 2)),
                             Inst(f"v_permlane32_swap_b32_e32 v{w + 1}, v{w + 3}", PERM, rd=vr(w + 1) + vr(w + 3), wr=vr(w + 1) + vr(w + 3))]
                stage[4].append(Inst(f"buffer_store_dwordx4 v[{w}:{w + 3}], v{V_OOFF[j]}, s[{S_OD}:{S_OD + 3}], 0 offen offset:{64 * dt + 16 * u}",
                                     VSTORE, rd=vr(w, 4) + vr(V_OOFF[j]) + sr(S_OD, 4)))
            for k in range(5):
                ins += stage[k]
        return ins

    # ------------------------------------------------------------------ whole kernel
    def build(self):
        self.switches = []
        self.refit_regs = {}
        l_end = self.lab("end")
        self.l_tile0w = self.lab("tile0w")
        self.l_empty = self.lab("empty")
        self.lab_end = l_end
        l_epi = self.lab("epi")
        L = {k: self.lab(k) for k in ("fast0", "fast1", "sel0", "sel1", "masked0", "masked1", "last0", "last1",
                                      "cold", "coldw", "warm", "skip", "tile0", "diag0", "diag1", "dead0", "dead1")}
        code = []

        def emit_block(insts, pre=()):
            out, _ = add_waits(insts)
            out, nops = fix_hazards(out, pre=pre)
            code.extend(out)
            return out

        tailpad = [nop(15)]   # block entries: every predecessor ends with a barrier / branch; pad anyway
        code += [nop(0) for _ in range(OPT_SHIFT)]
        emit_block(self.entry())
        emit_block(self.item_start(L["cold"], L["coldw"], L["warm"], L["skip"], L["tile0"], l_epi, l_end), pre=tailpad)
        if OPT_DEFER:
            code.append(label(self.l_tile0w))
            emit_block(self.tile0(L["last0"], L["fast0"], L["sel0"], stores=True), pre=tailpad)
        code.append(label(L["tile0"]))
        emit_block(self.tile0(L["last0"], L["fast0"], L["sel0"]), pre=tailpad)
        refits = []
        f0, r = self.step(0, "fast", "f0"); refits += r
        f1, r = self.step(1, "fast", "f1"); refits += r
        m0, r = self.step(0, "masked", "m0"); refits += r
        m1, r = self.step(1, "masked", "m1"); refits += r
        la0, r = self.step(0, "last", "l0"); refits += r
        la1, r = self.step(1, "last", "l1"); refits += r
        if self.causal:
            dg0, r = self.step(0, "diag", "g0"); refits += r
            dg1, r = self.step(1, "diag", "g1"); refits += r
            dd0, r = self.step(0, "dead", "d0"); refits += r
            dd1, r = self.step(1, "dead", "d1"); refits += r
        I = Inst

        def select(par):
            """causal: the step's S(n+1) tile t = n + 1, not the item's last (n + 1 < NL1) ->
            u = S_WD - t: >= 1 visible (fast body), 0 diagonal, < 0 above the diagonal"""
            if not self.causal or OPT_NODIAG:
                return []
            t = S_SWT
            return [I(f"s_add_u32 s{t}, s{S_N}, 1", SALU),
                    I(f"s_cmp_ge_u32 s{t}, s{S_NL1}", SALU), I(f"s_cbranch_scc1 {L['masked%d' % par]}", BRANCH),
                    I(f"s_sub_i32 s{t}, s{S_WD}, s{t}", SALU),
                    I(f"s_cmp_gt_i32 s{t}, 0", SALU), I(f"s_cbranch_scc1 {L['fast%d' % par]}", BRANCH),
                    I(f"s_cmp_eq_u32 s{t}, 0", SALU), I(f"s_cbranch_scc1 {L['diag%d' % par]}", BRANCH),
                    I(f"s_branch {L['dead%d' % par]}", BRANCH)]
        code.append(label(L["fast0"]))
        emit_block(f0 + self.dump("f0_end"), pre=tailpad)
        code += [I(f"s_cmp_gt_i32 s{S_N}, s{S_NF2}", SALU), I(f"s_cbranch_scc1 {L['sel1']}", BRANCH)]
        code.append(label(L["fast1"]))
        emit_block(f1, pre=tailpad)
        code += [I(f"s_cmp_le_i32 s{S_N}, s{S_NF2}", SALU), I(f"s_cbranch_scc1 {L['fast0']}", BRANCH)]
        code.append(label(L["sel0"]))
        code += [I(f"s_cmp_eq_u32 s{S_N}, s{S_NL1}", SALU), I(f"s_cbranch_scc1 {L['last0']}", BRANCH)]
        code += select(0)
        code.append(label(L["masked0"]))
        emit_block(m0 + self.dump("m0_end"), pre=tailpad)
        code.append(label(L["sel1"]))
        code += [I(f"s_cmp_eq_u32 s{S_N}, s{S_NL1}", SALU), I(f"s_cbranch_scc1 {L['last1']}", BRANCH)]
        code += select(1)
        code.append(label(L["masked1"]))
        emit_block(m1, pre=tailpad)
        code += [I(f"s_branch {L['sel0']}", BRANCH)]
        code.append(label(L["last0"]))
        emit_block(self.stamp_point(0) + la0 + self.dump("l0_end"), pre=tailpad)
        code += [I(f"s_branch {l_epi}", BRANCH)]
        if self.causal:
            for par, body in ((0, dg0), (1, dg1)):
                code.append(label(L["diag%d" % par]))
                emit_block(body, pre=tailpad)
                code += [I(f"s_branch {L['sel%d' % (1 - par)]}", BRANCH)]
            for par, body in ((0, dd0), (1, dd1)):
                code.append(label(L["dead%d" % par]))
                emit_block(body, pre=tailpad)
                code += [I(f"s_branch {L['sel%d' % (1 - par)]}", BRANCH)]
        code.append(label(L["last1"]))
        emit_block(self.stamp_point(0) + la1, pre=tailpad)
        code.append(label(l_epi))
        emit_block([nop(15)] + self.stamp_point(7) + self.epilogue() + self.stamp_point(8), pre=tailpad)
        # next item of this workgroup: warm when the DMA stream already runs into it
        code += [I(f"s_add_u32 s{S_ROUND}, s{S_ROUND}, 1", SALU),
                 I(f"s_cmp_eq_u32 s{S_WARM}, 1", SALU), I(f"s_cbranch_scc1 {L['warm']}", BRANCH),
                 I(f"s_branch {L['coldw']}", BRANCH)]
        code.append(label(l_end))
        if OPT_STAMP:
            T0 = S_TMP
            st = [I("s_waitcnt vmcnt(0) lgkmcnt(0)", WAIT),
                  I(f"s_memtime s[{T0}:{T0 + 1}]", SMEM), I(f"s_memrealtime s[{T0 + 2}:{T0 + 3}]", SMEM),
                  I("s_load_dwordx2 s[52:53], s[0:1], 0x48", SMEM),
                  I("s_getreg_b32 s44, hwreg(HW_REG_HW_ID)", SALU), I("s_getreg_b32 s45, hwreg(HW_REG_XCC_ID)", SALU),
                  I("s_waitcnt lgkmcnt(0)", WAIT)]
            st += [I(f"v_mov_b32_e32 v{i}, s{T0 + i}", VALU) for i in range(4)]
            st += [I("v_mov_b32_e32 v4, s44", VALU), I("v_mov_b32_e32 v5, s45", VALU),
                   I("v_mov_b32_e32 v6, s2", VALU), I(f"v_mov_b32_e32 v7, s{S_WAVE}", VALU),
                   I("s_cmp_eq_u64 s[52:53], 0", SALU), I("s_cselect_b32 s54, 0, 0x7fffffff", SALU),
                   I("s_mov_b32 s55, 0x20000", SALU), I("s_and_b32 s53, s53, 0xffff", SALU),
                   I("s_lshl_b32 s46, s2, 2", SALU), I(f"s_add_u32 s46, s46, s{S_WAVE}", SALU),
                   I("s_lshl_b32 s46, s46, 7", SALU),
                   I("v_mov_b32_e32 v8, 0", VALU), nop(4)]
            st += [I(f"buffer_store_dwordx4 v[{V_STAMP}:{V_STAMP + 3}], v8, s[52:55], s46 offen", VSTORE),
                   I("buffer_store_dwordx4 v[0:3], v8, s[52:55], s46 offen offset:16", VSTORE),
                   I(f"buffer_store_dwordx2 v[{V_STAMP + 4}:{V_STAMP + 5}], v8, s[52:55], s46 offen offset:32", VSTORE),
                   I("buffer_store_dwordx4 v[4:7], v8, s[52:55], s46 offen offset:48", VSTORE),
                   I(f"buffer_store_dwordx4 v[{V_SSUM}:{V_SSUM + 3}], v8, s[52:55], s46 offen offset:64", VSTORE),
                   I(f"buffer_store_dwordx4 v[{V_SSUM + 6}:{V_SSUM + 9}], v8, s[52:55], s46 offen offset:80", VSTORE),
                   I(f"buffer_store_dword v{V_SSUM + 5}, v8, s[52:55], s46 offen offset:96", VSTORE),
                   I("s_waitcnt vmcnt(0)", WAIT)]
            code.extend(st)
        code.append(I("s_endpgm", SOPP))
        for rb in refits:
            code.extend(rb)
        for sb in self.switches:
            emit_block(sb, pre=tailpad)
        return code

    def render(self):
        code = self.build()
        out = []
        out.append(f"\t.globl {self.name}")
        out.append("\t.p2align 8")
        out.append(f"\t.type {self.name},@function")
        out.append(f"{self.name}:")
        nm = 0
        for ins in code:
            if ins.kind == LABEL:
                if OPT_ALIGN and any(f"_{k}" in ins.text for k in ("fast0_", "fast1_", "masked0_", "masked1_",
                                                                     "diag0_", "diag1_", "dead0_", "dead1_")):
                    out.append(f"\t.p2align {OPT_ALIGN}")
                out.append(ins.text)
            else:
                out.append("\t" + ins.text)
                nm += ins.kind == MFMA
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
    out = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 5", "\t.text"]
    meta = []
    for d in (128, 64):
        configure(d)
        for k in [K(bf, ca) for bf in (True, False) for ca in (True, False)]:
            out.append(k.render())
            out.append(k.descriptor())
            meta.append(k.metadata().rstrip("\n"))
    out.append("\t.amdgpu_metadata\n---\namdhsa.kernels:")
    out += meta
    out.append("amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata")
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
