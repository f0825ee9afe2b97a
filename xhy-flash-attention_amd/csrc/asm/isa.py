"""Instruction model, hazard verifier and counter bookkeeping for hand-scheduled gfx950 code.

Used by gen_fwd.py to emit the assembly forward kernel.  Every instruction carries the registers it
reads and writes; the verifier walks the final instruction order and inserts the wait states gfx950
requires between dependent instructions (the rules below are the ones LLVM's hazard recognizer
applies for gfx950, confirmed by compiling probe kernels with hipcc: VALU write -> MFMA read 2,
8-pass XDL write -> VALU read 12 (`s_nop 11`), transcendental -> VALU use 1, VALU write ->
v_permlane read 2, VALU write -> v_readfirstlane read 1, SALU M0 write -> LDS-DMA 1, VALU SGPR
write -> VMEM read 5).  The v_readfirstlane rule was learnt the hard way: without it the wave index
was read stale on hardware, which misplaced every LDS-DMA piece (tools/probe_gen.py, asm_dump.py).  The counter pass
inserts `s_waitcnt lgkmcnt(N)` / `vmcnt(N)` before the first reader of a register that a still
outstanding LDS or VMEM load writes, counted (only the loads that have to land are waited for).
"""
import os

# instruction kinds
MFMA, VALU, TRANS, PERM, ACCR, ACCW, SALU, SMEM, LDS, DMA, VLOAD, VSTORE, WAIT, NOP, BRANCH, LABEL, \
    BARRIER, SOPP, RFL = range(19)
VALU_LIKE = (VALU, TRANS, PERM, ACCR, ACCW, RFL)

# issue cost in cycles (one wave alone on its SIMD; MI355X_MICROARCH.md per-instruction constants)
COST = {MFMA: 8, VALU: 4, TRANS: 8, PERM: 4, ACCR: 4, ACCW: 4, SALU: 2, SMEM: 2, LDS: 2, DMA: 8,
        VLOAD: 4, VSTORE: 4, WAIT: 1, NOP: 4, BRANCH: 2, LABEL: 0, BARRIER: 4, SOPP: 2, RFL: 4}
COST_LDS128 = None      # (LDS128=n) a separate weight for ds_read_b128


def apply_costs(spec):
    """scheduling weights, e.g. "LDS=5,SALU=3": each generator applies its defaults, then
    FA_ISA_COST and its own FA_G*_COST (dev A/B, tools/asm_variant.sh).  The gap scheduler fills a
    gap while the weights fit the budget, so a heavier LDS weight spreads the reads over more gaps."""
    global COST_LDS128
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        if k == "LDS128":
            COST_LDS128 = int(v)
            continue
        COST[{"TRANS": TRANS, "VALU": VALU, "LDS": LDS, "SALU": SALU, "DMA": DMA, "PERM": PERM}[k]] = int(v)


def vr(i, n=1):
    return [("v", i + k) for k in range(n)]


def ar(i, n=1):
    return [("a", i + k) for k in range(n)]


def sr(i, n=1):
    return [("s", i + k) for k in range(n)]


def rtxt(kind, i, n=1):
    return f"{kind}{i}" if n == 1 else f"{kind}[{i}:{i + n - 1}]"


class Inst:
    __slots__ = ("text", "kind", "rd", "wr", "rd_c", "key", "dl", "eg", "cost", "deps", "name")

    def __init__(self, text, kind, rd=(), wr=(), rd_c=(), key=0, deadline=None, earliest=None,
                 deps=(), name=None):
        self.text = text
        self.kind = kind
        self.rd = frozenset(rd)
        self.wr = frozenset(wr)
        self.rd_c = frozenset(rd_c)   # MFMA SrcC registers (subset of rd)
        self.key = key                # scheduling priority (lower first)
        self.dl = deadline            # must be emitted before MFMA number dl of its phase
        self.eg = earliest            # may not be emitted before gap eg (after MFMA eg)
        self.cost = COST[kind]
        if COST_LDS128 is not None and kind == LDS and text.startswith("ds_read_b128"):
            self.cost = COST_LDS128
        self.deps = list(deps)        # filler ops that must precede this one
        self.name = name

    def ws(self):
        """wait states this instruction provides to later ones"""
        if self.kind == NOP:
            return int(self.text.split()[1]) + 1
        if self.kind == LABEL:
            return 0
        return 1

    def __repr__(self):
        return self.text


def nop(n):
    return Inst(f"s_nop {n}", NOP)


def label(name):
    return Inst(f"{name}:", LABEL)


# ------------------------------------------------------------------------------------------------
# hazards
# ------------------------------------------------------------------------------------------------
XDL_RAW = 12      # 8-pass XDL (v_mfma_f32_32x32x16_*) write -> any non-chain access
VALU_MFMA = 2     # VALU / v_accvgpr_write write -> MFMA read
TRANS_USE = 1
VALU_PERM = 2
VALU_RFL = 1      # VALU write -> v_readfirstlane / v_readlane read of that VGPR
M0_DMA = 1
VSGPR_VMEM = 5
STORE_WAR = 2     # buffer_store_dwordx4 data -> VALU overwrite
MFMA_LDS_WAR = 4  # MFMA reading A/B -> LDS / VMEM load overwriting them (conservative)


def required(prev, cur):
    """wait states `cur` needs after `prev` (0 if independent)"""
    need = 0
    if prev.kind == MFMA:
        touched = (cur.rd | cur.wr) & prev.wr
        if touched:
            if cur.kind == MFMA and prev.wr == cur.wr and cur.rd_c == cur.wr and not (cur.rd - cur.rd_c) & prev.wr:
                pass   # accumulation chain: same D, previous D read whole as C
            else:
                need = max(need, XDL_RAW)
        if cur.kind != MFMA and cur.wr & (prev.rd_c - prev.wr):
            need = max(need, XDL_RAW)   # WAR on SrcC (conservative)
        if cur.kind in (LDS, VLOAD) and cur.wr & (prev.rd - prev.rd_c):
            need = max(need, MFMA_LDS_WAR)
    if prev.kind in VALU_LIKE and cur.kind == MFMA and prev.wr & cur.rd:
        need = max(need, VALU_MFMA)
    if prev.kind == TRANS and cur.kind in VALU_LIKE and prev.wr & cur.rd:
        need = max(need, TRANS_USE)
    if prev.kind in VALU_LIKE and cur.kind == PERM and prev.wr & cur.rd:
        need = max(need, VALU_PERM)
    if prev.kind in VALU_LIKE and cur.kind == RFL and prev.wr & cur.rd:
        need = max(need, VALU_RFL)
    if prev.kind == SALU and ("m0", 0) in prev.wr and cur.kind == DMA:
        need = max(need, M0_DMA)
    if prev.kind in VALU_LIKE and cur.kind in (DMA, VLOAD, VSTORE, SMEM):
        if any(r[0] == "s" for r in prev.wr & cur.rd):
            need = max(need, VSGPR_VMEM)
    if prev.kind == VSTORE and cur.kind in VALU_LIKE and cur.wr & prev.rd:
        need = max(need, STORE_WAR)
    return need


WINDOW = 24


def violation(hist, cur):
    """(needed extra wait states) for placing `cur` after the instruction list `hist`"""
    have = 0
    worst = 0
    for prev in reversed(hist[-WINDOW:]):
        if prev.kind == LABEL:
            continue
        need = required(prev, cur)
        if need > have:
            worst = max(worst, need - have)
        have += prev.ws()
        if have >= XDL_RAW:
            break
    return worst


def fix_hazards(insts, pre=()):
    """insert s_nop where `insts` (preceded by the instructions `pre`) violates a rule"""
    out = []
    hist = list(pre)
    nops = 0
    for ins in insts:
        if ins.kind != LABEL:
            v = violation(hist, ins)
            while v > 0:
                n = min(v, 16) - 1
                nn = nop(n)
                out.append(nn)
                hist.append(nn)
                nops += n + 1
                v = violation(hist, ins)
        out.append(ins)
        hist.append(ins)
    return out, nops


# ------------------------------------------------------------------------------------------------
# counters
# ------------------------------------------------------------------------------------------------
class Counters:
    """outstanding LDS reads (lgkmcnt) and VMEM operations (vmcnt), in issue order"""

    def __init__(self):
        self.lds = []    # list of register sets written
        self.vm = []

    def waits_for(self, ins):
        """the s_waitcnt to emit before `ins` (or None), updating the outstanding lists"""
        need_l = None
        for i, w in enumerate(self.lds):
            if w & (ins.rd | ins.wr):
                need_l = i
        need_v = None
        for i, w in enumerate(self.vm):
            if w & (ins.rd | ins.wr):
                need_v = i
        parts = []
        if need_l is not None:
            k = len(self.lds) - 1 - need_l
            parts.append(f"lgkmcnt({min(k, 15)})")
            self.lds = self.lds[need_l + 1:] if k <= 15 else self.lds[len(self.lds) - 15:]
        if need_v is not None:
            k = len(self.vm) - 1 - need_v
            parts.append(f"vmcnt({min(k, 63)})")
            self.vm = self.vm[need_v + 1:] if k <= 63 else self.vm[len(self.vm) - 63:]
        return Inst("s_waitcnt " + " ".join(parts), WAIT) if parts else None

    def issue(self, ins):
        if ins.kind == LDS:
            self.lds.append(ins.wr)
        elif ins.kind in (DMA, VLOAD, VSTORE):
            self.vm.append(ins.wr if ins.kind == VLOAD else frozenset())
        elif ins.kind == SMEM:
            self.lds.append(ins.wr)
        elif ins.kind == WAIT:
            t = ins.text
            if "lgkmcnt(" in t:
                k = int(t.split("lgkmcnt(")[1].split(")")[0])
                self.lds = self.lds[len(self.lds) - k:] if k else []
            if "vmcnt(" in t:
                k = int(t.split("vmcnt(")[1].split(")")[0])
                self.vm = self.vm[len(self.vm) - k:] if k else []


def add_waits(insts, ctr=None):
    """insert counted waits before the readers of outstanding loads"""
    ctr = ctr or Counters()
    out = []
    for ins in insts:
        if ins.kind not in (LABEL, WAIT):
            w = ctr.waits_for(ins)
            if w is not None:
                out.append(w)
        ctr.issue(ins)
        out.append(ins)
    return out, ctr


# ------------------------------------------------------------------------------------------------
# gap scheduler: fixed MFMA sequence, filler ops placed into the gaps between them
# ------------------------------------------------------------------------------------------------
def schedule(mfmas, fillers, budget=24, pre=(), tail_budget=None, lat=None):
    """Place `fillers` (Inst with deps / key / earliest / deadline) into the gaps of `mfmas`.

    Gap g follows MFMA g (gap -1 precedes the first MFMA).  Per gap, fillers are added in priority
    order while their issue cost fits `budget` cycles; an op is eligible once its deps are placed and
    placing it needs no wait states (checked against the instructions already emitted).  Ops whose
    deadline is the next MFMA are forced in.  What is left after the last MFMA is appended.

    lat (optional): result latencies {kind: cycles}.  The scheduler then keeps an issue-time estimate
    (fillers at their issue cost, MFMAs paced 32 cycles apart) and a ready time per register; among
    the eligible fillers of a gap it takes, in priority order, the first whose operands are ready, and
    only when none is, the one that stalls least (the stall counts against the gap's budget).
    """
    out = []
    hist = list(pre)
    placed = set()
    # data dependencies in list (program) order: RAW, WAR and WAW on every register, incl. vcc / scc / m0
    for i, op in enumerate(fillers):
        for prev in fillers[:i]:
            if (op.rd & prev.wr) or (op.wr & (prev.rd | prev.wr)):
                if prev not in op.deps:
                    op.deps.append(prev)
    remaining = list(fillers)
    remaining.sort(key=lambda x: x.key)

    clk = [0, -32]          # issue-time estimate, start of the last MFMA
    ready = {}

    def stall(op):
        if lat is None:
            return 0
        return max([0] + [ready.get(r, 0) - clk[0] for r in op.rd])

    def account(op):
        if lat is None:
            return
        start = clk[0] + stall(op)
        if op.kind == MFMA:
            start = max(start, clk[1] + 32)
            clk[1] = start
        clk[0] = start + op.cost
        lt = lat.get(op.kind)
        if lt is not None:
            for r in op.wr:
                ready[r] = start + lt

    def eligible(op, g, force=False):
        if any(id(d) not in placed for d in op.deps):
            return False
        if op.eg is not None and g < op.eg and not force:
            return False
        if not force and violation(hist, op) > 0:
            return False
        return True

    def emit(op):
        account(op)
        out.append(op)
        hist.append(op)
        placed.add(id(op))

    def ready_ancestor(op, seen):
        """an unplaced op in op's dependency cone (op included) whose own deps are all placed"""
        if id(op) in seen:
            return None
        seen.add(id(op))
        for d in op.deps:
            if id(d) not in placed:
                r = ready_ancestor(d, seen)
                if r is not None:
                    return r
        return op if all(id(d) in placed for d in op.deps) else None

    def fill(g, cap, nxt):
        used = 0
        while True:
            # forced: deadline before the next MFMA (its unplaced dependency cone first)
            forced = [op for op in remaining if op.dl is not None and op.dl <= nxt]
            progress = False
            if forced:
                op = ready_ancestor(forced[0], set())
                if op is None:
                    raise RuntimeError(f"scheduler: cannot place {forced[0]}")
                remaining.remove(op)
                emit(op)
                used += op.cost
                continue
            if cap is not None and used >= cap:
                break
            best = None
            for op in remaining:
                if cap is not None and used + op.cost > cap and used > 0:
                    continue
                if eligible(op, g):
                    st = stall(op)
                    if best is None or st < best[0]:
                        best = (st, op)
                    if st == 0:
                        break
            if best is not None:
                st, op = best
                if cap is not None and st and used + st + op.cost > cap and used > 0:
                    break
                remaining.remove(op)
                emit(op)
                used += op.cost + st
                progress = True
            if not progress:
                break

    n = len(mfmas)
    fill(-1, budget if n else None, 0)
    for g, m in enumerate(mfmas):
        late = [op for op in remaining if op.dl is not None and op.dl <= g]
        if late:
            raise RuntimeError(f"scheduler: {late[0]} missed its deadline (MFMA {late[0].dl})")
        emit(m)
        fill(g, budget if g + 1 < n else tail_budget, g + 1 if g + 1 < n else 10 ** 9)
    # flush (hazard-checked placement happens in fix_hazards)
    while remaining:
        progress = False
        for op in list(remaining):
            if all(id(d) in placed for d in op.deps):
                remaining.remove(op)
                emit(op)
                progress = True
                break
        if not progress:
            raise RuntimeError("scheduler: dependency cycle among " + ", ".join(map(str, remaining[:5])))
    return out


# ------------------------------------------------------------------------------------------------
# work-order decode (fa_params.h ItemDecode): item index -> (block, batch, head, kv head), in SALU
# ------------------------------------------------------------------------------------------------
def item_decode_ops(L, M, pa, pb, t, u, o_blk, reverse):
    """SALU ops computing, from the item index in s[L] and the ItemDecode dwords in s[M..M+9]
    (mag PG HP H G, div PG HP H G, shifts, xs | (nblk - 1) << 8):
        i = L >> xs;  gi = i / PG, r = i - gi PG;  blk = r / HP, hr = r - blk HP
        bh = ((gi HP + hr) << xs) + (L & (2^xs - 1));  bidb = bh / H, head = bh - bidb H;  kvh = head / G
    Each q = n / d is s_mul_i32 / s_mul_hi_u32 by the magic number and one s_lshr_b64 by its shift.
    pa, pb: even-aligned SGPR pairs, t, u: SGPRs (temporaries); s[o_blk] gets nblk - 1 - blk
    (reverse) or blk and must not be one of pa, pb, t, u, L, M.  Results: bidb in s[pb], head in s[u],
    kvh in s[pa]."""
    a0, a1 = pa, pa + 1
    b0, b1 = pb, pb + 1
    mPG, mHP, mH, mG, dPG, dHP, dH, dG, SH, XN = (M + i for i in range(10))
    I = Inst
    ops = [I(f"s_and_b32 s{t}, s{XN}, 0xff", SALU),                           # xs
           I(f"s_lshr_b32 s{u}, s{L}, s{t}", SALU),                           # i
           I(f"s_mul_i32 s{a0}, s{u}, s{mPG}", SALU), I(f"s_mul_hi_u32 s{a1}, s{u}, s{mPG}", SALU),
           I(f"s_lshr_b64 s[{a0}:{a1}], s[{a0}:{a1}], s{SH}", SALU),          # gi
           I(f"s_mul_i32 s{a1}, s{a0}, s{dPG}", SALU), I(f"s_sub_u32 s{u}, s{u}, s{a1}", SALU),   # r
           I(f"s_mul_i32 s{a0}, s{a0}, s{dHP}", SALU),                        # gi HP
           I(f"s_lshr_b32 s{a1}, s{SH}, 8", SALU),
           I(f"s_mul_i32 s{b0}, s{u}, s{mHP}", SALU), I(f"s_mul_hi_u32 s{b1}, s{u}, s{mHP}", SALU),
           I(f"s_lshr_b64 s[{b0}:{b1}], s[{b0}:{b1}], s{a1}", SALU),          # blk
           I(f"s_mul_i32 s{a1}, s{b0}, s{dHP}", SALU), I(f"s_sub_u32 s{u}, s{u}, s{a1}", SALU),   # hr
           I(f"s_add_u32 s{a0}, s{a0}, s{u}", SALU),                          # hl
           I(f"s_lshl_b32 s{a0}, s{a0}, s{t}", SALU),
           I(f"s_lshl_b32 s{u}, 1, s{t}", SALU), I(f"s_sub_u32 s{u}, s{u}, 1", SALU),
           I(f"s_and_b32 s{u}, s{L}, s{u}", SALU), I(f"s_add_u32 s{a0}, s{a0}, s{u}", SALU)]  # bh
    if reverse:
        ops += [I(f"s_lshr_b32 s{o_blk}, s{XN}, 8", SALU), I(f"s_sub_u32 s{o_blk}, s{o_blk}, s{b0}", SALU)]
    else:
        ops += [I(f"s_mov_b32 s{o_blk}, s{b0}", SALU)]
    ops += [I(f"s_lshr_b32 s{t}, s{SH}, 16", SALU),
            I(f"s_mul_i32 s{b0}, s{a0}, s{mH}", SALU), I(f"s_mul_hi_u32 s{b1}, s{a0}, s{mH}", SALU),
            I(f"s_lshr_b64 s[{b0}:{b1}], s[{b0}:{b1}], s{t}", SALU),          # bidb
            I(f"s_mul_i32 s{u}, s{b0}, s{dH}", SALU), I(f"s_sub_u32 s{u}, s{a0}, s{u}", SALU),     # head
            I(f"s_lshr_b32 s{t}, s{SH}, 24", SALU),
            I(f"s_mul_i32 s{a0}, s{u}, s{mG}", SALU), I(f"s_mul_hi_u32 s{a1}, s{u}, s{mG}", SALU),
            I(f"s_lshr_b64 s[{a0}:{a1}], s[{a0}:{a1}], s{t}", SALU)]          # kvh
    return ops


def item_decode_ref(L, dec):
    """Python restatement of item_decode_ops (tests): dec = the 10 ItemDecode dwords"""
    mag, dv, sh, xn = dec[0:4], dec[4:8], dec[8], dec[9]
    xs, nb1 = xn & 0xFF, xn >> 8

    def div(n, k):
        return ((n * mag[k]) >> ((sh >> (8 * k)) & 63)) & 0xFFFFFFFF
    i = L >> xs
    gi = div(i, 0)
    r = i - gi * dv[0]
    blk = div(r, 1)
    hr = r - blk * dv[1]
    bh = ((gi * dv[1] + hr) << xs) + (L & ((1 << xs) - 1))
    bidb = div(bh, 2)
    head = bh - bidb * dv[2]
    return blk, nb1, bidb, head, div(head, 3)


def magic_div(d):
    """fa_params.h magic_div: (mag, sh) with n / d == (n * mag) >> sh for 0 <= n < 2^31"""
    l = 0
    while (1 << l) < d:
        l += 1
    return ((1 << (31 + l)) // d + 1) & 0xFFFFFFFF, 31 + l


def make_item_decode(xs, pg, hp, h, g, nblk):
    """fa_params.h make_item_decode: the 10 ItemDecode dwords"""
    m = [magic_div(x) for x in (pg, hp, h, g)]
    return [x[0] for x in m] + [pg, hp, h, g, m[0][1] | m[1][1] << 8 | m[2][1] << 16 | m[3][1] << 24,
                                xs | (nblk - 1) << 8]


def fwd_item_decode(nbh, h, g, nblk, hp=0):
    """fa_params.h fwd_item_decode (forward / dQ order)"""
    if nbh % 8 == 0 and hp > 0 and (nbh >> 3) % hp == 0:
        return make_item_decode(3, hp * nblk, hp, h, g, nblk)
    return make_item_decode(0, 0x7FFFFFFF, nbh, h, g, nblk)


def dkdv_item_decode(nbh, h_grid, g, nblk):
    """fa_params.h dkdv_item_decode (dK / dV order)"""
    if nbh % 8 == 0:
        return make_item_decode(3, nblk, 1, h_grid, g, nblk)
    return make_item_decode(0, 0x7FFFFFFF, nbh, h_grid, g, nblk)


def item_pos_ops(dst, r, w, grid, t, u):
    """persistent item loop: s[dst] = r G + (r odd ? rev(w) : w), G = s[grid], w = s[w], r = s[r]
    (snake order over the heaviest-first item list, so each pair of rounds pairs heavy and light
    items); rev(w) = G - 8 - (w & ~7) + (w & 7) when G % 8 == 0 -- the reversal runs over groups of 8
    workgroups, so workgroup w stays on the items of the XCD it runs on (w mod 8) -- else G - 1 - w.
    t, u: temporaries (distinct from dst, r, w, grid)"""
    I = Inst
    return [I(f"s_and_b32 s{u}, s{w}, 7", SALU),
            I(f"s_lshl_b32 s{u}, s{u}, 1", SALU),
            I(f"s_sub_u32 s{t}, s{grid}, 8", SALU),
            I(f"s_sub_u32 s{t}, s{t}, s{w}", SALU),
            I(f"s_add_u32 s{t}, s{t}, s{u}", SALU),                  # G - 8 - (w & ~7) + (w & 7)
            I(f"s_sub_u32 s{u}, s{grid}, 1", SALU),
            I(f"s_sub_u32 s{u}, s{u}, s{w}", SALU),                  # G - 1 - w
            I(f"s_and_b32 s{dst}, s{grid}, 7", SALU),
            I(f"s_cmp_lg_u32 s{dst}, 0", SALU),
            I(f"s_cselect_b32 s{t}, s{u}, s{t}", SALU),              # rev(w)
            I(f"s_bitcmp1_b32 s{r}, 0", SALU),
            I(f"s_cselect_b32 s{t}, s{t}, s{w}", SALU),              # odd round: rev(w)
            I(f"s_mul_i32 s{dst}, s{r}, s{grid}", SALU),
            I(f"s_add_u32 s{dst}, s{dst}, s{t}", SALU)]
