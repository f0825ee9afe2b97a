#!/usr/bin/env python3
"""Functional CPU emulator for the gfx950 instruction subset that csrc/asm/gen_fwd.py emits (dev /
test tool, not part of the product).

It executes one kernel of a generated .s file on a flat byte heap, workgroup by workgroup, its 4
waves interleaved at every s_barrier.  Every instruction takes effect at once and in program order,
so the emulator checks the LOGIC of a hand-written kernel -- register allocation, addressing, LDS
layouts, MFMA operand layouts, the online-softmax algebra, loop control -- not its timing: counted
waits and wait states are checked statically by csrc/asm/isa.py.

Lane layouts modelled (the ones the HIP kernels rely on, fa_common.h):
  * v_mfma_f32_32x32x16_{bf16,f16}: lane l (r = l & 31, h = l >> 5) holds A[r][8h + j] and
    B[8h + j][r] (j = 0..7, two 16-bit values per dword, low half first); accumulator register g of
    lane l is D[(g & 3) + 8 (g >> 2) + 4 h][r].
  * ds_read_b64_tr_b16: in every group of 16 lanes, lane i reads 4 16-bit values D_i[0..3] at its
    address and receives out_i[q] = D_{4q + (i >> 2)}[i & 3] (a 4 x 16 block transposed).
  * v_permlane32_swap_b32 x, y: lanes 32..63 of x exchange with lanes 0..31 of y.
  * buffer_* with a raw descriptor: base = s0 | (s1 & 0xffff) << 32, num_records = s2; an access
    whose [offset, offset + size) leaves [0, num_records) reads 0 / is dropped; `lds` loads write
    16 bytes per lane at M0 + 16 lane.
"""
import os
import re
import struct

import numpy as np

HEAP_BASE = 0x10000000
LDS_SIZE = 163840
U32 = np.uint32


def f2u(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def u2f(x):
    return np.asarray(x, dtype=np.uint32).view(np.float32)


def bf16_to_f32(u16):
    return (np.asarray(u16, dtype=np.uint32) << 16).view(np.float32)


def f32_to_bf16(x):
    u = f2u(x).astype(np.uint64)
    nan = np.isnan(np.asarray(x, dtype=np.float32))
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32) & 0xFFFF
    r = np.where(nan, ((u >> 16) | 0x40).astype(np.uint32) & 0xFFFF, r)
    return r.astype(np.uint32)


def f32_to_f16(x):
    return np.asarray(x, dtype=np.float32).astype(np.float16).view(np.uint16).astype(np.uint32)


def f16_to_f32(u16):
    return np.asarray(u16, dtype=np.uint16).view(np.float16).astype(np.float32)


class Heap:
    def __init__(self, size):
        self.mem = np.zeros(size, dtype=np.uint8)
        self.top = 0

    def alloc(self, nbytes, align=256):
        self.top = (self.top + align - 1) // align * align
        a = self.top
        self.top += nbytes
        assert self.top <= self.mem.size, "heap full"
        return HEAP_BASE + a

    def put(self, arr):
        b = np.ascontiguousarray(arr).view(np.uint8).ravel()
        a = self.alloc(b.size)
        self.mem[a - HEAP_BASE:a - HEAP_BASE + b.size] = b
        return a

    def get(self, addr, nbytes):
        o = addr - HEAP_BASE
        return self.mem[o:o + nbytes]


REG = re.compile(r"^(-?)([vas])(?:\[(\d+):(\d+)\]|(\d+))$")


def parse_kernel(text, name):
    lines = text.split("\n")
    start = lines.index(f"{name}:")
    insts, labels = [], {}
    for ln in lines[start + 1:]:
        s = ln.strip()
        if s.startswith(f".L{name}_fend"):
            break
        if not s or s.startswith(";") or s.startswith("."):
            if s.endswith(":") and s.startswith(".L"):
                labels[s[:-1]] = len(insts)
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(insts)
            continue
        parts = s.split(None, 1)
        op = parts[0]
        args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
        # split trailing modifiers ("0 offen offset:64 lds", "v148 offset:8192")
        mods = {}
        clean = []
        for a in args:
            toks = a.split()
            clean.append(toks[0])
            for t in toks[1:]:
                if ":" in t:
                    k, v = t.split(":", 1)
                    mods[k] = int(v, 0)
                else:
                    mods[t] = True
        insts.append((op, clean, mods, s))
    return insts, labels


# FA_EMU_POISON=1: registers start as fp32 NaN and LDS as 0xff bytes (bf16 / f16 NaN) instead of
# zero -- a kernel that reads a register or LDS byte it never wrote then shows NaN in its outputs, as
# it may on the GPU, where that state is whatever the previous wave left
POISON = os.environ.get("FA_EMU_POISON") == "1"


class Wave:
    def __init__(self, wid, nregs=512):
        self.r = np.zeros((nregs, 64), dtype=np.uint32)   # v0..v255, a0..a255 at 256..511
        if POISON:
            self.r[:] = 0x7fc00000
        self.s = np.zeros(128, dtype=np.uint32)
        self.vcc = np.zeros(64, dtype=bool)
        self.scc = False
        self.m0 = 0
        self.pc = 0
        self.done = False
        self.at_barrier = False
        self.wid = wid
        self.vm = []        # outstanding VMEM ops in issue order: LDS-DMA writes (dst, bytes), ("reg", index, data) or None


class Emu:
    def __init__(self, text, name, heap):
        self.insts, self.labels = parse_kernel(text, name)
        self.heap = heap
        self.count = 0
        self.mfma_count = 0
        self.trace_labels = None   # substrings of labels to log (wave, label) when reached
        self.hooks = {}            # label -> fn(emu, wave) called when a wave reaches it
        self.trace = []
        self.label_at = {v: k for k, v in self.labels.items()}
        self.races = None          # check_races(): list of cross-wave LDS conflicts within a barrier interval

    # ---------------------------------------------------------------- LDS race checker
    def check_races(self, benign=()):
        """record LDS accesses per 16-byte granule and barrier interval: a wave reading (or writing)
        bytes another wave wrote, or will overwrite, between the same two barriers, or bytes an
        LDS-DMA of another wave still has in flight, is a race whatever order the hardware picks.
        benign: (lo, hi) byte ranges to ignore (e.g. bytes every wave DMAs identically)."""
        n = 163840 // 16
        self.races = []
        self.benign = [(lo // 16, (hi + 15) // 16) for lo, hi in benign]
        self.epoch = 0
        self.wr_ep = np.full(n, -1, np.int64)
        self.wr_wv = np.full(n, -1, np.int64)
        self.rd_ep = np.full(n, -1, np.int64)
        self.rd_mask = np.zeros(n, np.int64)
        self.pend = np.zeros(n, np.int64)       # bitmask of waves with an LDS-DMA in flight there

    def _grs(self, addrs, nb):
        g = set()
        for a_ in addrs:
            for x in range(int(a_) // 16, (int(a_) + nb - 1) // 16 + 1):
                g.add(x)
        return [x for x in sorted(g) if not any(lo <= x < hi for lo, hi in self.benign)]

    def _race(self, w, kind, gr):
        if len(self.races) < 50:
            op = self.insts[w.pc - 1][3] if w.pc > 0 else "?"
            self.races.append(f"epoch {self.epoch} wave {w.wid} {kind} at LDS {16 * gr}: {op}")

    def _lds_read(self, w, addrs, nb):
        if self.races is None:
            return
        bit = 1 << w.wid
        for gr in self._grs(addrs, nb):
            if self.pend[gr] & ~bit:
                self._race(w, "read of another wave's in-flight DMA", gr)
            if self.wr_ep[gr] == self.epoch and self.wr_wv[gr] != w.wid:
                self._race(w, f"read after wave {self.wr_wv[gr]}'s write", gr)
            if self.rd_ep[gr] != self.epoch:
                self.rd_ep[gr], self.rd_mask[gr] = self.epoch, 0
            self.rd_mask[gr] |= bit

    def _lds_write(self, w, addrs, nb, dma=False):
        if self.races is None:
            return
        bit = 1 << w.wid
        for gr in self._grs(addrs, nb):
            if self.rd_ep[gr] == self.epoch and self.rd_mask[gr] & ~bit:
                self._race(w, "write of bytes another wave read" + (" (DMA)" if dma else ""), gr)
            if not dma:
                if self.wr_ep[gr] == self.epoch and self.wr_wv[gr] != w.wid:
                    self._race(w, f"write after wave {self.wr_wv[gr]}'s write", gr)
                if self.pend[gr] & ~bit:
                    self._race(w, "write of another wave's in-flight DMA", gr)
                self.wr_ep[gr], self.wr_wv[gr] = self.epoch, w.wid
            else:
                self.pend[gr] |= bit

    def _dma_land(self, w, dst, nb):
        if self.races is None:
            return
        bit = 1 << w.wid
        for gr in self._grs([dst], nb):
            self.pend[gr] &= ~bit
            self.wr_ep[gr], self.wr_wv[gr] = self.epoch, w.wid

    # ---------------------------------------------------------------- operands
    def reg_index(self, tok):
        m = REG.match(tok)
        if not m:
            return None
        neg, kind, lo, hi, one = m.groups()
        if one is not None:
            lo = hi = int(one)
        else:
            lo, hi = int(lo), int(hi)
        return neg == "-", kind, lo, hi

    def vsrc(self, w, tok, flt=False):
        """64-lane uint32 value of a VALU source operand"""
        r = self.reg_index(tok)
        if r is not None:
            neg, kind, lo, hi = r
            if kind == "v":
                val = w.r[lo].copy()
            elif kind == "a":
                val = w.r[256 + lo].copy()
            else:
                val = np.full(64, w.s[lo], dtype=np.uint32)
            if neg:
                val = val ^ np.uint32(0x80000000)
            return val
        if tok == "vcc":
            raise ValueError("vcc as vsrc")
        return np.full(64, self.const(tok, flt), dtype=np.uint32)

    def const(self, tok, flt):
        if re.match(r"^-?\d+\.\d+$", tok):
            return int(f2u(np.float32(float(tok))))
        v = int(tok, 0)
        return v & 0xFFFFFFFF

    def ssrc(self, w, tok):
        r = self.reg_index(tok)
        if r is not None:
            _, kind, lo, hi = r
            assert kind == "s"
            return int(w.s[lo])
        if tok == "m0":
            return w.m0
        return self.const(tok, False)

    def ssrc64(self, w, tok):
        if tok == "vcc":
            return int(np.packbits(w.vcc[::-1]).view(">u8")[0]) if False else sum(1 << i for i in range(64) if w.vcc[i])
        _, kind, lo, hi = self.reg_index(tok)
        return int(w.s[lo]) | (int(w.s[lo + 1]) << 32)

    def vdst(self, w, tok, val):
        _, kind, lo, hi = self.reg_index(tok)
        base = 0 if kind == "v" else 256
        w.r[base + lo] = np.asarray(val, dtype=np.uint32)

    def regs(self, w, tok):
        _, kind, lo, hi = self.reg_index(tok)
        base = 0 if kind == "v" else 256
        return base + lo, hi - lo + 1

    # ---------------------------------------------------------------- memory
    def desc(self, w, tok):
        _, kind, lo, hi = self.reg_index(tok)
        s = w.s
        base = int(s[lo]) | ((int(s[lo + 1]) & 0xFFFF) << 32)
        return base, int(s[lo + 2])

    def mem_read(self, addr, n):
        return self.heap.get(addr, n)

    # ---------------------------------------------------------------- execution
    def run_wg(self, wg_id, kernarg_addr, nwaves=4, order=None):
        """order: the waves' order between two barriers (None: 0 first; "reverse": the last first --
        a read of data another wave writes in the same barrier interval then sees the other version)"""
        lds = np.full(LDS_SIZE, 0xff if POISON else 0, dtype=np.uint8)
        waves = [Wave(i) for i in range(nwaves)]
        for w in waves:
            w.s[0] = kernarg_addr & 0xFFFFFFFF
            w.s[1] = kernarg_addr >> 32
            w.s[2] = wg_id
            w.r[0] = np.arange(64, dtype=np.uint32) + 64 * w.wid
        seq = waves[::-1] if order == "reverse" else waves
        while True:
            progressed = False
            for w in seq:
                while not w.done and not w.at_barrier:
                    self.step(w, lds)
                    progressed = True
            live = [w for w in waves if not w.done]
            if not live:
                break
            if all(w.at_barrier for w in live):
                for w in live:
                    w.at_barrier = False
                if self.races is not None:
                    self.epoch += 1
                continue
            if not progressed:
                raise RuntimeError("deadlock")

    def step(self, w, lds):
        if self.hooks and w.pc in self.label_at and self.label_at[w.pc] in self.hooks:
            self.hooks[self.label_at[w.pc]](self, w)
        if self.trace_labels is not None and w.pc in self.label_at:
            name = self.label_at[w.pc]
            if any(t in name for t in self.trace_labels) and not name.endswith('_back'):
                self.trace.append((w.wid, name))
        op, a, mods, text = self.insts[w.pc]
        w.pc += 1
        self.count += 1
        if self.count > 50_000_000:
            raise RuntimeError("instruction limit")
        try:
            self.exec(w, lds, op, a, mods)
        except Exception as e:
            raise RuntimeError(f"pc {w.pc - 1}: {text}: {e}") from e

    def exec(self, w, lds, op, a, mods):
        base = op.replace("_e32", "").replace("_e64", "")
        F = lambda t: u2f(self.vsrc(w, t, True))  # noqa: E731
        I_ = lambda t: self.vsrc(w, t).view(np.int32)  # noqa: E731
        U = lambda t: self.vsrc(w, t)  # noqa: E731
        # ------------------------------------------------ scalar
        if op == "s_waitcnt":
            # LDS-DMA data lands as late as the program allows: at the wait that forces it
            for t in a + [k for k in mods]:
                if t.startswith("vmcnt("):
                    n = int(t[6:-1])
                    while len(w.vm) > n:
                        self._land(w, lds, w.vm.pop(0))
            return
        if op == "s_nop" or op == "s_setprio":
            return
        if op == "s_endpgm":
            for e in w.vm:
                self._land(w, lds, e)
            w.vm = []
            w.done = True
            return
        if op == "s_barrier":
            w.at_barrier = True
            return
        if op == "s_branch":
            w.pc = self.labels[a[0]]
            return
        if op in ("s_cbranch_scc1", "s_cbranch_scc0"):
            if bool(w.scc) == (op == "s_cbranch_scc1"):
                w.pc = self.labels[a[0]]
            return
        if op in ("s_cbranch_vccnz", "s_cbranch_vccz"):
            if w.vcc.any() == (op == "s_cbranch_vccnz"):
                w.pc = self.labels[a[0]]
            return
        if op.startswith("s_load_dword"):
            n = {"s_load_dword": 1, "s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8,
                 "s_load_dwordx16": 16}[op]
            _, _, lo, _ = self.reg_index(a[0])
            b = self.ssrc64(w, a[1])
            off = self.ssrc(w, a[2])
            data = self.mem_read(b + off, 4 * n).view(np.uint32)
            w.s[lo:lo + n] = data
            return
        if op.startswith("s_"):
            self.salu(w, op, a)
            return
        # ------------------------------------------------ memory
        if op.startswith("buffer_"):
            self.buffer(w, lds, op, a, mods)
            return
        if op == "ds_read_b128":
            addr = self.vsrc(w, a[1]).astype(np.int64) + mods.get("offset", 0)
            self._lds_read(w, addr, 16)
            ri, n = self.regs(w, a[0])
            for lane in range(64):
                d = lds[addr[lane]:addr[lane] + 16].view(np.uint32)
                w.r[ri:ri + 4, lane] = d
            return
        if op in ("ds_write_b64", "ds_write_b128"):
            addr = self.vsrc(w, a[0]).astype(np.int64) + mods.get("offset", 0)
            ri, n = self.regs(w, a[1])
            nb = 8 if op == "ds_write_b64" else 16
            self._lds_write(w, addr, nb)
            for lane in range(64):
                lds[addr[lane]:addr[lane] + nb] = w.r[ri:ri + nb // 4, lane].astype(np.uint32).view(np.uint8)
            return
        if op == "ds_read_b64_tr_b16":
            addr = self.vsrc(w, a[1]).astype(np.int64) + mods.get("offset", 0)
            self._lds_read(w, addr, 8)
            ri, n = self.regs(w, a[0])
            loaded = np.stack([lds[addr[l]:addr[l] + 8].view(np.uint16) for l in range(64)])  # [64][4]
            out = np.zeros((64, 4), dtype=np.uint16)
            for g in range(4):
                for i in range(16):
                    for q in range(4):
                        out[16 * g + i, q] = loaded[16 * g + 4 * q + (i >> 2), i & 3]
            packed = out.view(np.uint32)   # [64][2]
            w.r[ri] = packed[:, 0]
            w.r[ri + 1] = packed[:, 1]
            return
        # ------------------------------------------------ vector
        if base.startswith("v_mfma_f32_32x32x16"):
            self.mfma(w, op, a)
            return
        if base == "v_readfirstlane_b32":
            _, _, lo, _ = self.reg_index(a[0])
            w.s[lo] = U(a[1])[0]
            return
        if base.startswith("v_cmp_"):
            self.vcmp(w, op, base, a)
            return
        if base == "v_cndmask_b32":
            if len(a) == 4 and a[3] != "vcc":
                m = self.ssrc64(w, a[3])
                mask = np.array([(m >> i) & 1 for i in range(64)], dtype=bool)
            else:
                mask = w.vcc
            self.vdst(w, a[0], np.where(mask, U(a[2]), U(a[1])))
            return
        if base == "v_permlane32_swap_b32":
            x = U(a[0])
            y = U(a[1])
            nx, ny = x.copy(), y.copy()
            nx[32:] = y[:32]
            ny[:32] = x[32:]
            self.vdst(w, a[0], nx)
            self.vdst(w, a[1], ny)
            return
        if base == "v_accvgpr_write_b32" or base == "v_accvgpr_read_b32" or base == "v_mov_b32":
            self.vdst(w, a[0], U(a[1]))
            return
        res = self.valu(w, base, a, F, I_, U)
        self.vdst(w, a[0], res)

    def valu(self, w, base, a, F, I_, U):
        with np.errstate(all="ignore"):
            if base == "v_lshrrev_b32":
                return U(a[2]) >> (U(a[1]) & 31)
            if base == "v_lshlrev_b32":
                return U(a[2]) << (U(a[1]) & 31)
            if base == "v_and_b32":
                return U(a[1]) & U(a[2])
            if base == "v_xor_b32":
                return U(a[1]) ^ U(a[2])
            if base == "v_lshl_add_u32":
                return (U(a[1]) << (U(a[2]) & 31)) + U(a[3])
            if base == "v_add_u32":
                return U(a[1]) + U(a[2])
            if base == "v_sub_u32":
                return U(a[1]) - U(a[2])
            if base == "v_subrev_u32":
                return U(a[2]) - U(a[1])
            if base == "v_mul_u32_u24":
                return (U(a[1]) & 0xFFFFFF) * (U(a[2]) & 0xFFFFFF)
            if base == "v_or_b32":
                return U(a[1]) | U(a[2])
            if base == "v_lshl_or_b32":
                return (U(a[1]) << (U(a[2]) & 31)) | U(a[3])
            if base == "v_mul_lo_u32":
                return (U(a[1]).astype(np.uint64) * U(a[2]).astype(np.uint64)).astype(np.uint32)
            if base == "v_min_i32":
                return np.minimum(I_(a[1]), I_(a[2])).view(np.uint32)
            if base == "v_bfe_u32":
                return (U(a[1]) >> U(a[2])) & ((np.uint32(1) << U(a[3])) - 1)
            if base == "v_cvt_f32_u32":
                return f2u(U(a[1]).astype(np.float32))
            if base == "v_cvt_f32_f16":
                return f2u(f16_to_f32((U(a[1]) & 0xFFFF).astype(np.uint16)).astype(np.float32))
            if base in ("v_dot2_f32_bf16", "v_dot2_f32_f16"):
                cv = bf16_to_f32 if base.endswith("bf16") else f16_to_f32
                x, y = U(a[1]), U(a[2])
                lo = cv((x & 0xFFFF).astype(np.uint16)).astype(np.float64) * cv((y & 0xFFFF).astype(np.uint16))
                hi = cv((x >> 16).astype(np.uint16)).astype(np.float64) * cv((y >> 16).astype(np.uint16))
                return f2u(np.float32(lo + hi + F(a[3])))
            if base == "v_fma_f32":
                return f2u(np.float32(F(a[1]).astype(np.float64) * F(a[2]) + F(a[3])))
            if base == "v_exp_f32":
                return f2u(np.exp2(F(a[1])))
            if base == "v_log_f32":
                return f2u(np.log2(F(a[1])))
            if base == "v_rcp_f32":
                return f2u(np.float32(1.0) / F(a[1]))
            if base == "v_add_f32":
                return f2u(F(a[1]) + F(a[2]))
            if base == "v_sub_f32":
                return f2u(F(a[1]) - F(a[2]))
            if base == "v_mul_f32":
                return f2u(F(a[1]) * F(a[2]))
            if base == "v_max_f32":
                return f2u(np.fmax(F(a[1]), F(a[2])))
            if base == "v_max3_f32":
                return f2u(np.fmax(np.fmax(F(a[1]), F(a[2])), F(a[3])))
            if base == "v_cvt_pk_bf16_f32":
                return f32_to_bf16(F(a[1])) | (f32_to_bf16(F(a[2])) << 16)
            if base == "v_cvt_pk_f16_f32":
                return f32_to_f16(F(a[1])) | (f32_to_f16(F(a[2])) << 16)
        raise NotImplementedError(base)

    def vcmp(self, w, op, base, a):
        kind = base.split("_")[2]
        ty = base.split("_")[3]
        if ty == "f32":
            x, y = u2f(self.vsrc(w, a[1], True)), u2f(self.vsrc(w, a[2], True))
        elif ty == "i32":
            x, y = self.vsrc(w, a[1]).view(np.int32), self.vsrc(w, a[2]).view(np.int32)
        else:
            x, y = self.vsrc(w, a[1]), self.vsrc(w, a[2])
        with np.errstate(all="ignore"):
            r = {"gt": x > y, "lt": x < y, "ge": x >= y, "le": x <= y, "eq": x == y,
                 "neq": ~(x == y), "nge": ~(x >= y), "lg": (x < y) | (x > y), "ne": x != y}[kind]
        if a[0] == "vcc":
            w.vcc = r
        else:
            _, _, lo, _ = self.reg_index(a[0])
            m = sum(1 << i for i in range(64) if r[i])
            w.s[lo] = m & 0xFFFFFFFF
            w.s[lo + 1] = m >> 32

    def salu(self, w, op, a):
        s = w.s
        if op in ("s_cmp_eq_u64", "s_cmp_lg_u64"):
            x = self.ssrc64(w, a[0])
            y = self.ssrc64(w, a[1]) if a[1] in ("vcc",) or a[1].startswith("s[") else int(a[1], 0)
            w.scc = (x == y) if op == "s_cmp_eq_u64" else (x != y)
            return
        if op in ("s_and_b64", "s_lshl_b64", "s_lshr_b64"):
            x = self.ssrc64(w, a[1])
            if op == "s_and_b64":
                r = x & self.ssrc64(w, a[2])
            elif op == "s_lshl_b64":
                r = (x << (self.ssrc(w, a[2]) & 63)) & (2 ** 64 - 1)
            else:
                r = x >> (self.ssrc(w, a[2]) & 63)
            if a[0] == "vcc":
                w.vcc = np.array([(r >> i) & 1 for i in range(64)], dtype=bool)
            else:
                _, _, lo, _ = self.reg_index(a[0])
                s[lo] = r & 0xFFFFFFFF
                s[lo + 1] = r >> 32
            w.scc = r != 0
            return
        if op.startswith("s_cmp_") or op == "s_bitcmp1_b32":
            x, y = self.ssrc(w, a[0]), self.ssrc(w, a[1])
            if op == "s_bitcmp1_b32":
                w.scc = bool((x >> y) & 1)
                return
            kind, ty = op.split("_")[2], op.split("_")[3]
            if ty == "i32":
                x = x - (1 << 32) if x >= 1 << 31 else x
                y = y - (1 << 32) if y >= 1 << 31 else y
            w.scc = {"eq": x == y, "lg": x != y, "lt": x < y, "le": x <= y, "gt": x > y, "ge": x >= y}[kind]
            return
        dst = a[0]
        x = self.ssrc(w, a[1]) if len(a) > 1 else 0
        y = self.ssrc(w, a[2]) if len(a) > 2 else 0
        sx = x - (1 << 32) if x >= 1 << 31 else x
        sy = y - (1 << 32) if y >= 1 << 31 else y
        if op == "s_mov_b32":
            r = x
        elif op == "s_add_u32":
            t = x + y
            r, w.scc = t & 0xFFFFFFFF, t >> 32 != 0
        elif op == "s_addc_u32":
            t = x + y + int(w.scc)
            r, w.scc = t & 0xFFFFFFFF, t >> 32 != 0
        elif op == "s_sub_u32":
            r, w.scc = (x - y) & 0xFFFFFFFF, y > x
        elif op == "s_sub_i32":
            r = (sx - sy) & 0xFFFFFFFF
        elif op == "s_mul_i32":
            r = (sx * sy) & 0xFFFFFFFF
        elif op == "s_mul_hi_u32":
            r = (x * y) >> 32
        elif op == "s_lshl_b32":
            r = (x << (y & 31)) & 0xFFFFFFFF
            w.scc = r != 0
        elif op == "s_lshr_b32":
            r = x >> (y & 31)
            w.scc = r != 0
        elif op == "s_and_b32":
            r = x & y
            w.scc = r != 0
        elif op == "s_or_b32":
            r = x | y
            w.scc = r != 0
        elif op == "s_min_u32":
            r = min(x, y)
        elif op == "s_min_i32":
            r = min(sx, sy) & 0xFFFFFFFF
        elif op == "s_max_i32":
            r = max(sx, sy) & 0xFFFFFFFF
        elif op == "s_cselect_b32":
            r = x if w.scc else y
        else:
            raise NotImplementedError(op)
        if dst == "m0":
            w.m0 = r
        else:
            _, _, lo, _ = self.reg_index(dst)
            s[lo] = r

    def _land(self, w, lds, e):
        """a VMEM load completes: LDS-DMA bytes or (POISON) deferred register data"""
        if e is None:
            return
        if e[0] == "reg":
            w.r[e[1]:e[1] + e[2].shape[0]] = e[2]
            return
        lds[e[0]:e[0] + len(e[1])] = e[1]
        self._dma_land(w, e[0], len(e[1]))

    def buffer(self, w, lds, op, a, mods):
        n = {"buffer_load_dword": 1, "buffer_load_dwordx4": 4, "buffer_store_dword": 1, "buffer_store_dwordx2": 2,
             "buffer_store_dwordx4": 4}[op]
        if mods.get("lds"):       # buffer_load_* vaddr, srsrc, soffset ... lds (no data register)
            a = [None] + list(a)
        base, nrec = self.desc(w, a[2])
        voff = self.vsrc(w, a[1]).astype(np.int64) if mods.get("offen") else np.zeros(64, np.int64)
        off = voff + mods.get("offset", 0) + self.ssrc(w, a[3])
        size = 4 * n
        ok = (off >= 0) & (off + size <= nrec)
        if op.startswith("buffer_load"):
            data = np.zeros((64, n), dtype=np.uint32)
            for lane in range(64):
                if ok[lane]:
                    data[lane] = self.mem_read(base + int(off[lane]), size).view(np.uint32)
            if mods.get("lds"):
                # lands later (s_waitcnt vmcnt): a read before the wait sees the old LDS contents
                dst = w.m0
                w.vm.append((dst, np.ascontiguousarray(data).view(np.uint8).ravel().copy()))
                self._lds_write(w, [dst], 64 * size, dma=True)
                return
            else:
                ri, _ = self.regs(w, a[0])
                if POISON:   # lands at the wait that forces it, as the LDS-DMA data (a missing wait reads poison)
                    w.vm.append(("reg", ri, np.ascontiguousarray(data.T)))
                    return
                w.r[ri:ri + n] = data.T
        else:
            ri, _ = self.regs(w, a[0])
            for lane in range(64):
                if ok[lane]:
                    self.heap.get(base + int(off[lane]), size)[:] = np.ascontiguousarray(w.r[ri:ri + n, lane]).view(np.uint8)
        if not mods.get("lds"):
            w.vm.append(None)

    def mfma(self, w, op, a):
        self.mfma_count += 1
        bf = op.endswith("bf16")
        dr, _ = self.regs(w, a[0])
        ar_, _ = self.regs(w, a[1])
        br, _ = self.regs(w, a[2])

        def unpack(ri):
            x = w.r[ri:ri + 4].T.copy().view(np.uint16).reshape(64, 8)   # lane, element j
            return bf16_to_f32(x) if bf else f16_to_f32(x)

        A = unpack(ar_)   # [lane][j]: A[r][8h + j]
        B = unpack(br)
        Am = np.zeros((32, 16), np.float32)
        Bm = np.zeros((16, 32), np.float32)
        for h in range(2):
            Am[:, 8 * h:8 * h + 8] = A[32 * h:32 * h + 32]
            Bm[8 * h:8 * h + 8, :] = B[32 * h:32 * h + 32].T
        if a[3] == "0":
            C = np.zeros((32, 32), np.float32)
        else:
            cr, _ = self.regs(w, a[3])
            C = self.acc_to_mat(w.r[cr:cr + 16])
        Dm = (Am.astype(np.float64) @ Bm.astype(np.float64) + C).astype(np.float32)
        w.r[dr:dr + 16] = self.mat_to_acc(Dm)

    @staticmethod
    def acc_to_mat(regs):
        M = np.zeros((32, 32), np.float32)
        v = u2f(regs)   # [16][64]
        for g in range(16):
            for h in range(2):
                row = (g & 3) + 8 * (g >> 2) + 4 * h
                M[row, :] = v[g, 32 * h:32 * h + 32]
        return M

    @staticmethod
    def mat_to_acc(M):
        out = np.zeros((16, 64), np.uint32)
        for g in range(16):
            for h in range(2):
                row = (g & 3) + 8 * (g >> 2) + 4 * h
                out[g, 32 * h:32 * h + 32] = f2u(M[row, :])
        return out
