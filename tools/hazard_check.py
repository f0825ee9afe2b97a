#!/usr/bin/env python3
"""Independent wait-state check of the shipped gfx950 assembly kernels (test / dev tool).

The assembly generators insert their wait states with csrc/asm/isa.py.  This checker shares no code
with it: it reads the code objects embedded in libflash_attn_mi355x.so (the `fa_*_asm_co` byte
arrays: whole AMDGPU ELF files inside the host library), disassembles them with llvm-objdump, builds
each kernel's control-flow graph from the branch targets and, for every instruction, walks every
path backwards through its predecessors until the largest requirement is covered, checking the
gfx950 rules below (wait states = issued instructions in between, `s_nop N` counting N + 1):

    producer -> consumer                                                   wait states
    VALU (incl. v_accvgpr_write) writes a VGPR/AGPR -> MFMA reads it             2
    MFMA 32x32 (8 passes) writes -> any non-MFMA read or write of those regs    12
    MFMA 32x32 writes -> another MFMA reads them, except as the same
        accumulator (C == D, the accumulation chain)                           12
    VALU writes an SGPR -> VMEM (buffer / global, LDS-DMA included) reads it     5
    SALU writes M0 -> LDS-DMA (buffer_load ... lds)                              1
    transcendental (v_exp / v_log / v_rcp / ...) -> VALU reads its result        1
    VALU writes a VGPR -> v_permlane*_swap reads it                              2
    VALU writes a VGPR -> v_readfirstlane / v_readlane reads it                  1
    v_dot* writes a VGPR -> another VALU reads it (except the same v_dot
        opcode reading it as the accumulator, src2)                            3

    python tools/hazard_check.py [LIB.so]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "xhy-flash-attention_amd", "libflash_attn_mi355x.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
EM_AMDGPU = 224
TRANS_OPS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")

RULES = {   # name: wait states
    "valu->mfma": 2, "mfma->access": 12, "mfma->mfma": 12, "valu_sgpr->vmem": 5, "m0->lds_dma": 1,
    "trans->valu": 1, "valu->permlane": 2, "valu->readlane": 1, "dot->valu": 3,
}
MAXWS = max(RULES.values())


def embedded_code_objects(blob):
    """AMDGPU ELF images embedded in the host library (skipping the host ELF at offset 0)"""
    out, i = [], 1
    while True:
        j = blob.find(b"\x7fELF", i)
        if j < 0:
            return out
        i = j + 4
        if j + 64 > len(blob) or blob[j + 4] != 2 or blob[j + 5] != 1:
            continue
        machine = struct.unpack_from("<H", blob, j + 18)[0]
        if machine != EM_AMDGPU:
            continue
        shoff = struct.unpack_from("<Q", blob, j + 40)[0]
        shentsize, shnum = struct.unpack_from("<HH", blob, j + 58)
        end = j + shoff + shentsize * shnum
        if end > len(blob) or shnum == 0:
            continue
        out.append(blob[j:end])
        i = end


def regs(tok):
    """register set of one operand: {('v', n), ('a', n), ('s', n), ('vcc',), ('m0',), ('scc',)}"""
    tok = tok.strip()
    if tok.startswith("-"):
        tok = tok[1:]
    m = re.match(r"^([vas])\[(\d+):(\d+)\]$", tok)
    if m:
        return {(m.group(1), k) for k in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"^([vas])(\d+)$", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    if tok in ("vcc", "vcc_lo", "vcc_hi"):
        return {("s", "vcc")}
    if tok == "m0":
        return {("m0",)}
    return set()


class Ins:
    __slots__ = ("addr", "op", "ops", "target", "text", "kind", "rd", "wr", "rd_c", "rd_ab", "srsrc")

    def __init__(self, addr, text, target):
        self.addr, self.text, self.target = addr, text, target
        parts = text.split(None, 1)
        self.op = parts[0]
        body = parts[1] if len(parts) > 1 else ""
        self.ops = [o.strip() for o in re.split(r",\s*", body.split(" offen")[0].split(" offset:")[0])] if body else []
        self.rd, self.wr, self.rd_c, self.rd_ab, self.srsrc = set(), set(), set(), set(), set()
        op, o = self.op, self.ops
        if op.startswith("v_mfma"):
            self.kind = "mfma"
            self.wr = regs(o[0])
            self.rd_ab = regs(o[1]) | regs(o[2])
            self.rd_c = regs(o[3]) if len(o) > 3 else set()
            self.rd = self.rd_ab | self.rd_c
        elif op.startswith("v_"):
            self.kind = "trans" if op.startswith(TRANS_OPS) else "valu"
            if op.startswith("v_permlane"):
                self.kind = "permlane"
                self.wr = regs(o[0]) | regs(o[1])
                self.rd = set(self.wr)
            elif op.startswith("v_cmp") and op.endswith("_e32"):
                self.wr = {("s", "vcc")}
                self.rd = set().union(*(regs(x) for x in o[1:]))
            else:
                self.wr = regs(o[0])
                self.rd = set().union(*(regs(x) for x in o[1:])) if len(o) > 1 else set()
                if op.startswith("v_cndmask") and op.endswith("_e32"):
                    self.rd |= {("s", "vcc")}
            if op.startswith(("v_readfirstlane", "v_readlane")):
                self.kind = "readlane"
        elif op.startswith("ds_"):
            self.kind = "lds"
            if op.startswith("ds_read"):
                self.wr = regs(o[0])
                self.rd = regs(o[1])
            else:
                self.rd = set().union(*(regs(x) for x in o))
        elif op.startswith(("buffer_", "global_")):
            lds = re.search(r"\blds\b", text) is not None
            self.kind = "lds_dma" if lds else "vmem"
            if lds:
                self.rd = set().union(*(regs(x) for x in o))
                self.srsrc = set().union(*(regs(x) for x in o[1:]))
            elif "load" in op:
                self.wr = regs(o[0])
                self.rd = set().union(*(regs(x) for x in o[1:]))
                self.srsrc = set().union(*(regs(x) for x in o[2:]))
            else:
                self.rd = set().union(*(regs(x) for x in o))
                self.srsrc = set().union(*(regs(x) for x in o[2:]))
            self.rd |= {("m0",)} if lds else set()
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            self.kind = "smem"
            self.wr = regs(o[0])
            self.rd = set().union(*(regs(x) for x in o[1:]))
            self.srsrc = set(self.rd)
        elif op == "s_nop":
            self.kind = "nop"
        elif op.startswith("s_"):
            self.kind = "salu"
            if o and not op.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier",
                                        "s_endpgm", "s_setprio")):
                self.wr = regs(o[0])
                self.rd = set().union(*(regs(x) for x in o[1:])) if len(o) > 1 else set()
            else:
                self.rd = set().union(*(regs(x) for x in o)) if o else set()
        else:
            self.kind = "other"

    def ws(self):
        return int(self.ops[0], 0) + 1 if self.kind == "nop" else 1


def parse(txt):
    kernels, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            kernels[cur] = []
            continue
        if cur is None or "//" not in line:
            continue
        code, com = line.split("//", 1)
        code = code.strip()
        m = re.match(r"\s*([0-9A-Fa-f]+):", com)
        if not code or not m:
            continue
        t = re.search(r"<\S+\+0x([0-9a-f]+)>", com)
        kernels[cur].append((int(m.group(1), 16), code, t))
    out = {}
    for name, rows in kernels.items():
        base = rows[0][0] if rows else 0
        ins = [Ins(a, c, base + int(t.group(1), 16) if t and c.split()[0].startswith(("s_branch", "s_cbranch")) else None)
               for a, c, t in rows]
        out[name] = ins
    return out


def need(p, c):
    """(rule, wait states) that consumer c needs after producer p, or None"""
    found = []
    if p.kind == "mfma":
        touched = (c.rd | c.wr) & p.wr
        if touched:
            if c.kind == "mfma":
                chain = c.wr == p.wr and c.rd_c == c.wr and not (c.rd_ab & p.wr)
                if not chain:
                    found.append("mfma->mfma")
            else:
                found.append("mfma->access")
    if p.kind in ("valu", "trans", "permlane", "readlane"):
        vw = {r for r in p.wr if r[0] in ("v", "a")}
        sw = {r for r in p.wr if r[0] == "s"}
        if c.kind == "mfma" and vw & c.rd:
            found.append("valu->mfma")
        if c.kind in ("vmem", "lds_dma") and sw & c.srsrc:
            found.append("valu_sgpr->vmem")
        if c.kind == "permlane" and vw & c.rd:
            found.append("valu->permlane")
        if c.kind == "readlane" and vw & c.rd:
            found.append("valu->readlane")
        if p.kind == "trans" and c.kind in ("valu", "trans", "permlane", "readlane") and vw & c.rd:
            found.append("trans->valu")
        if p.op.startswith("v_dot") and c.kind in ("valu", "trans", "permlane", "readlane") and vw & c.rd:
            co = c.ops
            acc_only = (c.op == p.op and len(co) > 3 and not (vw & (regs(co[1]) | regs(co[2]))))
            if not acc_only:
                found.append("dot->valu")
    if p.kind == "salu" and ("m0",) in p.wr and c.kind == "lds_dma":
        found.append("m0->lds_dma")
    if not found:
        return None
    r = max(found, key=lambda k: RULES[k])
    return r, RULES[r]


def check_kernel(name, ins):
    """list of violations (text) over every control-flow path"""
    at = {x.addr: i for i, x in enumerate(ins)}
    preds = [[] for _ in ins]
    for i, x in enumerate(ins):
        falls = not (x.op in ("s_branch", "s_endpgm", "s_setpc_b64") )
        if falls and i + 1 < len(ins):
            preds[i + 1].append(i)
        if x.target is not None and x.target in at:
            preds[at[x.target]].append(i)
    bad = []
    for k, c in enumerate(ins):
        if c.kind in ("nop", "other"):
            continue
        seen = set()
        stack = [(j, 0) for j in preds[k]]
        while stack:
            j, ws = stack.pop()
            if ws >= MAXWS or (j, ws) in seen:
                continue
            seen.add((j, ws))
            p = ins[j]
            r = need(p, c)
            if r is not None and ws < r[1]:
                bad.append(f"{name}+0x{c.addr - ins[0].addr:x}: `{c.text}` {ws} wait states after "
                           f"`{p.text}` (+0x{p.addr - ins[0].addr:x}), rule {r[0]} needs {r[1]}")
            stack += [(q, ws + p.ws()) for q in preds[j]]
    return bad


ASM_PREFIXES = (b"fa_fwd_asm_", b"fa_fwdnf_asm_", b"fa_bwd_dkdv_asm_", b"fa_bwd_dq_asm_", b"fa_bwd2_dkdv_asm_")


def check_library(path=LIB):
    """{kernel: (instructions, violations)} over the assembly kernels' code objects (the hipcc-built
    kernels in the offload bundle are the compiler hazard recognizer's; tests/test_isa_hazards.py
    checks their inline-asm LDS-DMA separately)"""
    blob = open(path, "rb").read()
    cos = [co for co in embedded_code_objects(blob) if any(p in co for p in ASM_PREFIXES)]
    results = {}
    with tempfile.TemporaryDirectory() as tmp:
        for n, co in enumerate(cos):
            p = os.path.join(tmp, f"co{n}.elf")
            open(p, "wb").write(co)
            txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", p], capture_output=True, text=True, check=True).stdout
            for name, ins in parse(txt).items():
                if name.encode().startswith(ASM_PREFIXES):
                    results[name] = (len(ins), check_kernel(name, ins))
    return results


if __name__ == "__main__":
    res = check_library(sys.argv[1] if len(sys.argv) > 1 else LIB)
    total = 0
    for name, (n, bad) in sorted(res.items()):
        print(f"{name}: {n} instructions, {len(bad)} violations")
        for b in bad[:10]:
            print("   ", b)
        total += len(bad)
    sys.exit(1 if total else 0)
