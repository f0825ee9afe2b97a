"""ISA check of the built gfx950 code objects (CPU only: disassembles libflash_attn_mi355x.so).

Every LDS-DMA (`buffer_load_* ... lds`) is inline asm (fa_common.h dma16 / dma4), which the
compiler's hazard recognizer does not look into.  gfx950 needs five wait states between a VALU
write of an SGPR and a VMEM instruction that reads it, and under SGPR pressure the compiler reloads
the buffer descriptor from a spill lane (`v_readlane_b32`) right before the asm.  With one wait
state that DMA read a stale descriptor word: the masked non-causal dropout forward at d = 128
produced a wrong LSE / NaN (Known issues, round 2).  The asm therefore opens with
`s_nop 4`; this test holds every DMA in the shipped library to that, path-independently (the nop
and the DMA are one asm block, no branch target between them), and separately reports any VALU
SGPR write inside the five-state window of the linear stream.
"""
import os
import re
import shutil
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "xhy-flash-attention_amd", "libflash_attn_mi355x.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(blob):
    """gfx950 ELF code objects of every offload bundle in the .hip_fatbin section."""
    out, i = [], 0
    while True:
        j = blob.find(MAGIC, i)
        if j < 0:
            return out
        n = struct.unpack_from("<Q", blob, j + 24)[0]
        p = j + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                out.append(blob[j + off:j + off + size])
        i = j + len(MAGIC)


def _sgprs(tok):
    tok = tok.strip()
    m = re.match(r"s\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    if m:
        return {int(m.group(1))}
    return {"m0"} if tok == "m0" else set()


def _disassemble():
    if not os.path.exists(LIB) or not os.path.exists(OBJDUMP):
        pytest.skip("library not built or llvm-objdump missing")
    with open(LIB, "rb") as f:
        blob = f.read()
    cos = _code_objects(blob)
    assert cos, "no gfx950 code object in the library"
    tmp = tempfile.mkdtemp()
    try:
        kernels = {}
        for n, co in enumerate(cos):
            path = os.path.join(tmp, f"co{n}.elf")
            with open(path, "wb") as f:
                f.write(co)
            txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", path], capture_output=True, text=True,
                                 check=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    cur = m.group(1)
                    kernels[cur] = []
                    continue
                s = line.strip()
                if cur and s and not s.startswith(";"):
                    kernels[cur].append(s.split("//")[0].strip())
        return kernels
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def test_lds_dma_preceded_by_five_wait_states():
    kernels = _disassemble()
    n_dma, bad, window = 0, [], []
    for name, ins in kernels.items():
        for k, s in enumerate(ins):
            if not (s.startswith("buffer_load") and re.search(r"\blds\b", s)):
                continue
            n_dma += 1
            prev = ins[k - 1] if k else ""
            m = re.match(r"s_nop (\d+)", prev)
            if not (m and int(m.group(1)) >= 4):
                bad.append(f"{name}: `{prev}` before `{s}`")
            ops = [o.strip() for o in s.split(None, 1)[1].split(",")]
            used = _sgprs(ops[1]) | {"m0"}
            ws, j = 0, k - 1
            while j >= 0 and ws < 5:
                p = ins[j]
                op = p.split()[0]
                if op == "s_nop":
                    ws += int(p.split()[1]) + 1
                else:
                    if op.startswith("v_") and len(p.split()) > 1:
                        if _sgprs(p.split(None, 1)[1].split(",")[0]) & used:
                            window.append(f"{name}: `{p}` within {ws} wait states of `{s}`")
                    ws += 1
                j -= 1
    assert n_dma > 0, "no LDS-DMA found: disassembly format changed?"
    assert not bad, f"{len(bad)} LDS-DMA without the s_nop 4 guard, e.g. {bad[:3]}"
    assert not window, f"VALU SGPR writes inside the hazard window: {window[:3]}"
