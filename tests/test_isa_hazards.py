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


# ------------------------------------------------------------------------------------------------
# the assembly kernels (csrc/asm/gen_*.py), re-checked by a hazard table that shares no code with
# the generators' wait-state inserter (csrc/asm/isa.py): tools/hazard_check.py
# ------------------------------------------------------------------------------------------------
sys_path_tools = os.path.join(ROOT, "tools")

PLANTED = """
	.amdgcn_target "amdgcn-amd-amdhsa--gfx950"
	.text
	.globl fa_fwd_asm_planted
	.p2align 8
	.type fa_fwd_asm_planted,@function
fa_fwd_asm_planted:
	v_cvt_pk_bf16_f32 v0, v1, v2
	v_mfma_f32_32x32x16_bf16 v[16:31], v[0:3], v[4:7], 0
	s_nop 15
	v_cvt_pk_bf16_f32 v0, v1, v2
	s_nop 1
	v_mfma_f32_32x32x16_bf16 a[0:15], v[0:3], v[4:7], 0
	v_mfma_f32_32x32x16_bf16 a[0:15], v[0:3], v[4:7], a[0:15]
	s_nop 10
	v_accvgpr_read_b32 v40, a15
	s_nop 15
	s_mov_b32 m0, s5
	buffer_load_dwordx4 v1, s[8:11], 0 offen lds
	v_readfirstlane_b32 s8, v3
	s_nop 2
	buffer_load_dwordx4 v1, s[8:11], 0 offen lds
	v_exp_f32_e32 v9, v9
	v_add_f32_e32 v10, v9, v10
	v_mov_b32_e32 v50, v51
	s_cbranch_scc1 .Lt
	s_nop 15
	s_nop 15
.Lt:
	v_mfma_f32_32x32x16_bf16 v[60:75], v[50:53], v[4:7], 0
	s_endpgm
.Lend:
	.size fa_fwd_asm_planted, .Lend-fa_fwd_asm_planted
"""


def test_hazard_checker_catches_planted_hazards(tmp_path):
    """every rule of the independent checker fires on a planted violation -- the last one only
    along the taken branch (the fall-through path is padded)"""
    import sys
    sys.path.insert(0, sys_path_tools)
    import hazard_check as hc

    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump missing")
    src, obj = tmp_path / "t.s", tmp_path / "t.o"
    src.write_text(PLANTED)
    subprocess.run(["/opt/rocm/lib/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", str(src), "-o", str(obj)], check=True)
    txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(obj)], capture_output=True, text=True, check=True).stdout
    (name, ins), = hc.parse(txt).items()
    bad = hc.check_kernel(name, ins)
    rules = sorted({b.split("rule ")[1].split()[0] for b in bad})
    assert rules == sorted(["valu->mfma", "mfma->access", "m0->lds_dma", "valu_sgpr->vmem", "trans->valu"]), bad
    # the chained accumulation (C == D) is not a violation; the branch path is
    assert not any("a[0:15], v[0:3], v[4:7], a[0:15]` 0" in b for b in bad)
    assert any("v[60:75]" in b for b in bad)


def test_shipped_assembly_kernels_hazard_free():
    """every kernel of the seven embedded code objects, every control-flow path"""
    import sys
    sys.path.insert(0, sys_path_tools)
    import hazard_check as hc

    if not os.path.exists(LIB) or not os.path.exists(OBJDUMP):
        pytest.skip("library not built or llvm-objdump missing")
    res = hc.check_library(LIB)
    names = sorted(res)
    assert len([n for n in names if n.startswith("fa_fwd_asm_")]) == 8, names
    assert len([n for n in names if n.startswith("fa_fwdnf_asm_")]) == 8, names      # without the Q fold
    assert len([n for n in names if n.startswith("fa_bwd_dkdv_asm_d128")]) == 8, names   # (+ the c = 1 kernels)
    assert len([n for n in names if n.startswith("fa_bwd_dkdv_asm_d64")]) == 8, names    # head dim 64
    assert len([n for n in names if n.startswith("fa_bwd_dq_asm_d128")]) == 4, names
    assert len([n for n in names if n.startswith("fa_bwd_dq_asm_d64")]) == 8, names      # head dim 64 (+ c = 1)
    assert len([n for n in names if n.startswith("fa_bwd2_dkdv_asm_")]) == 8, names  # two waves per SIMD
    for n, (count, bad) in res.items():
        assert count > 1000, (n, count)
        assert not bad, f"{n}: {len(bad)} violations, e.g. {bad[:3]}"
