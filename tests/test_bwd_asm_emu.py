"""CPU checks of the hand-scheduled assembly dK / dV kernel (csrc/asm/gen_bwd.py).

The generated program runs in the functional emulator (tools/asm_emu.py) on small shapes that cover
every step variant (first / masked / regular / last, the drain), causal and full attention, ragged
seqlen_q and seqlen_k, sq != sk, GQA reduced in-kernel over the group (the sweep crossing head
boundaries, with an odd subtile count padded) and expanded per query head, bf16 and fp16 -- compared
with a float64 restatement of the reference's backward (tools/emu_bwd.py).  Timing (counted waits,
wait states) is checked statically by the generator (isa.py) and on the GPU
(tests/test_flash_attn_gpu.py, which runs this kernel for every head-dim-128 backward).
"""
import importlib.util
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import emu_bwd  # noqa: E402


@pytest.fixture(scope="module")
def asm_text():
    return emu_bwd.asm_text()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16,reduce", [
    (1, 64, 128, 1, 1, True, True, False),      # one step: first + last + masked
    (1, 300, 300, 1, 1, True, True, False),     # masked -> fast, ragged both
    (1, 200, 330, 2, 1, True, True, True),      # GQA reduce: the sweep crosses a head boundary
    (1, 330, 200, 2, 1, True, True, False),     # GQA expanded, sq > sk
    (1, 257, 129, 1, 1, False, True, False),    # full attention, odd subtile count (padded)
    (1, 96, 300, 3, 1, True, False, True),      # fp16, keys past every query (zero sweep)
])
def test_asm_dkdv_in_emulator(asm_text, b, sq, sk, h, hk, causal, bf16, reduce):
    ek, ev, *_ = emu_bwd.run(b, sq, sk, h, hk, causal, bf16, reduce, seed=0, text=asm_text, verbose=False)
    # bf16 / fp16 rounding of P, dS (MFMA operands) and of the outputs, relative to max |dK|, |dV|
    tol = 1e-2 if bf16 else 2e-3
    assert ek <= tol and ev <= tol, (ek, ev)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16,reduce", [
    (1, 300, 300, 1, 1, True, True, False),     # masked -> fast, ragged both
    (1, 257, 129, 2, 1, False, False, True),    # fp16, full attention, GQA reduce
])
def test_asm_dkdv_unit_c_in_emulator(asm_text, b, sq, sk, h, hk, causal, bf16, reduce):
    """the _c1 kernels (c = 1: P = exp2(S') with no multiply; launch_bwd's backward on Q')"""
    ek, ev, *_ = emu_bwd.run(b, sq, sk, h, hk, causal, bf16, reduce, seed=5, text=asm_text, verbose=False,
                             unit_c=True)
    tol = 1e-2 if bf16 else 2e-3
    assert ek <= tol and ev <= tol, (ek, ev)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,reduce,grid", [
    (1, 200, 300, 2, 1, True, True, 1),      # one workgroup walks all 3 key blocks (+ causal skips)
    (2, 150, 130, 4, 2, False, False, 3),    # 16 items over 3 workgroups, snake rounds
    (1, 100, 260, 8, 8, True, False, 8),     # G % 8 == 0: reversal over groups of 8; empty items
])
def test_asm_dkdv_persistent_loop(asm_text, b, sq, sk, h, hk, causal, reduce, grid):
    """the persistent item loop (fa_bwd_asm.cpp, knob 6): fewer workgroups than items"""
    ek, ev, *_ = emu_bwd.run(b, sq, sk, h, hk, causal, True, reduce, seed=3, text=asm_text, verbose=False, grid=grid)
    assert ek <= 1e-2 and ev <= 1e-2, (ek, ev)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("lens,h,hk,causal,reduce,grid", [
    ([200, 70, 300], 2, 1, True, True, None),     # varlen, one workgroup per item (empty key blocks exit)
    ([200, 70, 300], 2, 1, True, True, 4),        # 2-3 items per workgroup: an item without keys, then none
    ([130, 0, 260, 40], 2, 1, True, True, 3),     # an empty sequence; short items (< 3 steps) -> stalled cursors
    ([90, 257, 33], 3, 3, False, False, 2),       # full attention, heads expanded
])
@pytest.mark.parametrize("table", [False, True])
def test_asm_dkdv_varlen_in_emulator(asm_text, lens, h, hk, causal, reduce, grid, table):
    """varlen (cu_seqlens) launches, one workgroup per item and the item loop over several items
    (FLASH_ATTN_MI355X_VARLEN_ROUNDS): the pipelined loop switches items whose work order skips
    blocks past a sequence's end; table: the items from the device-built list (flags bit 2, the
    persistent varlen launch)"""
    ek, ev, *_ = emu_bwd.run(h=h, hk=hk, causal=causal, bf16=True, reduce=reduce, seed=1, text=asm_text, verbose=False,
                             grid=grid, lens=lens, table=table)
    assert ek <= 1e-2 and ev <= 1e-2, (ek, ev)


@pytest.mark.timeout(900)
def test_asm_dkdv_pipelined_loop_in_emulator():
    """the pipelined item loop (dev switch FA_GBW_CONT=1, off in the shipped build: the next item's
    subtiles DMA'd and its K / V loaded under the current item's last steps, a stalled cursor
    re-issued at the item switch): fixed length over 3 workgroups, varlen with short items, empty
    sequences and blocks without keys, from the decoded order and from the device list"""
    env = dict(os.environ, FA_GBW_CONT="1")
    text = subprocess.run([sys.executable, emu_bwd.GEN], check=True, capture_output=True, text=True, env=env).stdout
    ek, ev, *_ = emu_bwd.run(2, 150, 130, 4, 2, False, True, False, seed=3, text=text, verbose=False, grid=3)
    assert ek <= 1e-2 and ev <= 1e-2, (ek, ev)
    for table in (False, True):
        ek, ev, *_ = emu_bwd.run(h=2, hk=1, causal=True, bf16=True, reduce=True, seed=1, text=text, verbose=False,
                                 grid=3, lens=[130, 0, 260, 40], table=table)
        assert ek <= 1e-2 and ev <= 1e-2, (table, ek, ev)


def test_generated_dkdv_kernels_are_hazard_free():
    spec = importlib.util.spec_from_file_location(
        "asm_isa", os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "isa.py"))
    isa = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(isa)
    text = subprocess.run([sys.executable, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_bwd.py")],
                          check=True, capture_output=True, text=True).stdout
    assert text.count(".amdhsa_kernel ") == 8
    assert ".amdhsa_group_segment_fixed_size 151552" in text
    lines = [x.strip() for x in text.splitlines()]
    for i, x in enumerate(lines):
        if x.startswith("buffer_load_dword") and x.endswith(" lds"):
            prev = lines[i - 1]
            assert not prev.startswith("s_add_u32 m0") and not prev.startswith("s_mov_b32 m0"), (i, prev)
        if x.startswith("v_readfirstlane_b32"):
            # no VALU write of the read VGPR in the instruction before (VALU -> readfirstlane: 1 wait state)
            src = x.split(",")[1].strip()
            prev = lines[i - 1]
            assert not (prev.startswith("v_") and not prev.startswith("v_readfirstlane")
                        and prev.split()[1].rstrip(",") == src), (i, prev)


# ------------------------------------------------------------------------------------------------
# the assembly dQ kernel (csrc/asm/gen_dq.py), against the float64 dQ of tools/emu_dq.py
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def dq_text():
    import emu_dq
    return emu_dq.asm_text()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16", [
    (1, 64, 64, 1, 1, True, True),              # one step: first + last + masked
    (1, 300, 300, 1, 1, True, True),            # fast -> masked, ragged both
    (1, 330, 200, 2, 1, True, True),            # GQA, sq > sk (rows past every key)
    (1, 257, 129, 1, 1, False, True),           # full attention, odd subtile count (padded)
    (1, 96, 300, 3, 1, True, False),            # fp16, sq < sk
])
def test_asm_dq_in_emulator(dq_text, b, sq, sk, h, hk, causal, bf16):
    import emu_dq
    e, *_ = emu_dq.run(b, sq, sk, h, hk, causal, bf16, seed=0, text=dq_text, verbose=False)
    assert e <= (1e-2 if bf16 else 2e-3), e


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,grid", [
    (1, 600, 600, 2, 1, True, 1),       # one workgroup walks 6 items (3 query blocks x 2 heads)
    (2, 300, 200, 4, 2, False, 3),      # 16 items over 3 workgroups, snake rounds
])
def test_asm_dq_persistent_loop(dq_text, b, sq, sk, h, hk, causal, grid):
    import emu_dq
    e, *_ = emu_dq.run(b, sq, sk, h, hk, causal, True, seed=4, text=dq_text, verbose=False, grid=grid)
    assert e <= 1e-2, e


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16", [
    (1, 330, 200, 2, 1, True, True),            # GQA, ragged last group (rows past seqlen_q: zero scratch)
    (1, 96, 300, 3, 1, True, False),            # fp16 (v_dot2_f32_f16)
])
def test_asm_dq_fused_pre_in_emulator(dq_text, b, sq, sk, h, hk, causal, bf16):
    """flags bit 1 (knob 8): the dQ kernel computes D = rowsum(dO o O) itself (bwd_pre_kernel's work):
    the softmax_d input is NaN, the outputs softmax_d and the dK/dV scratch are checked too"""
    import emu_dq
    e, *_ = emu_dq.run(b, sq, sk, h, hk, causal, bf16, seed=2, text=dq_text, verbose=False, fused=True)
    assert e <= (1e-2 if bf16 else 2e-3), e


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16,grid", [
    (1, 330, 200, 2, 1, True, True, None),      # GQA, ragged last group (Q' rows past seqlen_q not stored)
    (2, 130, 200, 2, 2, False, False, None),    # fp16 (v_cvt_f32_f16 unpack)
    (1, 600, 600, 2, 1, True, True, 2),         # persistent: 6 items over 2 workgroups (fold state per item)
])
def test_asm_dq_q_fold_in_emulator(dq_text, b, sq, sk, h, hk, causal, bf16, grid):
    """flags bit 2 (the backward of the folded forward, launch_bwd): the dQ kernel rewrites its Q
    fragments as bf16/f16(c Q) and stores them for dK/dV -- compared bitwise with the forward's
    rounding -- then scores with c = 1; dQ against float64 on that Q'"""
    import emu_dq
    e, *_ = emu_dq.run(b, sq, sk, h, hk, causal, bf16, seed=6, text=dq_text, verbose=False, fused=True, qfold=True,
                       grid=grid)
    assert e <= (1e-2 if bf16 else 2e-3), e


def test_generated_dq_kernels_assemble_shape():
    text = subprocess.run([sys.executable, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_dq.py")],
                          check=True, capture_output=True, text=True).stdout
    assert text.count(".amdhsa_kernel ") == 4
    assert ".amdhsa_group_segment_fixed_size 147456" in text
    lines = [x.strip() for x in text.splitlines()]
    for i, x in enumerate(lines):
        if x.startswith("buffer_load_dword") and x.endswith(" lds"):
            prev = lines[i - 1]
            assert not prev.startswith("s_add_u32 m0") and not prev.startswith("s_mov_b32 m0"), (i, prev)


# ------------------------------------------------------------------------------------------------
# the dK / dV kernel with two waves per SIMD (csrc/asm/gen_bwd2.py, knob 10): 8 waves by role, P
# crossing from the P waves to the dS waves through LDS once per phase.  Same cases as above,
# bitwise against the one-wave kernel, the waves run in both orders between barriers, and the
# emulator's race checker on: no wave touches LDS bytes another wave writes (ds_write or in-flight
# LDS-DMA) between the same two barriers.
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def asm2_text():
    return emu_bwd.asm_text(2)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16,reduce,grid,order", [
    (1, 64, 128, 1, 1, True, True, False, None, None),
    (1, 200, 330, 2, 1, True, True, True, None, "reverse"),
    (1, 257, 129, 1, 1, False, False, False, None, "reverse"),
    (2, 160, 160, 2, 1, True, True, True, 3, None),      # persistent loop, several items per workgroup
])
def test_asm_dkdv_two_waves_in_emulator(asm_text, asm2_text, b, sq, sk, h, hk, causal, bf16, reduce, grid, order):
    r1 = emu_bwd.run(b, sq, sk, h, hk, causal, bf16, reduce, seed=3, text=asm_text, verbose=False, grid=grid)
    r2 = emu_bwd.run(b, sq, sk, h, hk, causal, bf16, reduce, seed=3, text=asm2_text, verbose=False, grid=grid,
                     ver=2, order=order)
    assert not emu_bwd.RACES, emu_bwd.RACES[:3]
    assert (r1[2] == r2[2]).all() and (r1[4] == r2[4]).all()
    assert max(r2[0], r2[1]) < 1e-2


@pytest.mark.timeout(900)
def test_asm_dkdv_two_waves_varlen_in_emulator(asm2_text):
    ek, ev, *_ = emu_bwd.run(lens=[130, 0, 1, 257], h=2, hk=1, causal=True, text=asm2_text, verbose=False, ver=2)
    assert not emu_bwd.RACES, emu_bwd.RACES[:3]
    assert max(ek, ev) < 1e-2


# ------------------------------------------------------------------------------------------------
# head dim 64 (csrc/asm/gen_bwd64.py): 4 waves x 64 keys (two 32-key groups a wave sharing every A
# fragment), 256-key blocks, 2-piece subtile DMA; against the float64 restatement, race checker on
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def asm64_text():
    return emu_bwd.asm_text(64)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16,reduce,grid,unit_c", [
    (1, 64, 256, 1, 1, True, True, False, None, False),     # one step: first + last + masked
    (1, 300, 300, 2, 1, True, True, True, None, False),     # GQA reduce across a head boundary
    (1, 40, 600, 1, 1, False, True, False, None, False),    # three key blocks, the last ragged
    (1, 333, 257, 4, 2, False, False, True, None, True),    # fp16, c = 1 (the folded backward)
    (2, 300, 700, 2, 1, True, True, True, 3, False),        # persistent loop
    (1, 600, 40, 2, 2, True, True, False, None, False),     # keys fewer than a group
])
def test_asm_dkdv_d64_in_emulator(asm64_text, b, sq, sk, h, hk, causal, bf16, reduce, grid, unit_c):
    ek, ev, *_ = emu_bwd.run(b, sq, sk, h, hk, causal, bf16, reduce, seed=1, text=asm64_text, verbose=False,
                             grid=grid, unit_c=unit_c, ver=64)
    assert not emu_bwd.RACES, emu_bwd.RACES[:3]
    assert max(ek, ev) < (1e-2 if bf16 else 2e-3), (ek, ev)


@pytest.mark.timeout(900)
def test_asm_dkdv_d64_varlen_in_emulator(asm64_text):
    ek, ev, *_ = emu_bwd.run(lens=[130, 0, 1, 557], h=2, hk=1, causal=True, text=asm64_text, verbose=False, ver=64)
    assert not emu_bwd.RACES, emu_bwd.RACES[:3]
    assert max(ek, ev) < 1e-2


# ------------------------------------------------------------------------------------------------
# head dim 64 dQ (csrc/asm/gen_dq64.py: gen_dq.py's kernel at d = 64, one K and one V DMA piece a
# wave per subtile), against the float64 dQ of tools/emu_dq.py
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def dq64_text():
    import emu_dq
    return emu_dq.asm_text(64)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b,sq,sk,h,hk,causal,bf16,grid,fused,qfold", [
    (1, 64, 64, 1, 1, True, True, None, False, False),         # one step: first + last + masked
    (1, 330, 200, 2, 1, True, True, None, False, False),       # GQA, sq > sk
    (2, 130, 77, 2, 1, False, True, None, False, False),       # full attention, ragged
    (1, 96, 300, 3, 1, True, False, None, True, False),        # fp16, fused D (v_dot2 over 16 registers)
    (1, 330, 200, 2, 1, True, True, None, True, True),         # the Q fold (Q' stored bitwise)
    (1, 600, 600, 2, 1, True, True, 2, True, True),            # persistent loop, fold state per item
])
def test_asm_dq_d64_in_emulator(dq64_text, b, sq, sk, h, hk, causal, bf16, grid, fused, qfold):
    import emu_dq
    e, *_ = emu_dq.run(b, sq, sk, h, hk, causal, bf16, seed=5, text=dq64_text, verbose=False, grid=grid,
                       fused=fused, qfold=qfold, d=64)
    assert e <= (1e-2 if bf16 else 2e-3), e


def test_generated_dq64_kernels_assemble_shape():
    text = subprocess.run([sys.executable, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm", "gen_dq64.py")],
                          check=True, capture_output=True, text=True).stdout
    assert text.count(".amdhsa_kernel fa_bwd_dq_asm_d64_") == 8      # (+ the c = 1 kernels)
    assert ".amdhsa_group_segment_fixed_size 73728" in text


@pytest.mark.timeout(900)
@pytest.mark.parametrize("d,sq,sk,causal", [(64, 1, 1, False), (128, 17, 17, False), (64, 130, 77, True)])
def test_asm_dq_fp16_large_scores(d, sq, sk, causal):
    """fp16, |LSE| large (Q x 5, K / V x 3): the keys past seqlen_k in the last step (zero K / V)
    must get P = 0, or P dS overflows the fp16 dS pack and 0 x inf puts NaN into dQ (found on the GPU
    by test_flash_attn_bwd_overflow at d = 64)"""
    import emu_dq
    _, dq, ref = emu_dq.run(2, sq, sk, 2, 2, causal, False, seed=1, verbose=False, d=d, qmul=5, kmul=3,
                            text=emu_dq.asm_text(d))
    assert np.isfinite(dq).all()
    assert np.abs(dq - ref).max() <= 2e-3 * max(1.0, np.abs(ref).max())
