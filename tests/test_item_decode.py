"""CPU checks of the assembly kernels' in-kernel work order (fa_params.h ItemDecode,
csrc/asm/isa.py item_decode_ops), which replaced the per-shape host tables:

1. the magic-number division is exact for every n < 2^31 on edge and random divisors;
2. the decoded orders equal the work orders the host tables used to hold (fa_common.h xcd_order /
   xcd_order_grouped, restated here as the former table builders), for the forward / dQ
   (head-fastest and XCD-grouped) and for dK / dV (XCD-major and not);
3. the SALU sequence itself, executed by the functional emulator (tools/asm_emu.py), gives the
   same items as the Python restatement;
4. whole kernels in the emulator with the XCD-grouped order (the C5-style launch).
"""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xhy-flash-attention_amd", "csrc", "asm"))

import isa  # noqa: E402


def test_magic_division_exact():
    rng = random.Random(0)
    divs = list(range(1, 1500)) + [2 ** k for k in range(31)] + [2 ** k + 1 for k in range(31)] + \
        [2 ** k - 1 for k in range(1, 32)] + [rng.randrange(1, 2 ** 31) for _ in range(1000)]
    for d in divs:
        mag, sh = isa.magic_div(d)
        assert 0 < mag < 2 ** 32 and 31 <= sh <= 62
        for n in (0, 1, d - 1, d, d + 1, 2 * d - 1, 2 ** 31 - 1, 2 ** 31 - 2, rng.randrange(2 ** 31)):
            if 0 <= n < 2 ** 31:
                assert (n * mag) >> sh == n // d, (n, d)


def fwd_table(b, h, hk, nmb, hp):
    """the former host table of the forward / dQ (fa_common.h xcd_order_grouped, heaviest first)"""
    nbh, g, out = b * h, h // hk, []
    for L in range(nbh * nmb):
        if nbh % 8 == 0 and hp > 0 and (nbh >> 3) % hp == 0:
            i = L >> 3
            pg = hp * nmb
            gi, r = divmod(i, pg)
            blk = r // hp
            bh = (gi * hp + r - blk * hp) * 8 + (L & 7)
        else:
            blk, bh = divmod(L, nbh)
        bidb, head = divmod(bh, h)
        out.append((nmb - 1 - blk, bidb, head, head // g))
    return out


def dkdv_table(b, nh, h, hk, nblk, reduce):
    """the former host table of dK / dV (fa_common.h xcd_order)"""
    nbh, g, out = b * nh, h // hk, []
    for L in range(nbh * nblk):
        if nbh % 8 == 0:
            hl, blk = divmod(L >> 3, nblk)
            bh = hl * 8 + (L & 7)
        else:
            blk, bh = divmod(L, nbh)
        bidb, hx = divmod(bh, nh)
        out.append((blk, bidb, hx, hx if reduce else hx // g))
    return out


@pytest.mark.parametrize("b,h,hk,nmb,hp", [(4, 16, 16, 32, 0), (8, 32, 8, 128, 2), (8, 32, 8, 128, 4),
                                           (3, 5, 1, 7, 0), (1, 8, 2, 3, 1), (2, 8, 8, 5, 2), (1, 1, 1, 1, 0)])
def test_forward_order(b, h, hk, nmb, hp):
    dec = isa.fwd_item_decode(b * h, h, h // hk, nmb, hp)
    want = fwd_table(b, h, hk, nmb, hp)
    for L, w in enumerate(want):
        blk, nb1, bidb, head, kvh = isa.item_decode_ref(L, dec)
        assert (nb1 - blk, bidb, head, kvh) == w, L


@pytest.mark.parametrize("b,nh,h,hk,nblk,red", [(4, 16, 16, 16, 64, False), (8, 8, 32, 8, 256, True),
                                                (8, 32, 32, 8, 256, False), (3, 5, 5, 1, 7, False),
                                                (1, 3, 6, 3, 9, True)])
def test_dkdv_order(b, nh, h, hk, nblk, red):
    dec = isa.dkdv_item_decode(b * nh, nh, 1 if red else h // hk, nblk)
    want = dkdv_table(b, nh, h, hk, nblk, red)
    for L, w in enumerate(want):
        blk, _, bidb, head, kvh = isa.item_decode_ref(L, dec)
        assert (blk, bidb, head, kvh) == w, L


def test_salu_sequence_in_emulator():
    """item_decode_ops on the emulator's SALU: s[2] = L, s[40:49] = the decode dwords"""
    from asm_emu import Emu, Heap, Wave, parse_kernel

    ops = isa.item_decode_ops(L=2, M=40, pa=32, pb=34, t=36, u=37, o_blk=29, reverse=True)
    text = "\t.globl k\n\t.type k,@function\nk:\n" + "\n".join("\t" + o.text for o in ops) + "\n\ts_endpgm\n.Lk_fend:\n"
    insts, _ = parse_kernel(text, "k")
    emu = Emu(text, "k", Heap(1 << 16))
    rng = random.Random(1)
    for (b, h, hk, nmb, hp) in [(8, 32, 8, 128, 2), (3, 5, 1, 7, 0), (64, 32, 8, 128, 4), (4, 16, 16, 32, 0)]:
        dec = isa.fwd_item_decode(b * h, h, h // hk, nmb, hp)
        n = b * h * nmb
        for L in sorted({0, 1, 7, 8, n - 1, n - 8} | {rng.randrange(n) for _ in range(200)}):
            if not 0 <= L < n:
                continue
            w = Wave(0)
            w.s[2] = L
            w.s[40:50] = np.array(dec, dtype=np.uint32)
            for op, a, mods, _t in insts:
                if op == "s_endpgm":
                    break
                emu.exec(w, None, op, a, mods)
            got = (int(w.s[29]), int(w.s[34]), int(w.s[37]), int(w.s[32]))
            blk, nb1, bidb, head, kvh = isa.item_decode_ref(L, dec)
            assert got == (nb1 - blk, bidb, head, kvh), (b, h, hk, nmb, hp, L)


@pytest.mark.timeout(600)
def test_forward_grouped_order_in_emulator():
    """the forward over the XCD-grouped order (hp = 1: b h = 8 heads in one group)"""
    import emu_fwd

    eo, el, *_ = emu_fwd.run(1, 300, 300, 8, 2, True, True, seed=2, verbose=False, d=64, hp=1)
    assert eo <= 1.6e-2 and el <= 1e-5, (eo, el)
    # ... and walked by a persistent grid of 4 workgroups (snake rounds over the grouped list)
    eo, el, *_ = emu_fwd.run(1, 600, 600, 8, 2, True, True, seed=5, verbose=False, d=64, hp=1, grid=4)
    assert eo <= 1.6e-2 and el <= 1e-5, (eo, el)


@pytest.mark.timeout(600)
def test_dq_grouped_order_in_emulator():
    import emu_dq

    e, _, _ = emu_dq.run(1, 260, 260, 8, 2, True, True, seed=3, verbose=False, hp=1)
    assert e <= 2e-2, e
    e, _, _ = emu_dq.run(1, 520, 520, 8, 2, True, True, seed=6, verbose=False, hp=1, grid=3)
    assert e <= 2e-2, e
