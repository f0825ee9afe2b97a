"""CPU checks of the dropout oracle (oracle/dropout_ref.py), the checker of the GPU dropout tests."""
import numpy as np

from oracle.dropout_ref import dropout_keep_mask, keep_threshold, philox


def test_keep_threshold_matches_reference_formula():
    # flash_api.cpp:94-100: p = 1.f - p_dropout; uint8_t(std::floor(p * 255.0))
    for p, t in [(0.0, 255), (0.1, 229), (0.17, 211), (0.5, 127), (0.9, 25)]:
        assert keep_threshold(p) == t


def test_philox_is_deterministic_and_keyed():
    a = philox(1234, np.arange(8, dtype=np.uint64), 7)
    b = philox(1234, np.arange(8, dtype=np.uint64), 7)
    c = philox(1235, np.arange(8, dtype=np.uint64), 7)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not all(np.array_equal(x, y) for x, y in zip(a, c))
    assert all(int(x.max()) < 2 ** 32 for x in a)


def test_element_map_is_a_bijection_per_block():
    # within a 16 x 32 block every (lane, byte) pair is used by exactly one element
    r = np.arange(16)[:, None]
    c = np.arange(32)[None, :]
    lane = 4 * (r % 8) + (c % 8) // 2
    byte = 8 * (c // 16) + (c % 2) + 2 * (r // 8) + 4 * ((c % 16) // 8)
    keys = (lane * 16 + byte).ravel()
    assert len(set(keys.tolist())) == 512 and keys.min() == 0 and keys.max() == 511


def test_mask_rate_and_independence():
    m = dropout_keep_mask(42, 0, 0, 0, 1, 512, 512, 0.3)
    assert abs(m.mean() - (keep_threshold(0.3) + 1) / 256) < 0.01
    m2 = dropout_keep_mask(42, 0, 0, 1, 2, 512, 512, 0.3)     # another head: another stream
    m3 = dropout_keep_mask(42, 64, 0, 0, 1, 512, 512, 0.3)    # another offset
    assert (m != m2).mean() > 0.3 and (m != m3).mean() > 0.3
    # a sub-block is the top-left corner of the larger mask (the stream depends on (row, col) only)
    assert np.array_equal(dropout_keep_mask(42, 0, 0, 0, 1, 100, 70, 0.3), m[:100, :70])


def test_philox_known_answers():
    """The reference's flash::philox (philox.cuh:27-47: 6 keyed rounds with key bumps + a final
    round) is Philox4x32 with R = 7.  Known-answer vectors published with the Random123 library
    (kat_vectors, "philox4x32 7 <ctr x4> <key x2> <out x4>"); ctr = (offset lo, offset hi,
    subsequence lo, subsequence hi), key = (seed lo, seed hi)."""
    def words(seed, sub, off):
        return [int(x) for x in philox(seed, np.uint64(sub), np.uint64(off))]

    assert words(0, 0, 0) == [0x5f6fb709, 0x0d893f64, 0x4f121f81, 0x4f730a48]
    ctr = [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344]
    key = [0xa4093822, 0x299f31d0]
    assert words(key[0] | key[1] << 32, ctr[2] | ctr[3] << 32, ctr[0] | ctr[1] << 32) == \
        [0x4dfccaba, 0x190a87f0, 0xc47362ba, 0xb6b5242a]


def _reference_apply_dropout_keep(seed, offset, bh, nheads_total_unused, m_block, n_block, kBlockM, kBlockN,
                                  kNWarps, p_dropout):
    """Element-by-element simulation of the reference's dropout, derived from the SM80 MMA layouts
    (independently of dropout_keep_mask's closed form):
      * m16n8k16 accumulator fragment of lane l (CUTLASS SM80_16x8x16_F32BF16BF16F32_TN C layout):
        c[2*i0 + j0] holds (row l/4 + 8*i0, col 2*(l%4) + j0) of the 16x8 tile;
      * rowcol layout ((2, MMA_M), (2, MMA_N)) of those registers, re-tiled by
        convert_layout_rowcol_Aregs (utils.h:241-257) to ((2, 2, 2), MMA_M, MMA_N/2): element i of
        mode 0 is (j0 = i % 2, i0 = (i/2) % 2, t = i/4), 8-column tile 2*nn + t;
      * apply_dropout (softmax.h:381-447): per (m, n) one philox(seed, (row_blk, col_blk), offset +
        lane) with row_blk = m_block*kBlockM/16 + warp + m*kNWarps, col_blk = n_block*kBlockN/32 + n;
        byte j*8 + i goes to tensor(i, m, 2n + j);
      * offset = rng offset + bh * 32 + lane (flash_fwd_kernel.h:316-318).
    Returns keep[kBlockM][kBlockN] of the (m_block, n_block) tile."""
    keep_u8 = int(np.floor(float(np.float32(1.0) - np.float32(p_dropout)) * 255.0))
    keep = np.zeros((kBlockM, kBlockN), dtype=bool)
    seen = np.zeros((kBlockM, kBlockN), dtype=int)
    mma_m = kBlockM // (16 * kNWarps)
    mma_n = kBlockN // 8
    for warp in range(kNWarps):
        for lane in range(32):
            for m in range(mma_m):
                row_blk = m_block * (kBlockM // 16) + warp + m * kNWarps
                for n in range(mma_n // 4):
                    col_blk = n_block * (kBlockN // 32) + n
                    w = philox(seed, np.uint64(row_blk | (col_blk << 32)), np.uint64(offset + bh * 32 + lane))
                    rnd = [(int(w[b // 4]) >> (8 * (b % 4))) & 0xFF for b in range(16)]
                    for j in range(2):
                        nn = 2 * n + j
                        for i in range(8):
                            j0, i0, t = i % 2, (i // 2) % 2, i // 4
                            tile8 = 2 * nn + t
                            row = (row_blk - m_block * (kBlockM // 16)) * 16 + lane // 4 + 8 * i0
                            col = tile8 * 8 + 2 * (lane % 4) + j0
                            keep[row, col] = rnd[j * 8 + i] <= keep_u8
                            seen[row, col] += 1
    assert (seen == 1).all()          # the simulation covers every element of the tile exactly once
    return keep


def test_element_byte_map_matches_mma_layout_derivation():
    """dropout_keep_mask (the closed form the GPU tests compare the kernels with) equals the
    element-by-element simulation of the reference's loop over the MMA fragment layouts, for the
    reference's forward tile shapes (hdim 128: 128 x 64, 4 warps; hdim 64: 128 x 128, 4 warps)."""
    seed, offset, p = 0x1234_5678_9abc, 24, 0.17
    h, bidb, bidh = 3, 1, 2
    bh = bidb * h + bidh
    for (bm, bn, nw) in ((128, 64, 4), (128, 128, 4), (64, 128, 4)):
        for (mb, nb) in ((0, 0), (1, 2)):
            sim = _reference_apply_dropout_keep(seed, offset, bh, None, mb, nb, bm, bn, nw, p)
            full = dropout_keep_mask(seed, offset, bidb, bidh, h, (mb + 1) * bm, (nb + 1) * bn, p)
            assert np.array_equal(sim, full[mb * bm:(mb + 1) * bm, nb * bn:(nb + 1) * bn]), (bm, bn, mb, nb)
