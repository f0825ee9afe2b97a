"""The dropout kernels' byte exchange (csrc/fa_dropout.h, round 5), simulated on the host lane by lane
against the reference's element -> (call, byte) map (oracle/dropout_ref.py, after the reference's
softmax.h:380-447 / philox.cuh:27-47): whatever calls a lane runs and however the words travel
between lanes, every lane must end with exactly the bytes of the scores its MFMA fragment holds.

* forward / dQ (dropout_lane_bytes): lane (r, hh) holds keys 8u + 4hh + b (b < 4) of query r; lanes
  r and r ^ 8 run one call each, swap words over the 16-lane DPP row (row_ror:8) and assemble with
  v_perm_b32 and a per-lane selector;
* dK/dV (dropout_block_words / dropout_col_bytes): lane (c, hh) holds queries 8u + 4hh + j of key c;
  call words go through LDS as [row block][word][t][g] dwords, read back as one 16-byte vector per
  row block and picked apart by v_perm_b32.
"""
import numpy as np
import pytest

from oracle.dropout_ref import philox


def _words(seed, off_bh, row0, col0):
    """words[R][L] = the 4 uint32 words of the call of 16-row block R, lane L of the 32 x 32 block"""
    R = np.arange(2, dtype=np.uint64)[:, None]
    L = np.arange(32, dtype=np.uint64)[None, :]
    sub = (np.uint64(row0 // 16) + R) | (np.uint64(col0 // 32) << np.uint64(32))
    w = philox(seed, sub + L * np.uint64(0), np.uint64(off_bh) + L + R * np.uint64(0))
    return np.stack([np.asarray(x, dtype=np.uint64) for x in w], axis=-1)   # (2, 32, 4)


def _ref_byte(words, r32, c):
    """the reference's byte of element (row r32, column c) of the block"""
    R, rr = r32 // 16, r32 % 16
    L = 4 * (rr % 8) + (c % 8) // 2
    b = 8 * (c // 16) + (c % 2) + 2 * (rr // 8) + 4 * ((c % 16) // 8)
    return int(words[R, L, b // 4] >> np.uint64(8 * (b % 4))) & 0xFF


def _perm(s0, s1, sel):
    """v_perm_b32: byte i of the result = byte sel_i of {s0 (bytes 4-7) : s1 (bytes 0-3)}"""
    pool = [(s1 >> (8 * k)) & 0xFF for k in range(4)] + [(s0 >> (8 * k)) & 0xFF for k in range(4)]
    return sum(pool[(sel >> (8 * k)) & 0xFF] << (8 * k) for k in range(4))


@pytest.mark.parametrize("seed,offset,bh,row0,col0", [(0, 0, 0, 0, 0), (1234567, 4096, 5, 64, 96),
                                                       (2**63 + 77, 2**40 - 3, 31, 8160, 8128)])
def test_forward_lane_pair_exchange(seed, offset, bh, row0, col0):
    off_bh = offset + bh * 32
    words = _words(seed, off_bh, row0, col0)
    own = {}
    for lane in range(64):   # the call each lane runs
        r, hh = lane & 31, lane >> 5
        up = (r >> 3) & 1
        own[lane] = [int(x) for x in words[r >> 4, 4 * (r & 7) + 2 * hh + up]]
    for lane in range(64):
        r, hh = lane & 31, lane >> 5
        sel = 0x07060302 if (r >> 3) & 1 else 0x01000504
        partner = lane ^ 8                    # row_ror:8 inside the 16-lane row
        assert partner // 16 == lane // 16
        for u in range(4):
            rb = _perm(own[lane][u], own[partner][u], sel)
            for b in range(4):
                assert (rb >> (8 * b)) & 0xFF == _ref_byte(words, r, 8 * u + 4 * hh + b), (lane, u, b)


@pytest.mark.parametrize("seed,offset,bh,row0,col0", [(0, 0, 0, 0, 0), (987654321, 64, 3, 32, 4064),
                                                       (2**64 - 1, 2**50, 17, 96, 0)])
def test_dkdv_word_exchange(seed, offset, bh, row0, col0):
    off_bh = offset + bh * 32
    words = _words(seed, off_bh, row0, col0)
    lds = {}
    for lane in range(64):   # dropout_block_words: lane = (row block R, call lane L = 4g + t)
        R, L = lane >> 5, lane & 31
        g, t = L >> 2, L & 3
        for i in range(4):
            addr = ((4 * R + i) * 4 + t) * 8 + g
            assert addr not in lds
            lds[addr] = int(words[R, L, i])
    assert sorted(lds) == list(range(256))
    # a dword store per word index: the 32 lanes of a half write 32 distinct consecutive dwords
    for R in range(2):
        for i in range(4):
            addrs = sorted(((4 * R + i) * 4 + (L & 3)) * 8 + (L >> 2) for L in range(32))
            assert addrs == list(range(addrs[0], addrs[0] + 32))
    for lane in range(64):   # dropout_col_bytes: lane = (key c, hh)
        c, hh = lane & 31, lane >> 5
        sel_pair = 0x07030501 if c & 1 else 0x06020400
        rb = [0] * 4
        for R in range(2):
            base = ((4 * R + (c >> 3)) * 4 + ((c & 7) >> 1)) * 8 + 4 * hh
            assert base % 4 == 0             # one 16-byte aligned ds_read_b128
            v = [lds[base + j] for j in range(4)]
            t01, t23 = _perm(v[1], v[0], sel_pair), _perm(v[3], v[2], sel_pair)
            rb[2 * R], rb[2 * R + 1] = _perm(t23, t01, 0x05040100), _perm(t23, t01, 0x07060302)
        for u in range(4):
            for j in range(4):
                assert (rb[u] >> (8 * j)) & 0xFF == _ref_byte(words, 8 * u + 4 * hh + j, c), (lane, u, j)


def test_block_bytes_are_the_oracle_mask():
    """_ref_byte is the oracle's map: the keep mask of block (0, 0) from it equals dropout_keep_mask"""
    from oracle.dropout_ref import dropout_keep_mask, keep_threshold

    seed, offset, bh, p = 42, 1 << 20, 3, 0.17
    words = _words(seed, offset + bh * 32, 0, 0)
    thr = keep_threshold(p)
    mine = np.array([[_ref_byte(words, r, c) <= thr for c in range(32)] for r in range(32)])
    assert np.array_equal(mine, dropout_keep_mask(seed, offset, 0, bh, bh + 1, 32, 32, p))
