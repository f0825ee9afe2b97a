"""ORACLE -- test infrastructure only (the checker for the dropout path; never imported by the product).

CPU restatement of the reference's attention-dropout random stream, so that tests can check the
keep/drop pattern of the MI355X kernels element by element:

* Philox counter RNG, ``flash::philox`` (reference csrc/flash_attn/src/philox.cuh:8-47): key =
  seed (two 32-bit words), counter = (offset, subsequence) as two 64-bit halves; 6 rounds with the
  key bumped by (0x9E3779B9, 0xBB67AE85) after each, then one final round -- 7 rounds in all; a
  round is  (hi(B*c2) ^ c1 ^ k0, lo(B*c2), hi(A*c0) ^ c3 ^ k1, lo(A*c0)),  A = 0xD2511F53,
  B = 0xCD9E8D57.
* Element -> random byte (``flash::apply_dropout``, softmax.h:380-447, called with
  block_row_idx = row / 16, block_col_idx = col / 32, flash_fwd_kernel.h:417-432 and
  flash_bwd_kernel.h:848-857): one Philox call per (16-row x 32-column block, CUDA lane), with
  subsequence = (row/16) | (col/32) << 32 and offset = base + (batch * nheads + head) * 32 + lane
  (flash_fwd_kernel.h:316-318).  Inside the block, lane = 4 * (r % 8) + (c % 8) / 2 holds the
  m16n8k16 A-register group ((2 cols, 2 row halves, 2 eight-column halves), utils.h:242-257), so
  element (r, c) takes byte  8 * (c // 16) + (c % 2) + 2 * (r // 8) + 4 * ((c % 16) // 8)  of the
  16 little-endian output bytes.
* keep  <=>  byte <= floor((1 - p_dropout) * 255)   (flash_api.cpp:94-100, softmax.h:436).

The reference code is CUDA and cannot run here, so this restatement is the pin: the kernels'
returned S_dmask sign pattern must equal ``dropout_keep_mask`` bit for bit.
"""
import numpy as np

__all__ = ["philox", "dropout_keep_mask", "keep_threshold"]

_M32 = np.uint64(0xFFFFFFFF)
_A = np.uint64(0xD2511F53)
_B = np.uint64(0xCD9E8D57)
_KA = np.uint64(0x9E3779B9)
_KB = np.uint64(0xBB67AE85)


def _round(c0, c1, c2, c3, k0, k1):
    p0 = _A * c0          # products of two 32-bit values fit in uint64
    p1 = _B * c2
    return ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & _M32, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & _M32)


def philox(seed, subsequence, offset):
    """Vectorised flash::philox -> (x, y, z, w) uint32 words (as uint64 arrays)."""
    seed = np.uint64(seed)
    sub = np.asarray(subsequence, dtype=np.uint64)
    off = np.asarray(offset, dtype=np.uint64)
    sub, off = np.broadcast_arrays(sub, off)
    k0 = np.full(sub.shape, seed & _M32, dtype=np.uint64)
    k1 = np.full(sub.shape, seed >> np.uint64(32), dtype=np.uint64)
    c = (off & _M32, off >> np.uint64(32), sub & _M32, sub >> np.uint64(32))
    for _ in range(6):
        c = _round(*c, k0, k1)
        k0 = (k0 + _KA) & _M32
        k1 = (k1 + _KB) & _M32
    return _round(*c, k0, k1)


def keep_threshold(p_dropout):
    """uint8 threshold of the reference: floor(keep_prob * 255) (flash_api.cpp:94-100)."""
    keep = np.float32(1.0) - np.float32(p_dropout)      # params.p_dropout = 1.f - p_dropout (float)
    return int(np.floor(float(keep) * 255.0))          # uint8_t(std::floor(p * 255.0)) (double)


def dropout_keep_mask(seed, offset, batch_idx, head_idx, nheads, seqlen_q, seqlen_k, p_dropout):
    """bool (seqlen_q, seqlen_k): True where the element of (batch_idx, head_idx) is kept."""
    r = np.arange(seqlen_q, dtype=np.int64)[:, None]
    c = np.arange(seqlen_k, dtype=np.int64)[None, :]
    rr, cc = r % 16, c % 32
    lane = 4 * (rr % 8) + (cc % 8) // 2
    byte_idx = 8 * (cc // 16) + (cc % 2) + 2 * (rr // 8) + 4 * ((cc % 16) // 8)
    sub = (r // 16).astype(np.uint64) | ((c // 32).astype(np.uint64) << np.uint64(32))
    off = np.uint64(offset) + np.uint64((batch_idx * nheads + head_idx) * 32) + lane.astype(np.uint64)
    words = philox(seed, sub, off)
    w = np.select([byte_idx // 4 == i for i in range(4)], list(words))
    byte = (w >> (8 * (byte_idx % 4)).astype(np.uint64)) & np.uint64(0xFF)
    return byte <= np.uint64(keep_threshold(p_dropout))
