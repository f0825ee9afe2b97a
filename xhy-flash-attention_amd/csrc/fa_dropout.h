// Attention dropout for the MI355X kernels: the reference's random stream, element for element.
//
// The reference (csrc/flash_attn/src/philox.cuh:27-47, softmax.h:380-447, flash_fwd_kernel.h:316-318
// and :417-432, flash_bwd_kernel.h:848-857) draws one Philox call per (16-row x 32-column block,
// CUDA lane): subsequence = (row / 16) | (col / 32) << 32, offset = base + (batch * h + head) * 32
// + lane, and element (r, c) of the block (r < 16, c < 32) takes byte
//     8 * (c / 16) + (c % 2) + 2 * (r / 8) + 4 * ((c % 16) / 8)     of lane 4 * (r % 8) + (c % 8) / 2
// (the m16n8k16 A-register order of the SM80 MMA).  The element keeps iff byte <= keep_u8.
// The mapping is a function of the global (row, col) only, so the MI355X kernels -- whose MFMA
// fragments hold the elements in a different order -- reproduce the same keep/drop pattern:
//   * one wave covers a 32 x 32 block (two 16-row blocks x one 32-column block = 2 x 32 Philox
//     calls), i.e. exactly one call per lane;
//   * each lane scatters its 16 bytes into a 1-KiB per-wave LDS scratch laid out [row][col]
//     (or [col][row]), and reads back the 4-byte groups its accumulator fragment owns.
// oracle/dropout_ref.py restates the same stream on the host; tests compare the kernels' sign-encoded
// S_dmask with it bit for bit.
#pragma once

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

// The scratch is written with 8/16-bit stores and read back with 32-bit loads: may_alias types keep
// the compiler (type-based alias analysis) from hoisting the loads above the stores.
typedef unsigned short __attribute__((may_alias)) u16_alias;
typedef unsigned __attribute__((may_alias)) u32_alias;
typedef unsigned char __attribute__((may_alias)) u8_alias;

// flash::philox (reference philox.cuh:27-47): 6 rounds with key bumps, then a final round.
__device__ inline u32x4_t philox(uint64_t seed, uint64_t subsequence, uint64_t offset) {
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
  unsigned c0 = (unsigned)offset, c1 = (unsigned)(offset >> 32);
  unsigned c2 = (unsigned)subsequence, c3 = (unsigned)(subsequence >> 32);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0;
    const unsigned n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (unsigned)p1; c2 = n2; c3 = (unsigned)p0;
    if (i < 6) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
  }
  u32x4_t r = {c0, c1, c2, c3};
  return r;
}

// (seed, offset) of the stream: the device rng_state when the launcher passes one (AttnShape::
// philox_dev, backward), else the host values.  Read once per workgroup (scalar loads).
template <typename Shape>
__device__ inline uint64_t philox_seed_of(const Shape& s) {
  return s.philox_dev != nullptr ? s.philox_dev[0] : s.philox_seed;
}
template <typename Shape>
__device__ inline uint64_t philox_offset_of(const Shape& s) {
  return s.philox_dev != nullptr ? s.philox_dev[1] : s.philox_offset;
}

// This wave's 32 x 32 block of dropout bytes -- rows row0 .. row0+31 (queries), columns col0 ..
// col0+31 (keys), both multiples of 32 and relative to the sequence -- into the wave's 1-KiB LDS
// scratch `buf`, laid out [row][col] (TRANS = false) or [col][row] (TRANS = true).
// off_bh = philox offset + (batch * h + head) * 32.
template <bool TRANS>
__device__ inline void dropout_block_bytes(char* buf, uint64_t seed, uint64_t off_bh, int row0,
                                           int col0, int lane) {
  const int half = lane >> 5, L = lane & 31;
  // The scratch is reused block after block by the same wave, and an LDS store of this wave can
  // overtake its own earlier, still-pending LDS load of the same address (measured on gfx950: the
  // next block's bytes leaked into the previous block's reads).  So: drain this wave's LDS
  // operations before overwriting the scratch, and again before the caller reads it back.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint64_t sub = (uint64_t)(unsigned)(row0 / 16 + half) | ((uint64_t)(unsigned)(col0 / 32) << 32);
  const u32x4_t w = philox(seed, sub, off_bh + (uint64_t)L);
  const int g = L >> 2, t = L & 3;
#pragma unroll
  for (int b = 0; b < 16; b += 2) {
    const int j = b >> 3, i = b & 7;                    // i even: bytes b, b+1 are columns c, c+1
    const int r = g + 8 * ((i >> 1) & 1) + 16 * half;
    const int c = 16 * j + 2 * t + 8 * (i >> 2);
    const unsigned pair = (w[b >> 2] >> (8 * (b & 3))) & 0xffffu;
    if constexpr (TRANS) {
      *(u8_alias*)(buf + c * 32 + r) = (unsigned char)(pair & 0xff);
      *(u8_alias*)(buf + (c + 1) * 32 + r) = (unsigned char)(pair >> 8);
    } else {
      *(u16_alias*)(buf + r * 32 + c) = (unsigned short)pair;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// The same bytes without LDS: this lane's 16 dropout bytes of the wave's 32 x 32 block (rows row0 ..
// row0+31, columns col0 .. col0+31, multiples of 32) straight into the S^T accumulator order,
// rb[u] = bytes of keys col0 + 8u + 4hh + (0..3) of query row0 + r (what dropout_group_bytes reads back).
// Lane (r, hh) needs, of 16-row block r / 16, the calls of lanes 4 (r % 8) + 2hh (keys 4hh + 8u + 0, 1)
// and 4 (r % 8) + 2hh + 1 (keys + 2, 3); each of those calls also holds the same keys of row r ^ 8
// (bytes 0-1 of each word: row r % 8, bytes 2-3: row r % 8 + 8).  So the lanes r and r ^ 8 split the
// pair: the one with r & 8 == 0 runs the first call, its partner the second, and they swap words
// across the 16-lane DPP row (row_ror:8 = lane ^ 8).  One call per lane, as in dropout_block_bytes.
__device__ inline void dropout_lane_bytes(unsigned (&rb)[4], uint64_t seed, uint64_t off_bh, int row0,
                                          int col0, int lane) {
  const int r = lane & 31, hh = lane >> 5, up = (r >> 3) & 1;
  const uint64_t sub = (uint64_t)(unsigned)(row0 / 16 + (r >> 4)) | ((uint64_t)(unsigned)(col0 / 32) << 32);
  const u32x4_t w = philox(seed, sub, off_bh + (uint64_t)(4 * (r & 7) + 2 * hh + up));
  // v_perm_b32 selectors over {own word: bytes 4-7, partner word: bytes 0-3}
  const unsigned sel = up ? 0x07060302u : 0x01000504u;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const unsigned partner = (unsigned)__builtin_amdgcn_mov_dpp((int)w[u], 0x128, 0xf, 0xf, false);
    rb[u] = __builtin_amdgcn_perm(w[u], partner, sel);
  }
}

// The transposed consumer (dK/dV: lane = key c, rows 8u + 4hh + j) needs two bytes of each of eight
// calls, so the bytes still cross lanes through the wave's 1-KiB scratch, but word-wise: the lane of
// call (row block R = lane / 32, L = lane % 32 = 4g + t) stores its word w (columns 8w + 2t, +1;
// bytes: row g even / odd column, row g + 8 even / odd) at word ((4R + w) 4 + t) 8 + g -- four
// conflict-free ds_write_b32 instead of sixteen byte stores -- and the consumer of column c reads the
// words of g = 4hh .. 4hh + 3 of its (R, c / 8, c % 8 / 2) as one ds_read_b128 per row block, then
// picks its bytes with v_perm.  Same drains as dropout_block_bytes (the scratch is reused per block).
__device__ inline void dropout_block_words(char* buf, uint64_t seed, uint64_t off_bh, int row0, int col0,
                                           int lane) {
  const int R = lane >> 5, L = lane & 31, g = L >> 2, t = L & 3;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint64_t sub = (uint64_t)(unsigned)(row0 / 16 + R) | ((uint64_t)(unsigned)(col0 / 32) << 32);
  const u32x4_t w = philox(seed, sub, off_bh + (uint64_t)L);
#pragma unroll
  for (int i = 0; i < 4; ++i) *(u32_alias*)(buf + 4 * (((4 * R + i) * 4 + t) * 8 + g)) = w[i];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// rb[u] byte j = the byte of (row 8u + 4hh + j, column c = lane % 32) from dropout_block_words
__device__ inline void dropout_col_bytes(unsigned (&rb)[4], const char* buf, int lane) {
  const int c = lane & 31, hh = lane >> 5;
  // bytes (c & 1) and 2 + (c & 1) of words j = 0, 1 (resp. 2, 3) side by side
  const unsigned sel_pair = (c & 1) ? 0x07030501u : 0x06020400u;
#pragma unroll
  for (int R = 0; R < 2; ++R) {
    const u32x4_t v = *(const u32x4_t*)(buf + 4 * (((4 * R + (c >> 3)) * 4 + ((c & 7) >> 1)) * 8 + 4 * hh));
    const unsigned t01 = __builtin_amdgcn_perm(v[1], v[0], sel_pair);
    const unsigned t23 = __builtin_amdgcn_perm(v[3], v[2], sel_pair);
    rb[2 * R] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
    rb[2 * R + 1] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
  }
}

// The 4 bytes of accumulator group u (elements 4u .. 4u+3) of a 32x32 MFMA tile whose lane column
// is `r` and whose row index of element g is (g & 3) + 8 (g >> 2) + 4 hh: bytes of [r][8u + 4hh ..].
__device__ inline unsigned dropout_group_bytes(const char* buf, int r, int hh, int u) {
  return *(const u32_alias*)(buf + r * 32 + 8 * u + 4 * hh);
}

__device__ inline bool dropout_keep(unsigned bytes4, int k, unsigned keep_u8) {
  return ((bytes4 >> (8 * k)) & 0xffu) <= keep_u8;
}

}  // namespace fa
