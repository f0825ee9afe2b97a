// Shared device-side building blocks for the MI355X (gfx950 / CDNA4) FlashAttention-2 kernels.
//
// Everything here is written for wave64 + the gfx950 32x32x16 bf16/f16 MFMA:
//   * mfma_f32_32x32x16_{bf16,f16}: lane l (r = l&31, h = l>>5) holds A[r][8h+j] and B[8h+j][r]
//     (j = 0..7) and accumulator element g at (row = (g&3) + 8(g>>2) + 4h, col = r).
//   * An accumulator tile X used as the next MFMA's B operand ("X as operand", no lane movement):
//     registers 8s..8s+7 packed to 16-bit form the fragment of k-step s, whose element j of lane
//     half h is row 16s + 8(j>>2) + 4h + (j&3) of X.  The other operand must supply the same
//     permuted k order, which ds_read_b64_tr_b16 (4 rows x 16 cols per 16-lane group, column-major
//     delivery) gives directly from a row-major LDS tile.
//
// LDS tile layout ("panel" layout), used for every K/V/Q/dO/dS image in this library:
//   a [rows][D] 16-bit tile is stored as D/32 panels of [rows][32 elements] (64-byte rows).  The
//   16-byte chunk c (0..3) of row `row` inside a panel lives at chunk c ^ ((row >> 2) & 3).
//   With 64-byte rows four consecutive rows fill one 256-byte LDS bank line, so
//     - ds_read_b128 row reads (16 distinct rows, same logical chunk) hit 16 distinct 16-byte slots,
//     - ds_read_b64_tr_b16 reads (4 consecutive rows x 64 bytes per half-wave) fill one bank line,
//   i.e. both access kinds are conflict-free on the same image, for any D that is a multiple of 32.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "fa_params.h"

namespace fa {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(4))) short i16x4_t;
typedef __attribute__((ext_vector_type(8))) short i16x8_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
typedef __attribute__((address_space(3))) i16x4_t lds_i16x4_t;

constexpr float kNegInf = -__builtin_huge_valf();
// forward online softmax (fa_fwd.hip; the assembly forward uses the same constants, asm/gen_fwd.py)
constexpr float kFwdRescaleThr = 8.f;   // deferred-max threshold, log2 units (P <= 256)
constexpr float kFwdSumThr = 256.f;     // fast-path guard on a lane's per-tile sum of P (= 2^8)
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ------------------------------------------------------------------------------------------------
// Element traits: 16-bit storage type, MFMA, f32 <-> 16-bit conversions.
// ------------------------------------------------------------------------------------------------
template <bool BF16> struct Elt;

template <> struct Elt<true> {
  __device__ static inline f32x16_t mfma(i16x8_t a, i16x8_t b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving).  Kept compiler-visible on purpose: an asm convert is
  // opaque to the hazard recognizer, which then omits the wait states between an MFMA and a
  // following VALU write of that MFMA's source registers (observed: corrupted dQ operands).
  // The pair goes through ONE vector fptrunc (__builtin_convertvector): two scalar casts plus a
  // build_vector were lowered in some kernels to cvt(lo, 0), cvt(lo, hi), v_bfi / v_perm -- twice the
  // VALU of the single v_cvt_pk_bf16_f32 (seen in the dK/dV kernel's P packing).
  __device__ static inline unsigned pack2(float lo, float hi) {
    const f32x2_t v = {lo, hi};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
  }
  __device__ static inline float to_f32(unsigned short x) {
    return __builtin_bit_cast(float, (unsigned)x << 16);
  }
};

template <> struct Elt<false> {
  __device__ static inline f32x16_t mfma(i16x8_t a, i16x8_t b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a),
                                                  __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  }
  __device__ static inline unsigned pack2(float lo, float hi) {   // v_cvt_pk_f16_f32 (RNE)
    const f32x2_t v = {lo, hi};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2_t));
  }
  __device__ static inline float to_f32(unsigned short x) {
    return (float)__builtin_bit_cast(_Float16, x);
  }
};

// Pack accumulator registers 8s..8s+7 of a 32x32 f32 tile into a 16-bit MFMA operand fragment.
template <bool BF16>
__device__ inline i16x8_t pack_frag(const f32x16_t& x, int s) {
  u32x4_t u;
  u[0] = Elt<BF16>::pack2(x[8 * s + 0], x[8 * s + 1]);
  u[1] = Elt<BF16>::pack2(x[8 * s + 2], x[8 * s + 3]);
  u[2] = Elt<BF16>::pack2(x[8 * s + 4], x[8 * s + 5]);
  u[3] = Elt<BF16>::pack2(x[8 * s + 6], x[8 * s + 7]);
  return __builtin_bit_cast(i16x8_t, u);
}

// ------------------------------------------------------------------------------------------------
// Panel-layout LDS addressing (see header comment).  `chunk` counts 16-byte chunks along D
// (0 .. D/8-1), `nrows` is the row count of the tile.
// ------------------------------------------------------------------------------------------------
__device__ __host__ inline int panel_off(int row, int chunk, int nrows) {
  return (chunk >> 2) * nrows * 64 + row * 64 + (((chunk & 3) ^ ((row >> 2) & 3)) << 4);
}

// ds_read_b64_tr_b16 of the 4x16 block whose rows start at `row0` (multiple of 4) and whose
// columns start at element `col0` (multiple of 16) of a panel-layout tile with `nrows` rows.
// `i` = lane & 15 (lane 4q+p addresses row q, columns 4p..4p+3).  Element q of the result holds
// row row0+q, column col0 + i.
__device__ inline i16x4_t tr_read(const char* tile, int row0, int col0, int nrows, int i) {
  const int q = i >> 2, p = i & 3;
  const int row = row0 + q;
  const int col = col0 + 4 * p;                       // element column
  const int off = panel_off(row, col >> 3, nrows) + ((col & 4) << 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(tile + off));
}

// Two tr reads -> one 8-element operand fragment (rows row0..row0+3 and row0+8..row0+11).
__device__ inline i16x8_t tr_frag(const char* tile, int row0, int col0, int nrows, int i) {
  i16x4_t lo = tr_read(tile, row0, col0, nrows, i);
  i16x4_t hi = tr_read(tile, row0 + 8, col0, nrows, i);
  i16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Row read of 8 consecutive elements (one 16-byte chunk) of a panel-layout tile.
__device__ inline i16x8_t row_read(const char* tile, int row, int chunk, int nrows) {
  return *(const i16x8_t*)(tile + panel_off(row, chunk, nrows));
}

// ------------------------------------------------------------------------------------------------
// Per-lane LDS bases for the two access kinds on a panel-layout tile, valid whenever the tile row
// offset R0 of the access is a multiple of 16.  Every address then is   base + compile-time
// constant, so the reads use the ds_* immediate offset and keep no per-read address VGPRs.
//   row read  (ds_read_b128, A/B operand rows r, chunk C):   tile + (C>>2)*NR*64 + R0*64 + rb[(C>>1)&1]
//   tr read   (ds_read_b64_tr_b16, rows R0+4h+q, 16 cols at DT*32 + 16(r>>4)):
//                                   lo = tile + DT*NR*64 + R0*64 + tb[0],  hi = ... + 8*64 + tb[1]
// ------------------------------------------------------------------------------------------------
struct LdsBases {
  int rb[2];  // row-read bases for chunk&3 = hh (even k-step) and 2+hh (odd k-step)
  int tb[2];  // tr-read bases for rows R0+4h+q and R0+8+4h+q
  __device__ inline LdsBases(int lane) {
    const int r = lane & 31, hh = lane >> 5, i = lane & 15;
    const int xr = (r >> 2) & 3;
    rb[0] = r * 64 + (((0 + hh) ^ xr) << 4);
    rb[1] = r * 64 + (((2 + hh) ^ xr) << 4);
    const int q = i >> 2, pp = i & 3;
    const int trc = 2 * (r >> 4) + (pp >> 1);
    tb[0] = (4 * hh + q) * 64 + ((trc ^ hh) << 4) + (pp & 1) * 8;
    tb[1] = (4 * hh + q) * 64 + ((trc ^ (2 + hh)) << 4) + (pp & 1) * 8;
  }
};

// Opaque 32-bit value: stops LICM / reassociation from turning "base + constant" LDS addresses into
// one hoisted VGPR per constant (the ring-buffer offset changes every tile).
__device__ inline int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Per-tile LDS addresses: the four lane bases of LdsBases shifted to one tile (byte offset
// `tile_off` from `smem`), made opaque so each read is   base VGPR + immediate offset.
struct TileAddr {
  int r[2], t[2];
  __device__ inline TileAddr(const LdsBases& b, int tile_off) {
    r[0] = opaque(tile_off + b.rb[0]); r[1] = opaque(tile_off + b.rb[1]);
    t[0] = opaque(tile_off + b.tb[0]); t[1] = opaque(tile_off + b.tb[1]);
  }
};

// 16-byte row read of chunk C (compile-time) for rows R0 + (lane & 31), R0 % 16 == 0.
template <int NR, int R0, int C>
__device__ inline i16x8_t row_read_c(const char* smem, const TileAddr& a) {
  static_assert(R0 % 16 == 0, "row offset must be a multiple of 16");
  return *(const i16x8_t*)(smem + a.r[(C >> 1) & 1] + ((C >> 2) * NR * 64 + R0 * 64));
}

// Operand fragment of the 16-row k-step at rows R0..R0+15 (R0 % 16 == 0), columns DT*32 + [0, 32),
// in the "accumulator as operand" k order (two ds_read_b64_tr_b16).
template <int NR, int R0, int DT>
__device__ inline i16x8_t tr_frag_c(const char* smem, const TileAddr& a) {
  static_assert(R0 % 16 == 0, "row offset must be a multiple of 16");
  constexpr int off = DT * NR * 64 + R0 * 64;
  const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(smem + a.t[0] + off));
  const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(smem + a.t[1] + off + 8 * 64));
  i16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Compile-time loop helper: f(std::integral_constant<int, I>) for I in [0, N).
template <int I, int N, typename F>
__device__ inline void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// max / sum across the two 32-lane halves (lanes l and l^32 hold the same query / key column).
__device__ inline float half_swap_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                            __builtin_bit_cast(unsigned, x), false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ inline float half_swap_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                            __builtin_bit_cast(unsigned, x), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

__device__ inline float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ inline float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ inline int wave_uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
template <typename T> __device__ inline const T* uniform_ptr(const T* p) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return (const T*)(((unsigned long long)hi << 32) | lo);
}

// LDS-DMA: 16 bytes per lane from a range-checked buffer (offsets past `bytes` read as zero) into
// the wave-uniform LDS address `lds_dst` + 16 * lane.
typedef __amdgpu_buffer_rsrc_t buf_rsrc_t;
__device__ inline buf_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
//
// Issued as inline asm on purpose: for the buffer_load_lds builtin the compiler cannot prove that
// later LDS reads (ds_read_b64_tr_b16 in particular) miss the DMA destination, and inserts an
// `s_waitcnt vmcnt(0)` before them -- which waits for the tile just issued two steps ahead and
// exposes its whole latency every iteration.  The kernels order DMA and LDS reads themselves
// (counted vmcnt + barrier per ring step), so the compiler must not see these stores.
//
// The asm opens with `s_nop 4` (five wait states) because the compiler's hazard recognizer does not
// look inside inline asm.  Two hazards apply to this instruction: M0 written by SALU -> LDS-DMA (one
// wait state) and "VALU writes an SGPR -> VMEM reads that SGPR" (five wait states).  The second one
// bites when SGPR pressure makes the compiler reload the descriptor from an SGPR spill lane
// (v_readlane_b32) right before the asm: with `s_nop 0` the DMA then read a stale descriptor word
// and filled the K tile with wrong bytes (the masked non-causal dropout forward at d = 128 returned
// a wrong LSE and NaN outputs; the d = 32 / 96 spill-heavy instantiations had the same pattern).
// tests/test_isa_hazards.py checks the built code object for this hazard.
__device__ inline unsigned lds_addr(const char* p) {
  return wave_uniform((int)(unsigned)(size_t)(__attribute__((address_space(3))) const char*)p);
}
__device__ inline void dma16(buf_rsrc_t rsrc, char* lds_dst, int voffset) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "{m0}"(lds_addr(lds_dst)), "v"(voffset), "s"(rsrc) : "memory");
}
__device__ inline void dma4(buf_rsrc_t rsrc, char* lds_dst, int voffset) {
  asm volatile("s_nop 4\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :: "{m0}"(lds_addr(lds_dst)), "v"(voffset), "s"(rsrc) : "memory");
}
// the same with the LDS destination as a byte address in the LDS aperture (wave-uniform)
__device__ inline void dma16_at(buf_rsrc_t rsrc, unsigned lds, int voffset) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "{m0}"(wave_uniform((int)lds)), "v"(voffset), "s"(rsrc) : "memory");
}
__device__ inline void dma4_at(buf_rsrc_t rsrc, unsigned lds, int voffset) {
  asm volatile("s_nop 4\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :: "{m0}"(wave_uniform((int)lds)), "v"(voffset), "s"(rsrc) : "memory");
}
__device__ inline void wait_dma_and_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Workgroup barrier for LDS hand-offs only: drains this wave's LDS operations but leaves its
// vector-memory operations (LDS-DMA of later tiles) in flight.  __syncthreads() would also wait
// for vmcnt(0), i.e. for the DMA just issued two tiles ahead.
__device__ inline void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 8]: at most n of this wave's vector-memory
// operations (in issue order, the youngest) may remain outstanding.
__device__ inline void wait_vmcnt(int n) {
  switch (n) {
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// vmcnt(0) that the compiler's own wait-count tracking sees (the asm waits are opaque to it): after
// this, register fragments loaded from global memory before a ring loop count as landed, so the
// compiler inserts no vmcnt wait inside the loop (which would also wait for the in-flight DMA).
__device__ inline void wait_vmem_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// End of a ring step: the tile issued `younger` DMA operations ago may stay in flight, everything
// older must have landed (in every wave) before any wave passes the barrier.
__device__ inline void wait_dma_keep_and_barrier(int younger) {
  wait_vmcnt(younger);
  lds_barrier();
}

// 16-byte global load with zero fill when !valid.
__device__ inline u32x4_t ld16(const void* p, bool valid) {
  u32x4_t z = {0u, 0u, 0u, 0u};
  return valid ? *(const u32x4_t*)p : z;
}

// XCD-aware workgroup order for a 1-D grid of nbh * nblk workgroups (nbh = batch x heads, nblk
// blocks per head).  The dispatcher deals workgroups round-robin to the 8 XCDs (L % 8 share one,
// MI355X_MICROARCH.md "Workgroup dispatch"), so the XCD of group j is given heads bh = j, j + 8, ...
// one after another, each with all of its blocks in order: the workgroups that stream the same
// head's K/V (or Q/dO) run together on one XCD and share its 4 MiB L2 instead of fetching the stream
// once per XCD.  Falls back to head-fastest order when nbh is not a multiple of 8.
__device__ inline void xcd_order(int L, int nbh, int nblk, int& bh, int& blk) {
  if ((nbh & 7) == 0) {
    const int i = L >> 3;
    const int hl = i / nblk;
    blk = i - hl * nblk;
    bh = hl * 8 + (L & 7);
  } else {
    blk = L / nbh;
    bh = L - blk * nbh;
  }
}

// Row `q` of the dense additive mask for (batch, head), or nullptr when there is no mask / q is out
// of range (AttnShape::mask; reference row_offset_mask, flash_fwd_kernel.h:640-643, with the query
// index taken modulo mask_sq per row).
template <typename Shape>
__device__ inline const unsigned short* mask_row_ptr(const Shape& s, int bidb, int head, int q) {
  if (s.mask == nullptr) return nullptr;
  const int64_t r = ((int64_t)bidb * s.mask_h + head % s.mask_h) * s.mask_sq + q % s.mask_sq;
  return (const unsigned short*)s.mask + r * s.mask_row;
}

// FlashMask: offset of the (batch, head) column-bound vectors (reference row_offset_sparse_mask,
// flash_fwd_kernel.h:1109: (bidb * h_sparsemask + bidh / (h / h_sparsemask)) * seqlen_k).
template <typename Shape>
__device__ inline int64_t fm_base(const Shape& s, int bidb, int head) {
  return ((int64_t)bidb * s.fm_h + head / (s.h / s.fm_h)) * s.seqlen_k;
}
// The bounds of one key column (absent vectors: neutral values) and whether they hide `row`.
// Unsigned compares as in the reference (softmax.h:180-298): apply_sparse_mask_causal(_withend) for
// causal (LTEnd absent = to the end), apply_sparse_mask pairwise (LT and UT ranges) when upstart is
// given, else rows >= LTStart or < UTEnd.  The causal (key > row) and key-bound parts stay with the
// caller.
struct FmCol {
  unsigned lts, lte, uts, ute;
};
template <typename Shape>
__device__ inline FmCol fm_load(const Shape& s, int64_t col) {
  FmCol c;
  c.lts = (unsigned)s.fm_lts[col];
  c.lte = s.fm_lte ? (unsigned)s.fm_lte[col] : 0xffffffffu;
  c.uts = s.fm_uts ? (unsigned)s.fm_uts[col] : 0u;
  c.ute = s.fm_ute ? (unsigned)s.fm_ute[col] : 0u;
  return c;
}
template <bool CAUSAL>
__device__ inline bool fm_hidden(const FmCol& c, bool pairwise, int row) {
  const unsigned r = (unsigned)row;
  if (CAUSAL) return r >= c.lts && r < c.lte;
  if (pairwise) return (r >= c.lts && r < c.lte) || (r >= c.uts && r < c.ute);
  return r >= c.lts || r < c.ute;
}
// Whether FlashMask removes (row, key); `col` = fm_base + key.
template <bool CAUSAL, typename Shape>
__device__ inline bool fm_masked(const Shape& s, int64_t col, int row) {
  return fm_hidden<CAUSAL>(fm_load(s, col), s.fm_uts != nullptr, row);
}
// Whether the bounds hide every key of [n0, n0 + nk) (keys >= sk count as hidden) from every row of
// [r0, r1): the reference's per-block max/min test (mask.h:4-126 scan, flash_fwd_kernel.h:1305-
// 1308), one key per lane (nk <= 64) and a wave reduction instead of a separate scan kernel.
// Conservative (a mixed block counts as live); the result is wave-uniform.
template <bool CAUSAL, typename Shape>
__device__ inline bool fm_tile_dead(const Shape& s, int64_t base, int n0, int nk, int sk, int r0, int r1,
                                    int lane) {
  const int key = n0 + lane;
  const bool ok = lane < nk && key < sk;   // other lanes: neutral values
  const int64_t col = base + (ok ? key : 0);
  unsigned lts = ok ? (unsigned)s.fm_lts[col] : 0u;
  unsigned lte = (ok && s.fm_lte) ? (unsigned)s.fm_lte[col] : 0xffffffffu;
  unsigned uts = (ok && s.fm_uts) ? (unsigned)s.fm_uts[col] : 0u;
  unsigned ute = (ok && s.fm_ute) ? (unsigned)s.fm_ute[col] : 0xffffffffu;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lts = max(lts, (unsigned)__shfl_xor((int)lts, off));
    lte = min(lte, (unsigned)__shfl_xor((int)lte, off));
    uts = max(uts, (unsigned)__shfl_xor((int)uts, off));
    ute = min(ute, (unsigned)__shfl_xor((int)ute, off));
  }
  const unsigned a = (unsigned)r0, e = (unsigned)r1;
  bool dead;
  if (CAUSAL) dead = a >= lts && e <= lte;
  else if (s.fm_uts != nullptr) dead = (a >= lts && e <= lte) || (a >= uts && e <= ute);
  else dead = a >= lts || e <= ute;
  return __builtin_amdgcn_readfirstlane((int)dead) != 0;
}

// The same with heads taken hp at a time: the XCD of group j walks groups of hp of its heads, and
// inside a group block-major / head-minor (block 0 -- the heaviest causal block -- of every head of
// the group first).  hp = 1 is xcd_order.  A larger hp keeps fewer heads' streams in flight than
// head-fastest order while bounding the causal tail: the last group's heaviest block starts after
// (G-1)/G of the XCD's work, G = heads per XCD / hp (launchers pick hp, xcd_head_group()).
// Requires nbh % 8 == 0 and (nbh / 8) % hp == 0; otherwise head-fastest order.
__device__ inline void xcd_order_grouped(int L, int nbh, int nblk, int hp, int& bh, int& blk) {
  if ((nbh & 7) == 0 && hp > 0 && ((nbh >> 3) % hp) == 0) {
    const int i = L >> 3;
    const int per_group = hp * nblk;
    const int g = i / per_group;
    const int r = i - g * per_group;
    blk = r / hp;
    const int hl = g * hp + (r - blk * hp);
    bh = hl * 8 + (L & 7);
  } else {
    blk = L / nbh;
    bh = L - blk * nbh;
  }
}


// Heads per group for xcd_order_grouped on a causal grid of nbh heads x nblk blocks whose block b
// costs ~(b + 1) units: the heaviest block (nblk units) must fit in 1/G of a CU's share of the work,
// G <= nbh (nblk + 1) / (2 * 256 CUs); hp = the smallest divisor of nbh / 8 giving G within that.
// Used only when the K/V (or Q/dO) stream of the launch is larger than the 256 MiB Infinity Cache
// (stream_bytes): below that the cache absorbs the re-reads of head-fastest order, which then keeps
// the better causal balance (measured at C3, 256 MiB of K/V: grouping -1.5%; at C5, 1 GiB: +16% fwd,
// +14% dQ).  causal = false: every block costs the same, one head per group.
// The threshold is the FLASH_ATTN_MI355X_XCD_GROUP_MIN_MIB knob (default 256), and
// FLASH_ATTN_MI355X_NO_XCD_GROUP=1 forces head-fastest order (fa_params.h Knob: read once).
inline int xcd_head_group(long long nbh, long long nblk, long long stream_bytes, bool causal, int min_mib = -1) {
  if (min_mib < 0) min_mib = knob(kKnobXcdGroupMinMiB);
  if (knob(kKnobNoXcdGroup) == 1 || stream_bytes <= ((long long)min_mib << 20)) return 0;
  if (nbh % 8 != 0 || nbh <= 0 || nblk <= 0) return 0;
  if (!causal) return 1;
  const long long h8 = nbh / 8;
  long long gmax = nbh * (nblk + 1) / 512;
  if (gmax < 1) gmax = 1;
  for (long long hp = 1; hp <= h8; ++hp)
    if (h8 % hp == 0 && h8 / hp <= gmax) return (int)hp;
  return (int)h8;
}

// Accumulator element g -> row offset inside a 32x32 tile for lane half h.
__device__ __host__ constexpr inline int acc_row(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

}  // namespace fa
