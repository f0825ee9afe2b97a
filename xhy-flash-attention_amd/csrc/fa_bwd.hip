// FlashAttention-2 backward for MI355X (gfx950): dQ, dK, dV with the softmax recomputed from LSE.
//
// Algorithm (math of the reference's backward, csrc/flash_attn/src/flash_bwd_kernel.h):
//   D  = rowsum(dO o O)                                   (compute_dot_do_o, :112-188)
//   P  = exp(scale * Q K^T - LSE)                          (:847)
//   dS = P o (dO V^T - D)                                  (:897-906)
//   dV = P^T dO,  dK = scale * dS^T Q,  dQ = scale * dS K  (:948-1008, epilogue :1046-1051)
//
// MI355X design (not the reference's seqk-parallel kernel with fp32 dQ atomics, which on this chip
// is bound by the ~1.3 TB/s global-atomic rate: 8.7 GB of dQ adds at the C3 headline shape):
//   1. bwd_pre_kernel   D = rowsum(dO o O)  (one 16-lane group per query row)
//   2. bwd_dkdv_kernel  one workgroup (8 waves) per 128-key block of a (batch, kv-head), the waves
//                       specialised by role: 4 "P" waves hold K and accumulate dV^T, 4 "dS" waves
//                       hold V and accumulate dK^T, P passing between them through LDS; (Q, dO,
//                       LSE, D) slices of 64 query rows arrive by LDS-DMA one slice ahead; the
//                       dS waves run one slice behind the P waves so one wave's VALU hides under
//                       the other's MFMAs with one barrier per slice; dK^T / dV^T accumulate in registers over every slice (and, for
//                       GQA, every query head of the group) and are written once: no atomics.
//   3. bwd_dq_kernel    one workgroup (8 waves) per 256-row query block, structured like the
//                       forward: Q and dO fragments in registers, K/V tiles by LDS-DMA ring,
//                       S^T and dP^T with the query on the MFMA lane (LSE and D are per-lane
//                       scalars), dQ^T += K^T dS^T with dS^T used in-register as the B operand;
//                       dQ written directly in bf16/f16 (no fp32 accumulator, no conversion pass).
// Both main kernels are deterministic (no atomics), so dQ is bitwise reproducible too.
//
//   * "Key on the lane" in dkdv: S = Q K^T and dP = dO V^T have the key on the MFMA column, so
//     their accumulators are directly the B operands of dV^T = dO^T P and dK^T = Q^T dS; dO^T and
//     Q^T come from the row-major LDS slice through ds_read_b64_tr_b16.
//   * Slices that need no mask skip the mask arithmetic (one wave-uniform test per slice).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_dropout.h"
#include "fa_params.h"

namespace fa {

typedef unsigned short u16;

// Tile shapes per head dim.  d <= 128: two waves per SIMD.  d in (128, 256]: the D x 32
// accumulators and the 32-key operand set need more than 256 registers per wave, so workgroups
// are 4 waves (one per SIMD, 512 registers) and the LDS tiles shrink to fit.
template <int D> struct DkdvTile {
  static constexpr int NW = D <= 128 ? 8 : 4;      // NW/2 "P" waves + NW/2 "dS" waves
  static constexpr int NKG = NW / 2;               // 32-key groups per workgroup
  static constexpr int BN = 32 * NKG;              // keys per workgroup
  static constexpr int BQ = D <= 128 ? 64 : 32;    // query rows per sweep step (32-row q-tiles)
};
template <int D> struct DqTile {
  static constexpr int NW = D <= 128 ? 8 : 4;
  static constexpr int BM = 32 * NW;               // query rows per dQ workgroup
  static constexpr int BN = D <= 128 ? 64 : 32;    // keys per streamed K/V tile
  static constexpr int MINB = D <= 128 ? 2 : 1;
};
constexpr int kDqMinBM = 128;                      // smallest dQ query block (grid-size check)
constexpr int kBwdBufs = 3;
#ifndef FA_DQ_STAGGER   // dev switch (A/B): staggered halves in bwd_dq_kernel
#define FA_DQ_STAGGER 1
#endif
#ifndef FA_DQ_PRIO      // dev switch (A/B): waves 4-7 of bwd_dq_kernel at s_setprio 1
#define FA_DQ_PRIO 1
#endif

// ------------------------------------------------------------------------------------------------
// geometry shared by the kernels (reference BlockInfo, block_info.h:14-31)
// ------------------------------------------------------------------------------------------------
struct SeqGeom {
  int sq, sk;
  int64_t q_off, k_off, v_off, o_off, do_off, dq_off, dk_off, dv_off;
};

__device__ inline SeqGeom seq_geom(const BwdParams& p, int bidb) {
  const AttnShape& s = p.s;
  SeqGeom g;
  g.sq = s.seqlen_q; g.sk = s.seqlen_k;
  g.q_off = (int64_t)bidb * p.q_batch; g.o_off = (int64_t)bidb * p.o_batch;
  g.do_off = (int64_t)bidb * p.do_batch; g.dq_off = (int64_t)bidb * p.dq_batch;
  g.k_off = (int64_t)bidb * p.k_batch; g.v_off = (int64_t)bidb * p.v_batch;
  g.dk_off = (int64_t)bidb * p.dk_batch; g.dv_off = (int64_t)bidb * p.dv_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    g.sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) {
      g.q_off = (int64_t)c0 * p.q_row; g.o_off = (int64_t)c0 * p.o_row;
      g.do_off = (int64_t)c0 * p.do_row; g.dq_off = (int64_t)c0 * p.dq_row;
    }
  }
  if (s.cu_seqlens_k) {
    const int c0 = s.cu_seqlens_k[bidb];
    g.sk = s.cu_seqlens_k[bidb + 1] - c0;
    if (!s.varlen_padded_input) {
      g.k_off = (int64_t)c0 * p.k_row; g.v_off = (int64_t)c0 * p.v_row;
      g.dk_off = (int64_t)c0 * p.dk_row; g.dv_off = (int64_t)c0 * p.dv_row;
    }
  }
  return g;
}

// bytes of rows [0, rows) of a strided operand, clamped to the buffer descriptor's range
__device__ inline int rec_bytes(int rows, int64_t row_stride, int elem_bytes) {
  const int64_t b = (int64_t)(rows > 0 ? rows : 0) * row_stride * elem_bytes;
  return (int)(b > 0x7fffffff ? 0x7fffffff : b);
}

// per-lane byte offset of piece `pc` of a panel-layout tile of NR rows (see fa_fwd.hip)
template <int NR>
__device__ inline int dma_voff(int pc, int lane, int64_t row_stride, int dlim) {
  const int panel = pc / (NR / 16);
  const int row = (pc % (NR / 16)) * 16 + (lane >> 2);
  const int col = panel * 32 + (((lane & 3) ^ ((row >> 2) & 3)) << 3);
  return col < dlim ? (int)(((int64_t)row * row_stride + col) * 2) : 0x7ffffff0;
}

// ------------------------------------------------------------------------------------------------
// 1. D = rowsum(dO * O)
// ------------------------------------------------------------------------------------------------
template <bool BF16>
__global__ void __launch_bounds__(256) bwd_pre_kernel(const BwdParams p) {
  // HBM-bound (reads O and dO once): each 16-lane group handles kPreRows rows 16 apart, all their
  // loads issued before any arithmetic, so a lane keeps 2 kPreRows 16-byte loads in flight
  constexpr int kPreRows = 4;
  using E = Elt<BF16>;
  const AttnShape s = p.s;
  const int bh = blockIdx.x;
  const int bidb = bh / s.h, head = bh - bidb * s.h;
  const SeqGeom g = seq_geom(p, bidb);
  const int l16 = threadIdx.x & 15;
  const int nch = s.d / 8;   // 16-byte chunks per row (<= 32)
  u32x4_t a[kPreRows][2], b[kPreRows][2];
#pragma unroll
  for (int r = 0; r < kPreRows; ++r) {
    const int row = blockIdx.y * (16 * kPreRows) + r * 16 + (threadIdx.x >> 4);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = l16 + 16 * u;
      a[r][u] = b[r][u] = u32x4_t{0, 0, 0, 0};
      if (row < g.sq && c < nch) {
        a[r][u] = *(const u32x4_t*)((const u16*)p.o + g.o_off + (int64_t)head * p.o_head + (int64_t)row * p.o_row + 8 * c);
        b[r][u] = *(const u32x4_t*)((const u16*)p.dout + g.do_off + (int64_t)head * p.do_head + (int64_t)row * p.do_row + 8 * c);
      }
    }
  }
  const int64_t bhi = (int64_t)bidb * s.h + head;
#pragma unroll
  for (int r = 0; r < kPreRows; ++r) {
    const int row = blockIdx.y * (16 * kPreRows) + r * 16 + (threadIdx.x >> 4);
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        acc += E::to_f32(a[r][u][w] & 0xffff) * E::to_f32(b[r][u][w] & 0xffff);
        acc += E::to_f32(a[r][u][w] >> 16) * E::to_f32(b[r][u][w] >> 16);
      }
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 16);
    if (l16 != 0) continue;
    if (row >= g.sq) {
      // assembly dK / dV path: the rows of the last 32-row group past seqlen_q read zero chain starts
      if (p.lsed != nullptr && row < ((g.sq + 31) & ~31)) {
        float* grp = p.lsed + (bhi * p.lsed_ng + (row >> 5)) * 64 + (row & 31);
        grp[0] = 0.f;
        grp[32] = 0.f;
      }
      continue;
    }
    // with dropout the reference keeps D scaled down by the keep probability (flash_bwd_kernel.h:178-182)
    const float dv = s.dropout ? acc * s.p_keep : acc;
    p.dsum[bhi * p.seqlen_q_rounded + row] = dv;
    // -LSE / scale: the initial accumulator of the dK/dV kernel's S chain (scale != 0: launch_bwd)
    const float ls = -p.lse[bhi * s.lse_pitch + row] / s.scale;
    if (p.lsed != nullptr) {   // assembly dK / dV: [-LSE / scale | -D] per 32-row group
      float* grp = p.lsed + (bhi * p.lsed_ng + (row >> 5)) * 64 + (row & 31);
      grp[0] = ls;
      grp[32] = -dv;
    } else {
      p.lse_s[bhi * p.seqlen_q_rounded + row] = ls;
    }
  }
}

#ifdef FA_STAMPS
// Dev timeline instrumentation (FA_STAMPS builds only, tools/stamps.py): s_memtime at phase
// boundaries of the dK/dV loop for workgroups 0-3, 64 slices, 8 points per slice.
constexpr int kStampWg = 4, kStampIt = 64, kStampPts = 8;
__device__ unsigned long long g_fa_stamps[kStampWg * 8 * kStampIt * kStampPts];
#define FA_STAMP(k)                                                                             \
  do {                                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                                          \
    if (blockIdx.x < kStampWg && it < kStampIt && lane == 0)                                    \
      g_fa_stamps[((blockIdx.x * 8 + wave) * kStampIt + it) * kStampPts + (k)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                          \
  } while (0)
#else
#define FA_STAMP(k) do {} while (0)
#endif
#ifndef FA_DKDV_DMA_POS      // dev A/B switch: where the dS waves issue the later DMA parts
#define FA_DKDV_DMA_POS 0
#endif
#ifndef FA_DKDV_UNFUSED_P   // dev A/B switch: 1 = the unfused P-wave step
#define FA_DKDV_UNFUSED_P 0
#endif

// ------------------------------------------------------------------------------------------------
// 2. dK / dV  (wave-specialised: 4 "P" waves + 4 "dS" waves per 128-key block)
// ------------------------------------------------------------------------------------------------
// Waves 0-3 ("P" waves) hold K of their 32 keys and accumulate dV^T; waves 4-7 ("dS" waves) hold
// -V of the same 32 keys and accumulate -dK^T.  Per 64-row query slice `it` (ONE barrier per step):
//   P waves:  S'(it) = Q K^T - LSE/scale (MFMA chain started from -LSE/scale, computed by
//             bwd_pre_kernel) -> P(it) = exp2(c S') (masked) -> P(it) to LDS (fp32)
//             -> dV^T += dO(it)^T P(it)
//   dS waves: dS''(it-1) = P(it-1) o dP''(it-1)      (P of the previous slice, from LDS)
//             -> dK''^T += Q(it-1)^T dS''(it-1)
//             -> dP''(it) = D - dO(it) V^T           (MFMA chain started from D, on -V)
// so dS'' = -dS and dK'' = -dK (sign folded into the epilogue scale): the dS step is one multiply
// per element.  On every SIMD one P wave and one dS wave run side by side with complementary
// phases -- the P wave's softmax VALU sits between its two MFMA blocks, the dS wave's VALU at the
// start of its step -- so one wave's VALU hides under the other's MFMAs without a second barrier.
// Slice lifetimes: Q (+ LSE, D) is read in steps it and it+1 (3-deep ring, one slice of DMA in
// flight), dO only in step it (2-deep ring), P(it) in steps it and it+1 (2 buffers).
// Each wave needs one 32-key operand set and one D x 32 accumulator set (<= 256 registers).
// MASKED (dense additive mask and/or FlashMask present): every slice takes the per-element path; the
// unmasked instantiations carry no mask code (as in fwd_kernel).
// ------------------------------------------------------------------------------------------------
// Q' = bf16/f16(c Q) for a call that folds (attn_folds_q): the backward always, the forward when it
// cannot take the assembly kernel.  The assembly forward rewrites its Q fragments as
// v_cvt_pk(v_mul_f32(q, c)) (gen_fwd.py q_scale_ops) -- the same fp32 product and
// round-to-nearest-even pack here, so every score a HIP kernel computes from Q' is bitwise the
// assembly kernel's.  HBM-bound elementwise pass, 16 bytes per thread (rows and heads are 16-byte
// aligned: d % 8 == 0, bwd_pre_kernel's own assumption); output in the compact layout (b or padded
// rows, seqlen_q, h, d), rows at the sequence offsets seq_geom uses (QFoldArgs, fa_params.h).
// ------------------------------------------------------------------------------------------------
template <bool BF16>
__global__ void __launch_bounds__(256) q_fold_kernel(const QFoldArgs a) {
  using E = Elt<BF16>;
  const int bidb = blockIdx.y;
  int sq = a.seqlen_q;
  int64_t q_off = (int64_t)bidb * a.q_batch;
  const int64_t hd = (int64_t)a.h * a.d;
  int64_t base = (int64_t)bidb * a.seqlen_q * hd;
  if (a.cu_seqlens_q != nullptr) {   // (seq_geom's rule for the Q rows)
    const int c0 = a.cu_seqlens_q[bidb];
    sq = a.cu_seqlens_q[bidb + 1] - c0;
    if (!a.padded) {
      q_off = (int64_t)c0 * a.q_row;
      base = (int64_t)c0 * hd;
    }
  }
  const int nch = a.d / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int ch = (int)(t % nch);
  const int64_t rh = t / nch;
  const int head = (int)(rh % a.h);
  const int64_t row = rh / a.h;
  if (row >= sq) return;
  const u32x4_t x = *(const u32x4_t*)((const u16*)a.q + q_off + (int64_t)head * a.q_head + row * a.q_row + 8 * ch);
  u32x4_t y;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = E::to_f32((unsigned short)(x[i] & 0xffffu)) * a.c;
    const float hi = E::to_f32((unsigned short)(x[i] >> 16)) * a.c;
    y[i] = E::pack2(lo, hi);
  }
  *(u32x4_t*)((u16*)a.qf + base + row * hd + (int64_t)head * a.d + 8 * ch) = y;
}

void launch_q_fold(const QFoldArgs& a, bool is_bf16, hipStream_t stream) {
  const int64_t per_seq = (int64_t)a.seqlen_q * a.h * (a.d / 8);
  if (a.b <= 0 || per_seq <= 0) return;
  if (a.d % 8 != 0 || (per_seq + 255) / 256 > 0x7fffffff || a.b > 65535)
    throw std::runtime_error("flash_attn: prescaled-Q grid too large");
  const dim3 grid((unsigned)((per_seq + 255) / 256), (unsigned)a.b);
  prof_begin(kTimeQFold, stream);
  if (is_bf16)
    hipLaunchKernelGGL((q_fold_kernel<true>), grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((q_fold_kernel<false>), grid, dim3(256), 0, stream, a);
  prof_end(kTimeQFold, stream);
}

template <bool BF16, int D, bool CAUSAL, bool DROPOUT, bool MASKED>
__global__ void __launch_bounds__(DkdvTile<D>::NW * 64, 1) bwd_dkdv_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int NW = DkdvTile<D>::NW;
  constexpr int NKG = DkdvTile<D>::NKG;
  constexpr int BKN = DkdvTile<D>::BN;
  constexpr int BQ = DkdvTile<D>::BQ;
  constexpr int NQT = BQ / 32;                      // 32-row q-tiles per slice
  constexpr int KS = D / 16;
  constexpr int NP = D / 32;
  constexpr int QTILE = BQ * D * 2;                 // bytes of a Q or dO slice
  constexpr int QSLOT = QTILE + 2 * 64 * 4;         // Q | lse[64] | D[64] (one dword per lane)
  constexpr int OBASE = 3 * QSLOT;                  // dO ring (2 slots)
  constexpr int XTILE = 32 * 32 * 4;                // one fp32 32x32 P tile
  constexpr int XBUF = NKG * NQT * XTILE;           // P of one slice: key groups x q-tiles
  constexpr int XBASE = OBASE + 2 * QTILE;
  constexpr int PIECES = QTILE / 1024;
  static_assert(QTILE % 1024 == 0, "slice must be whole DMA pieces");
  static_assert(BQ % 32 == 0 && NW % 2 == 0, "32-row q-tiles, two roles");
  // ... then (dropout) one 1-KiB random-byte scratch per P wave
  __shared__ __attribute__((aligned(16))) char smem[XBASE + 2 * XBUF + (DROPOUT ? NKG * 1024 : 0)];

  const AttnShape s = p.s;
  const uint64_t pseed = DROPOUT ? philox_seed_of(s) : 0, poff = DROPOUT ? philox_offset_of(s) : 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const bool pwave = wave < NKG;
  const int kg = wave % NKG;
  const int r = lane & 31, hh = lane >> 5;
  const LdsBases lb(lane);
  const int group = s.h / s.hk;

  const int nheads_grid = p.gqa_reduce ? s.hk : s.h;
  // XCD-aware order: the key blocks of one (batch, kv-head) run together on one XCD and read the
  // same Q / dO slices at about the same time (8.7% faster at C3 than head-fastest order)
  int bhx, nblk_idx;
  xcd_order(blockIdx.x, s.b * nheads_grid, p.num_n_blocks, bhx, nblk_idx);   // heaviest key block first
  const int bidb = bhx / nheads_grid;
  const int hx = bhx - bidb * nheads_grid;
  const int kvh = p.gqa_reduce ? hx : hx / group;
  const int h_begin = p.gqa_reduce ? hx * group : hx;
  const int nh = p.gqa_reduce ? group : 1;
  const SeqGeom geo = seq_geom(p, bidb);
  const int sq = geo.sq, sk = geo.sk;
  const int n0 = nblk_idx * BKN;
  if (n0 >= sk) return;
  const int dlim = s.d;

  // ---- this wave's 32 keys: K (P waves) or -V (dS waves) fragments, the B operand of phase 1 ----
  const int kw0 = n0 + 32 * kg;
  const int key = kw0 + r;
  i16x8_t kv[KS];
  {
    const bool ok = key < sk;
    const u16* src = pwave ? (const u16*)p.k + geo.k_off + (int64_t)kvh * p.k_head + (int64_t)(ok ? key : 0) * p.k_row
                           : (const u16*)p.v + geo.v_off + (int64_t)kvh * p.v_head + (int64_t)(ok ? key : 0) * p.v_row;
    const unsigned flip = pwave ? 0u : 0x80008000u;   // sign bits of both 16-bit halves
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      u32x4_t w = ld16(src + d0, ok && d0 < dlim);
      w[0] ^= flip; w[1] ^= flip; w[2] ^= flip; w[3] ^= flip;
      kv[ks] = __builtin_bit_cast(i16x8_t, w);
    }
  }

  // ---- query sweep: (head, BQ-row slice) pairs; causal: queries >= n0 only ----
  const int m_first = CAUSAL ? (n0 / BQ) : 0;
  const int m_count = (sq + BQ - 1) / BQ;
  const int ns = m_count > m_first ? m_count - m_first : 0;
  const int total = ns * nh;

  // The slice DMA is issued by the dS waves (waves [DW0, DW0 + DWN)): the P waves' step (S, exp,
  // P store, dV) is the longer one, and taking the DMA issue off it measured -4% (min) / -9%
  // (median) dK/dV time at C3 against every wave issuing; P waves only: -2%.  4-wave workgroups
  // (d > 128): every wave.
  constexpr int DWN = NW == 8 ? 4 : NW, DW0 = NW == 8 ? 4 : 0;
  constexpr int PPWI = (PIECES + DWN - 1) / DWN;
  const int dwv = wave - DW0;
  const bool dma_wave = dwv >= 0 && dwv < DWN;
  int voff_q[PPWI], voff_o[PPWI];
#pragma unroll
  for (int j = 0; j < PPWI; ++j) {
    voff_q[j] = dma_voff<BQ>(dwv + j * DWN, lane, p.q_row, dlim);
    voff_o[j] = dma_voff<BQ>(dwv + j * DWN, lane, p.do_row, dlim);
  }
  // Sweep order: the query slices of one head, then the next head of the GQA group.  (Last slice
  // first with the heads innermost -- every key block then starts on the same slice -- measured 3.5%
  // slower at C3 than this order under xcd_order.)
  auto slice_head = [&](int it) { return it / ns; };
  auto slice_q0 = [&](int it) { return (m_first + it % ns) * BQ; };
  // slice `sid` into ring position `it` (the same except when FlashMask skips slices)
  // DMA of the slice (query head h_begin + hrel, rows q0..) into ring position `it`; the dS waves
  // issue it (the P waves skip the address arithmetic too: the CU's scalar unit is shared)
  // The DMA of one slice is issued in DMA_PARTS parts (pieces [k PPWI / parts, (k+1) PPWI / parts) in
  // part k, the -LSE/scale and D rows with part 0), spread over the dS waves' step (FA_DKDV_DMA_POS).
  // (the plan holds plain scalars, made wave-uniform, and the descriptors are formed at each part:
  // a buffer descriptor kept live across the step can be assigned VGPRs, which the asm rejects)
  const unsigned smem_lds = lds_addr(smem);
  struct SliceDma {
    const u16* qp;
    const u16* dp;
    const float* lp;
    int qrec, orec, lrec, slot;
  };
  auto dma_plan = [&](int hrel, int q0, int it) {
    SliceDma d;
    const int hq = h_begin + hrel;
    d.slot = it;
    d.qp = (const u16*)p.q + geo.q_off + (int64_t)hq * p.q_head + (int64_t)q0 * p.q_row;
    d.dp = (const u16*)p.dout + geo.do_off + (int64_t)hq * p.do_head + (int64_t)q0 * p.do_row;
    d.qrec = rec_bytes(sq - q0, p.q_row, 2);
    d.orec = rec_bytes(sq - q0, p.do_row, 2);
    // -LSE/scale rows (dS wave 0), then D rows (dS wave 1), 64 x 4 bytes each; rows past the slice
    // land in the slot's padding or are never read
    const int64_t bhi = (int64_t)bidb * s.h + hq;
    d.lp = ((dwv == 0) ? p.lse_s : p.dsum) + bhi * p.seqlen_q_rounded + q0;
    d.lrec = rec_bytes(sq - q0, 1, 4);
    return d;
  };
  auto dma_part = [&](const SliceDma& d, auto KC, auto NC) {
    constexpr int k = decltype(KC)::value, n = decltype(NC)::value;
    const int it = wave_uniform(d.slot);
    const unsigned qdst = smem_lds + (it % 3) * QSLOT;
    const unsigned odst = smem_lds + OBASE + (it & 1) * QTILE;
    const buf_rsrc_t rq = make_rsrc(uniform_ptr(d.qp), wave_uniform(d.qrec));
    const buf_rsrc_t ro = make_rsrc(uniform_ptr(d.dp), wave_uniform(d.orec));
#pragma unroll
    for (int j = (k * PPWI) / n; j < ((k + 1) * PPWI) / n; ++j) {
      const int pc = dwv + j * DWN;
      if (PIECES % DWN == 0 || pc < PIECES) {
        dma16_at(rq, qdst + pc * 1024, voff_q[j]);
        dma16_at(ro, odst + pc * 1024, voff_o[j]);
      }
    }
    if (k == 0 && (dwv == 0 || dwv == 1))
      dma4_at(make_rsrc(uniform_ptr(d.lp), wave_uniform(d.lrec)), qdst + QTILE + dwv * 64 * 4, lane * 4);
  };
  auto issue = [&](int hrel, int q0, int it) {
    if (!dma_wave) return;
    const SliceDma d = dma_plan(hrel, q0, it);
    dma_part(d, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
  };

  // dV^T (P waves) or -dK^T (dS waves): D x 32 keys
  f32x16_t acc[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[t][g] = 0.f;

  const float c = s.scale_log2;

  // phase 1: S = Q K^T (P waves) / dP'' = D - dO V^T (dS waves) for both 32-row q-tiles of the
  // slice at `a1` (query on registers, key on lane), chains started from `init`
  auto phase1 = [&](int a1, f32x16_t (&sp)[NQT]) {
    const TileAddr ta(lb, a1);
    // Software-pipelined: the A fragments of k-group g+1 are requested before the MFMAs of group g
    // (sched_barrier keeps the scheduler from sinking the reads next to their MFMAs, which left
    // each LDS read's latency exposed in front of its two MFMAs).
    constexpr int G = KS >= 4 ? 2 : KS;   // k-steps per group
    constexpr int NG = KS / G;
    i16x8_t af[2][NQT][G];
    auto load = [&](auto GGC, i16x8_t (&dst)[NQT][G]) {
      constexpr int g0 = decltype(GGC)::value * G;
      static_for<0, G>([&](auto KK) {
        constexpr int ks = g0 + decltype(KK)::value;
        static_for<0, NQT>([&](auto QT) {
          constexpr int qt = decltype(QT)::value;
          dst[qt][ks - g0] = row_read_c<BQ, 32 * qt, 2 * ks>(smem, ta);
        });
      });
    };
    load(std::integral_constant<int, 0>{}, af[0]);
    static_for<0, NG>([&](auto GG) {
      constexpr int gg = decltype(GG)::value;
      if constexpr (gg + 1 < NG) load(std::integral_constant<int, gg + 1>{}, af[(gg + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < G; ++k)
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) sp[qt] = E::mfma(af[gg & 1][qt][k], kv[gg * G + k], sp[qt]);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  // phase 2: acc += A^T frag, transposed A operand of the slice tile at `a2`; the fragments of
  // d-group dt+1 are requested before the MFMAs of group dt
  auto phase2 = [&](int a2, const i16x8_t (&fr)[2 * NQT]) {
    const TileAddr ta2(lb, a2);
    i16x8_t tf[2][2 * NQT];
    auto tr_group = [&](auto DTC, i16x8_t (&t)[2 * NQT]) {
      constexpr int dt = decltype(DTC)::value;
      static_for<0, 2 * NQT>([&](auto KC) {
        constexpr int kk = decltype(KC)::value;
        t[kk] = tr_frag_c<BQ, 16 * kk, dt>(smem, ta2);
      });
    };
    tr_group(std::integral_constant<int, 0>{}, tf[0]);
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      if constexpr (dt + 1 < NP) tr_group(std::integral_constant<int, dt + 1>{}, tf[(dt + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 2 * NQT; ++kk) acc[dt] = E::mfma(tf[dt & 1][kk], fr[kk], acc[dt]);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // P = exp2(c S') with S' = S - LSE / scale (the chain started from -LSE / scale) for both q-tiles
  // into `xw` (this key group's P tiles), packed to `fr`
  // With dropout the LDS tile carries P sign-encoded (negative where dropped, reference
  // apply_dropout<encode_dropout_in_sign_bit=true>, flash_bwd_kernel.h:848-857) and the packed
  // operand of dV^T carries P o Z (zeros where dropped).
  char* const dscr = smem + XBASE + 2 * XBUF + kg * 1024;
  // (sp is read only: a write-back would make the scores' register set differ between the roles at
  // the join after the P step, which costs 32 copies per step)
  auto p_step = [&](auto MASKC, const f32x16_t (&sp)[NQT], int q0, int it_head, char* xw, i16x8_t (&fr)[2 * NQT]) {
    constexpr bool MASK = decltype(MASKC)::value;
    // FlashMask bounds of this lane's key for this slice's head, loaded once per slice
    FmCol fc = {0u, 0xffffffffu, 0u, 0u};
    const bool fm_on = MASK && MASKED && s.fm_lts != nullptr;
    if constexpr (MASK && MASKED)
      if (fm_on) fc = fm_load(s, fm_base(s, bidb, h_begin + it_head) + (key < sk ? key : 0));
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      f32x16_t pk;   // P (dropout: P o Z), the B operand of dV^T
      unsigned rb[4];
      if constexpr (DROPOUT) {
        const uint64_t doff = poff + (uint64_t)(bidb * s.h + h_begin + it_head) * 32;
        dropout_block_words(dscr, pseed, doff, q0 + 32 * qi, kw0, lane);
        dropout_col_bytes(rb, dscr, lane);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        f32x4_t pv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float x;
          if constexpr (MASK) {
            const int q = q0 + 32 * qi + 8 * u + 4 * hh + j;
            // non-short-circuit ORs and exp2(-inf) = 0: selects, no per-lane branches
            bool out = (key >= sk) | (q >= sq) | (CAUSAL && key > q);
            float sc = sp[qi][4 * u + j];
            if constexpr (MASKED) {
              out = out || (fm_on && fm_hidden<CAUSAL>(fc, s.fm_uts != nullptr, q));
              const u16* mrow = out ? nullptr : mask_row_ptr(s, bidb, h_begin + it_head, q);
              if (mrow != nullptr) sc += E::to_f32(mrow[key]) * s.mask_unscale;
            }
            x = fast_exp2(out ? kNegInf : sc * c);
          } else {
            x = fast_exp2(sp[qi][4 * u + j] * c);
          }
          if constexpr (DROPOUT) {
            const bool keep = dropout_keep(rb[u], j, s.keep_u8);
            pv[j] = keep ? x : -x;
            pk[4 * u + j] = keep ? x : 0.f;
          } else {
            pv[j] = x;
            pk[4 * u + j] = x;
          }
        }
        *(f32x4_t*)(xw + qi * XTILE + u * 1024) = pv;
      }
      fr[2 * qi] = pack_frag<BF16>(pk, 0);
      fr[2 * qi + 1] = pack_frag<BF16>(pk, 1);
    }
  };
  // dS'' = P o dP'' of the slice whose P tiles are at `xw`, packed to `fr`
  // (dropout: P'' = sign-encoded P;  dS'' = P o dP'' where kept, -P''... = P o D where dropped,
  //  reference flash_bwd_kernel.h:897-899 with our dS'' = -dS, dP'' = D - dP)
  auto ds_step = [&](const f32x16_t (&sp)[NQT], const char* xw, const float* dl, i16x8_t (&fr)[2 * NQT]) {
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      f32x16_t x;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4_t pv = *(const f32x4_t*)(xw + qi * XTILE + u * 1024);
        if constexpr (DROPOUT) {
          const f32x4_t dv = *(const f32x4_t*)(dl + 32 * qi + 8 * u + 4 * hh);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[4 * u + j] = pv[j] >= 0.f ? pv[j] * sp[qi][4 * u + j] : -pv[j] * dv[j];
        } else {
          (void)dl;
#pragma unroll
          for (int j = 0; j < 4; ++j) x[4 * u + j] = pv[j] * sp[qi][4 * u + j];
        }
      }
      fr[2 * qi] = pack_frag<BF16>(x, 0);
      fr[2 * qi + 1] = pack_frag<BF16>(x, 1);
    }
  };
  // P waves of the plain instantiations (no dropout, no mask, 2 q-tiles): S(it) -> P(it) ->
  // dV^T += dO(it)^T P(it) q-tile by q-tile.  The softmax of q-tile 0 (exp, fp32 store for the dS
  // waves, bf16 pack) is issued between the S MFMAs of q-tile 1 and that of q-tile 1 between the dV
  // MFMAs of q-tile 0, so it fills MFMA gaps instead of running as a VALU-only block between two
  // MFMA blocks (unfused: ~1000 of ~3400 cycles per slice on the P waves, tools/stamps.py).
  constexpr bool kFused = !DROPOUT && !MASKED && NQT == 2 && !FA_DKDV_UNFUSED_P;
  auto p_fused = [&](int it, int aq, int ao, char* xw, f32x16_t (&sp)[NQT]) {
    if constexpr (kFused) {
      const TileAddr ta(lb, aq), ta2(lb, ao);
      i16x8_t fr[2 * NQT];
      // half-piece h (0..7) of q-tile QF: elements 2h, 2h+1 of the lane's 16; the fp32 store of a row
      // group follows its odd half, the pack of a 16-row half follows h = 3 / 7
      auto half_piece = [&](auto QFC, auto HC) {
        constexpr int qf = decltype(QFC)::value, h = decltype(HC)::value;
        constexpr int u = h >> 1;
  #pragma unroll
        for (int j = 2 * (h & 1); j < 2 * (h & 1) + 2; ++j) sp[qf][4 * u + j] = fast_exp2(sp[qf][4 * u + j] * c);
        if constexpr (h & 1) {
          const f32x4_t pv = {sp[qf][4 * u], sp[qf][4 * u + 1], sp[qf][4 * u + 2], sp[qf][4 * u + 3]};
          *(f32x4_t*)(xw + qf * XTILE + u * 1024) = pv;
        }
        if constexpr ((h & 3) == 3) fr[2 * qf + (h >> 2)] = pack_frag<BF16>(sp[qf], h >> 2);
      };
      // an MFMA chain of N steps, operand k fetched two steps ahead, step k followed by fill(k)
      auto chain = [&](auto NC, auto&& load, auto&& mma, auto&& fill) {
        constexpr int N = decltype(NC)::value;
        i16x8_t a[3];
        a[0] = load(std::integral_constant<int, 0>{});
        if constexpr (N > 1) a[1] = load(std::integral_constant<int, 1>{});
        static_for<0, N>([&](auto KC) {
          constexpr int k = decltype(KC)::value;
          if constexpr (k + 2 < N) a[(k + 2) % 3] = load(std::integral_constant<int, k + 2>{});
          __builtin_amdgcn_sched_barrier(0);
          mma(KC, a[k % 3]);
          fill(KC);
          __builtin_amdgcn_sched_barrier(0);
        });
      };
      // fill of an N-step chain with the softmax of q-tile QF: half-pieces [8k/N, 8(k+1)/N) after step k
      auto softmax_fill = [&](auto QFC, auto NC) {
        return [&, QFC](auto KC) {
          constexpr int N = decltype(NC)::value, k = decltype(KC)::value;
          static_for<(8 * k) / N, (8 * (k + 1)) / N>([&](auto HC) { half_piece(QFC, HC); });
        };
      };
      auto no_fill = [](auto) {};
      auto s_chain = [&](auto QTC, auto&& fill) {
        constexpr int qt = decltype(QTC)::value;
        chain(std::integral_constant<int, KS>{},
              [&](auto KC) { return row_read_c<BQ, 32 * qt, 2 * decltype(KC)::value>(smem, ta); },
              [&](auto KC, const i16x8_t& a) { sp[qt] = E::mfma(a, kv[decltype(KC)::value], sp[qt]); },
              fill);
      };
      auto dv_chain = [&](auto QTC, auto&& fill) {
        constexpr int qt = decltype(QTC)::value;
        chain(std::integral_constant<int, 2 * NP>{},
              [&](auto KC) {
                constexpr int k = decltype(KC)::value;
                return tr_frag_c<BQ, 16 * (2 * qt + (k & 1)), k / 2>(smem, ta2);
              },
              [&](auto KC, const i16x8_t& a) {
                constexpr int k = decltype(KC)::value;
                acc[k / 2] = E::mfma(a, fr[2 * qt + (k & 1)], acc[k / 2]);
              },
              fill);
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      s_chain(I0{}, no_fill);
      s_chain(I1{}, softmax_fill(I0{}, std::integral_constant<int, KS>{}));
      FA_STAMP(3);
      dv_chain(I0{}, softmax_fill(I1{}, std::integral_constant<int, 2 * NP>{}));
      FA_STAMP(4);
      dv_chain(I1{}, no_fill);
    }
    (void)it; (void)aq; (void)ao; (void)xw; (void)sp;
  };
  auto xw_of = [&](int it) { return smem + XBASE + (it & 1) * XBUF + kg * NQT * XTILE + lane * 16; };

  // Static priority for the dS waves: on each SIMD the dS wave's step opens with its (short) VALU
  // block and then feeds the matrix pipe, while the P wave's exp-heavy block can wait; measured at
  // C3: dS waves at prio 1 +9%, P waves at prio 1 +5%, versus none.
#if defined(FA_DKDV_PRIO_NONE)
#elif defined(FA_DKDV_PRIO_P)
  if (pwave) __builtin_amdgcn_s_setprio(1);
#else
  if (!pwave) __builtin_amdgcn_s_setprio(1);
#endif
  // FlashMask slice skip: a slice is dead when the bounds hide every key of this workgroup from
  // every row of the slice (fm_tile_dead per 64 keys); all waves walk the same live slices
  auto slice_dead = [&](int sid) {
    if constexpr (!MASKED) {
      return false;
    } else {
      if (s.fm_lts == nullptr) return false;
      const int q0 = slice_q0(sid);
      const int64_t base = fm_base(s, bidb, h_begin + slice_head(sid));
#pragma unroll
      for (int k0 = 0; k0 < BKN; k0 += 64)
        if (!fm_tile_dead<CAUSAL>(s, base, n0 + k0, min(64, BKN - k0), sk, q0, min(q0 + BQ, sq), lane))
          return false;
      return true;
    }
  };
  auto next_live = [&](int sid) {
    if (sid >= total) return total;
    ++sid;
    while (sid < total && slice_dead(sid)) ++sid;
    return sid;
  };
  int sid = next_live(-1);
  if (sid < total) issue(slice_head(sid), slice_q0(sid), 0);
  wait_vmem_all();   // K/V fragments and slice 0 (compiler-visible: no vmcnt waits inside the loop)
  lds_barrier();

  // Each role runs its own copy of the slice loop (same trip count, the same one barrier per slice),
  // so each is register-allocated and scheduled for its own instruction mix:
  //   dS waves: dS''(it-1) from sp (VALU) | sp = dP''(it) (MFMA) | dK'' += Q(it-1)^T dS''(it-1)
  //   P waves:  sp = S(it) (MFMA) | P(it) (VALU) | dV += dO(it)^T P(it), fused q-tile by q-tile in the
  //             plain instantiations (p_fused)
  // unmasked walk: (query-slice index, head) of the current and the next slice, kept incrementally
  // (the slice id -> (head, row) division costs ~20 scalar instructions per use)
  const int sid0 = sid;
  // (DMAC: whether this loop's waves issue slice DMA -- the P waves' loop carries no DMA code, so
  // no DMA offsets stay live in it)
  // (DMAC: whether this loop's waves issue slice DMA -- the P waves' loop carries no DMA code, so
  // no DMA offsets stay live in it; NPC: the number of parts the DMA is issued in, part 0 at the
  // top of the step, part k by the body's dma(k))
  auto sweep = [&](auto DMAC, auto NPC, auto&& body) {
    constexpr bool DMA = decltype(DMAC)::value;
    int it = 0;   // ring position of slice sid (the same slice without a mask)
    int sd = sid0;
    int cq = 0, chd = 0, nqi = 1, nhd = 0;
    if (nqi == ns) { nqi = 0; nhd = 1; }
    for (; MASKED ? sd < total : it < total; ++it) {
      const int cur = MASKED ? sd : it;
      const int nxt = MASKED ? next_live(sd) : it + 1;
      FA_STAMP(0);
      const bool more = DMA && nxt < total;
      SliceDma d{};
      if (more) {
        if constexpr (MASKED) d = dma_plan(slice_head(nxt), slice_q0(nxt), it + 1);
        else d = dma_plan(nhd, (m_first + nqi) * BQ, it + 1);
      }
      if (more) dma_part(d, std::integral_constant<int, 0>{}, NPC);
      auto dma = [&](auto KC) {
        if (more) dma_part(d, KC, NPC);
      };
      FA_STAMP(1);
      const int q0 = MASKED ? slice_q0(cur) : (m_first + cq) * BQ;
      const int it_head = MASKED ? slice_head(cur) : chd;   // query head of this slice within the group
      body(it, q0, it_head, dma);
      FA_STAMP(5);
      wait_dma_keep_and_barrier(0);
      FA_STAMP(6);
      if constexpr (MASKED) sd = nxt;
      else {
        cq = nqi; chd = nhd;
        if (++nqi == ns) { nqi = 0; ++nhd; }
      }
    }
    return it;
  };
  // chain start: -LSE / scale (P waves) or D (dS waves) of the slice in ring position it, per row
  auto chain_init = [&](int it, f32x16_t (&sp)[NQT]) {
    const float* init = (const float*)(smem + (it % 3) * QSLOT + QTILE) + (pwave ? 0 : 64);
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4_t iv = *(const f32x4_t*)(init + 32 * qi + 8 * u + 4 * hh);
#pragma unroll
        for (int j = 0; j < 4; ++j) sp[qi][4 * u + j] = iv[j];
      }
  };

  int nlive;
  if (pwave) {
    nlive = sweep(std::bool_constant<DWN == NW>{}, std::integral_constant<int, 1>{},
                  [&](int it, int q0, int it_head, auto&&) {
      const int qs = (it % 3) * QSLOT, os = OBASE + (it & 1) * QTILE;
      f32x16_t sp[NQT];
      chain_init(it, sp);
      FA_STAMP(2);
      const bool fast = !MASKED && (q0 + BQ <= sq) && (n0 + BKN <= sk) && (!CAUSAL || q0 >= n0 + BKN - 1);
      if constexpr (kFused) {
        // masked elements (causal, ragged ends): the S' chain starts from -inf, so P = exp2(-inf) = 0
        // exactly (finite Q K^T), and the fused step itself carries no mask code
        if (!fast) {
#pragma unroll
          for (int qi = 0; qi < NQT; ++qi)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
              const int q = q0 + 32 * qi + 8 * (g >> 2) + 4 * hh + (g & 3);
              const bool out = (key >= sk) | (q >= sq) | (CAUSAL && key > q);
              sp[qi][g] = out ? kNegInf : sp[qi][g];
            }
        }
        p_fused(it, qs, os, xw_of(it), sp);
      } else {
        i16x8_t fr[2 * NQT];
        phase1(qs, sp);                       // S' = Q K^T - LSE/scale
        FA_STAMP(3);
        if (fast) p_step(std::false_type{}, sp, q0, it_head, xw_of(it), fr);
        else p_step(std::true_type{}, sp, q0, it_head, xw_of(it), fr);
        FA_STAMP(4);
        phase2(os, fr);                       // dV^T += dO^T P
      }
    });
  } else {
    f32x16_t sp[NQT];  // dP'' of the previous slice
    // DMA parts: at the top of the step, then after the dS step (bit 0 of FA_DKDV_DMA_POS) and
    // after phase 1 (bit 1)
    constexpr int kPos = FA_DKDV_DMA_POS;
    constexpr int kP1 = (kPos & 1) ? 1 : 0, kP2 = kP1 + ((kPos & 2) ? 1 : 0);
    nlive = sweep(std::true_type{}, std::integral_constant<int, 1 + kP2>{}, [&](int it, int, int, auto&& dma) {
      const int os = OBASE + (it & 1) * QTILE;
      i16x8_t fr[2 * NQT];
      if (it > 0) ds_step(sp, xw_of(it - 1), (const float*)(smem + ((it + 2) % 3) * QSLOT + QTILE) + 64, fr);
      if constexpr (kPos & 1) dma(std::integral_constant<int, kP1>{});
      FA_STAMP(2);
      chain_init(it, sp);
      phase1(os, sp);                         // dP'' = D - dO V^T
      if constexpr (kPos & 2) dma(std::integral_constant<int, kP2>{});
      FA_STAMP(3);
      FA_STAMP(4);
      if (it > 0) phase2(((it + 2) % 3) * QSLOT, fr);   // dK''^T += Q(it-1)^T dS''(it-1)
    });
    if (nlive > 0) {   // the last slice's dK update (no DMA after it: its Q is resident)
      i16x8_t fr[2 * NQT];
      ds_step(sp, xw_of(nlive - 1), (const float*)(smem + ((nlive - 1) % 3) * QSLOT + QTILE) + 64, fr);
      phase2(((nlive - 1) % 3) * QSLOT, fr);
    }
  }
  (void)nlive;

  // ---- epilogue: dV = (dV^T)^T from the P waves, dK = -scale * (dK''^T)^T from the dS waves ----
  if (key < sk) {
    const int hd = p.gqa_reduce ? kvh : hx;
    u16* row = pwave ? (u16*)p.dv + geo.dv_off + (int64_t)hd * p.dv_head + (int64_t)key * p.dv_row
                     : (u16*)p.dk + geo.dk_off + (int64_t)hd * p.dk_head + (int64_t)key * p.dk_row;
    const float rp = DROPOUT ? s.rp_dropout : 1.f;
    const float sc = pwave ? rp : -s.scale * rp;
#pragma unroll
    for (int dt = 0; dt < NP; ++dt)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int d0 = dt * 32 + 8 * u + 4 * hh;
        if (d0 < dlim) {
          u32x2_t w;
          w[0] = E::pack2(acc[dt][4 * u + 0] * sc, acc[dt][4 * u + 1] * sc);
          w[1] = E::pack2(acc[dt][4 * u + 2] * sc, acc[dt][4 * u + 3] * sc);
          *(u32x2_t*)(row + d0) = w;
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// 3. dQ  (forward-shaped: query on the lane, K/V streamed)
// ------------------------------------------------------------------------------------------------
template <bool BF16, int D, bool CAUSAL, bool DROPOUT, bool MASKED>
__global__ void __launch_bounds__(DqTile<D>::NW * 64, DqTile<D>::MINB) bwd_dq_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int NW = DqTile<D>::NW;
  constexpr int BN = DqTile<D>::BN;
  constexpr int BM = DqTile<D>::BM;
  constexpr int KS = D / 16;
  constexpr int NT = BN / 32;
  constexpr int NP = D / 32;
  constexpr int TILE = BN * D * 2;
  constexpr int PIECES = TILE / 1024;
  constexpr int PPW = (PIECES + NW - 1) / NW;
  constexpr int KG = (KS % 4 == 0) ? 4 : ((KS % 3 == 0) ? 3 : 2);
  static_assert(TILE % 1024 == 0 && KS % KG == 0, "tile shape");
  // Staggered halves (8-wave workgroups, as in fwd_kernel): waves 4-7 run the dQ MFMAs of each tile
  // one step late, so on every SIMD one wave opens its step with the S / dP MFMAs while its partner
  // opens with the dQ MFMAs of the previous tile and then the dS VALU.  The late dQ reads K(nb-1)
  // while tile nb+2 lands, hence a 4-deep ring.
  constexpr bool STAGGER = NW == 8 && FA_DQ_STAGGER;
  constexpr int BUFS = STAGGER ? 4 : kBwdBufs;
  // [buffer][K | V], then (dropout) NT 1-KiB random-byte scratch blocks per wave
  __shared__ __attribute__((aligned(16))) char smem[BUFS * 2 * TILE + (DROPOUT ? NW * NT * 1024 : 0)];

  const AttnShape s = p.s;
  const uint64_t pseed = DROPOUT ? philox_seed_of(s) : 0, poff = DROPOUT ? philox_offset_of(s) : 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const LdsBases lb(lane);
  const int num_m = (s.seqlen_q + BM - 1) / BM;
  // XCD-aware, heads grouped as in the forward (p.dq_head_group from launch_bwd)
  int bh, m_idx;
  xcd_order_grouped(blockIdx.x, s.b * s.h, num_m, p.dq_head_group, bh, m_idx);
  const int bidb = bh / s.h;
  const int head = bh - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int m_block = num_m - 1 - m_idx;   // heaviest causal block of a head first
  const SeqGeom geo = seq_geom(p, bidb);
  const int sq = geo.sq, sk = geo.sk;
  const int m0 = m_block * BM;
  if (m0 >= sq) return;
  const int dlim = s.d;

  const u16* __restrict__ K = (const u16*)p.k + geo.k_off + (int64_t)kvh * p.k_head;
  const u16* __restrict__ V = (const u16*)p.v + geo.v_off + (int64_t)kvh * p.v_head;
  const int64_t bhi = (int64_t)bidb * s.h + head;

  const int wq0 = m0 + 32 * wave;
  const int qi = wq0 + r;
  const bool q_ok = qi < sq;

  // Q and dO fragments: B operands of S^T = K Q^T and dP^T = V dO^T
  i16x8_t qf[KS], of[KS];
  {
    const u16* qrow = (const u16*)p.q + geo.q_off + (int64_t)head * p.q_head + (int64_t)(q_ok ? qi : 0) * p.q_row;
    const u16* orow = (const u16*)p.dout + geo.do_off + (int64_t)head * p.do_head + (int64_t)(q_ok ? qi : 0) * p.do_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      qf[ks] = __builtin_bit_cast(i16x8_t, ld16(qrow + d0, q_ok && d0 < dlim));
      of[ks] = __builtin_bit_cast(i16x8_t, ld16(orow + d0, q_ok && d0 < dlim));
    }
  }
  const float c = s.scale_log2;
  float lse_l2 = __builtin_huge_valf(), dsum_q = 0.f;
  if (q_ok) {
    lse_l2 = p.lse[bhi * s.lse_pitch + qi] * kLog2e;
    dsum_q = p.dsum[bhi * p.seqlen_q_rounded + qi];
  }

  const int n_end = CAUSAL ? min(sk, m0 + BM) : sk;
  const int nblk = n_end > 0 ? (n_end + BN - 1) / BN : 0;
  const int nfast = MASKED ? 0 : min(nblk, (CAUSAL ? min(sk, m0 + 1) : sk) / BN);
  const int64_t fmb = (MASKED && s.fm_lts) ? fm_base(s, bidb, head) : 0;
  const u16* mrow = MASKED ? mask_row_ptr(s, bidb, head, q_ok ? qi : 0) : nullptr;

  int voff_k[PPW], voff_v[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    voff_k[j] = dma_voff<BN>(wave + j * NW, lane, p.k_row, dlim);
    voff_v[j] = dma_voff<BN>(wave + j * NW, lane, p.v_row, dlim);
  }
  // K/V tile `nb` into ring position `pos` (the same except when FlashMask skips tiles)
  auto issue_at = [&](int nb, int pos) {
    const int n0 = nb * BN;
    char* dst = smem + (pos % BUFS) * 2 * TILE;
    const buf_rsrc_t rk = make_rsrc(K + (int64_t)n0 * p.k_row, rec_bytes(sk - n0, p.k_row, 2));
    const buf_rsrc_t rv = make_rsrc(V + (int64_t)n0 * p.v_row, rec_bytes(sk - n0, p.v_row, 2));
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = wave + j * NW;
      if (PIECES % NW == 0 || pc < PIECES) {
        dma16(rk, dst + pc * 1024, voff_k[j]);
        dma16(rv, dst + TILE + pc * 1024, voff_v[j]);
      }
    }
  };

  f32x16_t dq[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) dq[t][g] = 0.f;

  // S^T, dP^T and dS^T of tile nb (ring position pos), packed to df (the B operands of dQ^T)
  auto sdp = [&](auto MASKC, int nb, int pos, i16x8_t (&df)[2 * NT]) {
    constexpr bool MASK = decltype(MASKC)::value;
    const int n0 = nb * BN;
    const int kt = (pos % BUFS) * 2 * TILE;
    const TileAddr tk(lb, kt), tv(lb, kt + TILE);
    // dropout bytes of the tile's NT 32x32 blocks, generated before the S / dP chains (the Philox
    // temporaries then never overlap the live score tiles: generated inside the dS loop they made
    // the causal dropout instantiation spill ~140 registers).  dropout_lane_bytes hands each lane
    // its own 16 bytes (no cross-lane scatter); they wait in the lane's own 16-byte LDS slot, since
    // held in registers across the chains they spill (114-145 VGPRs).  Each slot is read back, and
    // the value used, before the next tile overwrites it.
    u32x4_t* const dslot = (u32x4_t*)(smem + BUFS * 2 * TILE + wave * NT * 1024) + lane;
    if constexpr (DROPOUT) {
      // the previous tile's reads of the slots must have returned before the slots are rewritten: a
      // wave's LDS store can overtake its own pending LDS load of the same address (fa_dropout.h),
      // and nothing else orders them (the compiler may issue these stores before it waits on the
      // previous tile's read)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint64_t doff = poff + (uint64_t)bhi * 32;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        unsigned w[4];
        dropout_lane_bytes(w, pseed, doff, wq0, n0 + 32 * t, lane);
        dslot[64 * t] = u32x4_t{w[0], w[1], w[2], w[3]};
      }
    }
    f32x16_t st[NT], pt[NT];
    static_for<0, NT>([&](auto T) {
      constexpr int t = decltype(T)::value;
#pragma unroll
      for (int g = 0; g < 16; ++g) { st[t][g] = 0.f; pt[t][g] = -dsum_q; }
      static_for<0, KS / KG>([&](auto GG) {
        constexpr int g0 = decltype(GG)::value * KG;
        i16x8_t ka[KG], va[KG];
        static_for<0, KG>([&](auto KK) {
          constexpr int ks = g0 + decltype(KK)::value;
          ka[ks - g0] = row_read_c<BN, t * 32, 2 * ks>(smem, tk);
          va[ks - g0] = row_read_c<BN, t * 32, 2 * ks>(smem, tv);
        });
#pragma unroll
        for (int k = 0; k < KG; ++k) {
          st[t] = E::mfma(ka[k], qf[g0 + k], st[t]);
          pt[t] = E::mfma(va[k], of[g0 + k], pt[t]);
        }
      });
    });
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      u32x4_t rb = {0u, 0u, 0u, 0u};
      if constexpr (DROPOUT) rb = dslot[64 * t];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        float pv;
        if constexpr (MASK) {
          const int kk = n0 + t * 32 + acc_row(g, hh);
          // non-short-circuit OR and exp2(-inf) = 0: selects, no per-lane branches
          bool out = (kk >= sk) | (CAUSAL && kk > qi);
          float sc = st[t][g];
          if constexpr (MASKED) {
            out = out || (s.fm_lts != nullptr && fm_masked<CAUSAL>(s, fmb + kk, qi));
            if (!out && mrow != nullptr) sc += E::to_f32(mrow[kk]) * s.mask_unscale;
          }
          pv = fast_exp2(out ? kNegInf : fmaf(sc, c, -lse_l2));
        } else {
          pv = fast_exp2(fmaf(st[t][g], c, -lse_l2));
        }
        // dS^T = P^T o (dP^T - D); dropped elements: -P D (reference flash_bwd_kernel.h:897-899)
        if constexpr (DROPOUT)
          pt[t][g] = dropout_keep(rb[g >> 2], g & 3, s.keep_u8) ? pv * pt[t][g] : -pv * dsum_q;
        else
          pt[t][g] = pv * pt[t][g];
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      df[2 * t] = pack_frag<BF16>(pt[t], 0);
      df[2 * t + 1] = pack_frag<BF16>(pt[t], 1);
    }
  };
  // dQ^T[d][q] += K^T[d][key] dS^T[key][q] with K^T from the tile at ring position pos
  auto dq_mma = [&](int pos, const i16x8_t (&df)[2 * NT]) {
    const TileAddr tk(lb, (pos % BUFS) * 2 * TILE);
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      i16x8_t a[2 * NT];
      static_for<0, 2 * NT>([&](auto KC) {
        constexpr int kk = decltype(KC)::value;
        a[kk] = tr_frag_c<BN, kk * 16, dt>(smem, tk);
      });
#pragma unroll
      for (int kk = 0; kk < 2 * NT; ++kk) dq[dt] = E::mfma(a[kk], df[kk], dq[dt]);
    });
  };
  auto tile = [&](auto MASKC, int nb, int pos) {
    i16x8_t df[2 * NT];
    sdp(MASKC, nb, pos, df);
    dq_mma(pos, df);
  };

  int ndma = 0;   // DMA operations one issue() leaves outstanding in this wave
#pragma unroll
  for (int j = 0; j < PPW; ++j)
    if (PIECES % NW == 0 || wave + j * NW < PIECES) ndma += 2;

  // FlashMask tile skip, as in fwd_kernel: all waves walk the same sequence of live tiles
  auto next_live = [&](int nb) {
    if (nb >= nblk) return nblk;
    ++nb;
    if constexpr (MASKED)
      if (s.fm_lts != nullptr)
        while (nb < nblk && fm_tile_dead<CAUSAL>(s, fmb, nb * BN, BN, sk, m0, min(m0 + BM, sq), lane)) ++nb;
    return nb;
  };
  const int tq0 = next_live(-1), tq1 = next_live(tq0);
  if (tq0 < nblk) issue_at(tq0, 0);
  wait_vmem_all();   // Q / dO fragments, LSE / D and tile 0 (compiler-visible)
  if (tq1 < nblk) issue_at(tq1, 1);
  lds_barrier();
  if (STAGGER && FA_DQ_PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if (!STAGGER || wave < NW / 2) {
    for (int nb = 0; nb < nfast; ++nb) {
      if (nb + 2 < nblk) issue_at(nb + 2, nb + 2);
      tile(std::false_type{}, nb, nb);
      wait_dma_keep_and_barrier(nb + 2 < nblk ? ndma : 0);
    }
  } else if (nfast > 0) {
    // late half: dQ of tile nb-1 (its dS^T carried across the barrier in dfp), then S / dP / dS of nb
    i16x8_t dfp[2 * NT];
    for (int nb = 0; nb < nfast; ++nb) {
      if (nb + 2 < nblk) issue_at(nb + 2, nb + 2);
      if (nb > 0) dq_mma(nb - 1, dfp);
      __builtin_amdgcn_sched_barrier(0);
      sdp(std::false_type{}, nb, nb, dfp);
      wait_dma_keep_and_barrier(nb + 2 < nblk ? ndma : 0);
    }
    // the last deferred dQ: K(nfast-1) stays resident until the general path issues tile nfast+3
    dq_mma(nfast - 1, dfp);
  }
  // ring position pos holds tile nb; a1 is the next live tile (already in flight)
  int nb = MASKED ? tq0 : nfast, a1 = MASKED ? tq1 : nfast + 1;
  for (int pos = nfast; nb < nblk; ++pos) {
    const int a2 = next_live(a1);
    if (a2 < nblk) issue_at(a2, pos + 2);
    if ((wq0 < sq) && (!CAUSAL || nb * BN <= wq0 + 31)) tile(std::true_type{}, nb, pos);
    wait_dma_keep_and_barrier(a2 < nblk ? ndma : 0);
    nb = a1; a1 = a2;
  }

  if (q_ok) {
    u16* drow = (u16*)p.dq + geo.dq_off + (int64_t)head * p.dq_head + (int64_t)qi * p.dq_row;
    const float sc = p.dq_scale * (DROPOUT ? s.rp_dropout : 1.f);
#pragma unroll
    for (int dt = 0; dt < NP; ++dt)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int d0 = dt * 32 + 8 * u + 4 * hh;
        if (d0 < dlim) {
          u32x2_t w;
          w[0] = E::pack2(dq[dt][4 * u + 0] * sc, dq[dt][4 * u + 1] * sc);
          w[1] = E::pack2(dq[dt][4 * u + 2] * sc, dq[dt][4 * u + 3] * sc);
          *(u32x2_t*)(drow + d0) = w;
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// dK/dV and dQ are independent once bwd_pre_kernel has written D and -LSE/scale, so they can run
// on two streams of the device, forked from and joined back into the caller's stream with events,
// and the two kernels' causal tails overlap instead of adding up (the reference launches its three
// backward kernels serially, flash_bwd_launch_template.h:49-88).  Modes (FLASH_ATTN_MI355X_BWD_OVERLAP,
// read once, or flash_attn_bwd_overlap(mode)): 0 both on the caller's stream (default: measured
// faster at C3, DESIGN.md "dQ overlap"), 1 dQ on a second stream of the same priority, 2 dQ on a
// lowest-priority stream, 3 dK/dV on a highest-priority stream and dQ on the caller's.
namespace {
struct SideStream {
  hipStream_t s[3] = {nullptr, nullptr, nullptr};   // per mode 1..3
  hipEvent_t fork = nullptr, join = nullptr;
};
std::mutex g_side_mu;
SideStream g_side[64];
int g_overlap = -1;
}  // namespace

void bwd_overlap_enable(int mode) {
  std::lock_guard<std::mutex> lk(g_side_mu);
  g_overlap = (mode >= 0 && mode <= 3) ? mode : 0;
}

template <bool BF16, int D, bool CAUSAL, bool DROPOUT>
static void run_bwd(const BwdParams& p, hipStream_t stream) {
  const int nheads_grid = p.gqa_reduce ? p.s.hk : p.s.h;
  const bool masked = p.s.mask != nullptr || p.s.fm_lts != nullptr;
  auto dkdv = [&](hipStream_t st) {
    dim3 grid(p.s.b * nheads_grid * p.num_n_blocks);   // 1-D, xcd_order
    prof_begin(kTimeBwdMain, st);
    if (p.lsed != nullptr)   // the assembly dK / dV kernel (launch_bwd chose it: fa_bwd_asm.cpp)
      launch_bwd_dkdv_asm(p, BF16, st);
    else if (masked)
      hipLaunchKernelGGL((bwd_dkdv_kernel<BF16, D, CAUSAL, DROPOUT, true>), grid, dim3(DkdvTile<D>::NW * 64), 0, st, p);
    else
      hipLaunchKernelGGL((bwd_dkdv_kernel<BF16, D, CAUSAL, DROPOUT, false>), grid, dim3(DkdvTile<D>::NW * 64), 0, st, p);
    prof_end(kTimeBwdMain, st);
  };
  auto dq = [&](hipStream_t st) {
    dim3 grid(p.s.b * p.s.h * ((p.s.seqlen_q + DqTile<D>::BM - 1) / DqTile<D>::BM));
    prof_begin(kTimeBwdDq, st);
    if ((D == 128 || D == 64) && !DROPOUT && !masked && dq_asm_applicable(p, p.fuse_pre)) {   // the assembly dQ kernel (fa_bwd_asm.cpp)
      BwdParams pa = p;   // (persistent: heads grouped per XCD as in the forward, knob 7)
      if (p.s.cu_seqlens_q == nullptr)
        pa.dq_head_group = xcd_head_group((long long)p.s.b * p.s.h, (p.s.seqlen_q + 255) / 256,
                                        4ll * p.s.b * p.s.seqlen_k * p.s.hk * p.s.d, p.s.causal,
                                        knob(kKnobAsmXcdGroupMinMiB));
      launch_bwd_dq_asm(pa, BF16, st);
    }
    else if (masked)
      hipLaunchKernelGGL((bwd_dq_kernel<BF16, D, CAUSAL, DROPOUT, true>), grid, dim3(DqTile<D>::NW * 64), 0, st, p);
    else
      hipLaunchKernelGGL((bwd_dq_kernel<BF16, D, CAUSAL, DROPOUT, false>), grid, dim3(DqTile<D>::NW * 64), 0, st, p);
    prof_end(kTimeBwdDq, st);
  };
  std::unique_lock<std::mutex> lk(g_side_mu);
  if (g_overlap < 0) {
    const char* e = std::getenv("FLASH_ATTN_MI355X_BWD_OVERLAP");
    g_overlap = (e != nullptr && e[0] >= '1' && e[0] <= '3' && e[1] == 0) ? e[0] - '0' : 0;
  }
  const int mode = g_overlap;
  int dev = 0;
  hipStream_t side = nullptr;
  SideStream* ss = nullptr;
  if (mode > 0 && hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
    ss = &g_side[dev];
    if (ss->fork == nullptr &&
        (hipEventCreateWithFlags(&ss->fork, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&ss->join, hipEventDisableTiming) != hipSuccess))
      throw std::runtime_error("flash_attn_bwd: creating the fork/join events failed");
    if (ss->s[mode - 1] == nullptr) {
      int least = 0, greatest = 0;
      if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
        throw std::runtime_error("flash_attn_bwd: stream priority range query failed");
      const int prio = mode == 1 ? 0 : mode == 2 ? least : greatest;
      if (hipStreamCreateWithPriority(&ss->s[mode - 1], hipStreamNonBlocking, prio) != hipSuccess)
        throw std::runtime_error("flash_attn_bwd: creating the side stream failed");
    }
    side = ss->s[mode - 1];
  }
  prof_begin(kTimeBwdBoth, stream);
  if (p.fuse_pre) {   // dQ writes D and the dK/dV scratch (no bwd_pre_kernel): dQ first, serially
    lk.unlock();
    dq(stream);
    dkdv(stream);
  } else if (side == nullptr) {
    lk.unlock();
    dkdv(stream);
    dq(stream);
  } else {
    // fork: the side stream waits for everything queued on the caller's stream so far (bwd_pre_kernel)
    if (hipEventRecord(ss->fork, stream) != hipSuccess || hipStreamWaitEvent(side, ss->fork, 0) != hipSuccess)
      throw std::runtime_error("flash_attn_bwd: stream fork failed");
    if (mode == 3) {
      dkdv(side);
      dq(stream);
    } else {
      dkdv(stream);
      dq(side);
    }
    // join: the caller's stream continues after the side stream's kernel
    if (hipEventRecord(ss->join, side) != hipSuccess || hipStreamWaitEvent(stream, ss->join, 0) != hipSuccess)
      throw std::runtime_error("flash_attn_bwd: stream join failed");
  }
  prof_end(kTimeBwdBoth, stream);
}

template <bool BF16, bool CAUSAL, bool DROPOUT>
static void dispatch_bwd_d(const BwdParams& p, hipStream_t stream) {
  const int d = p.s.d;
  if (d <= 32) run_bwd<BF16, 32, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 64) run_bwd<BF16, 64, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 96) run_bwd<BF16, 96, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 128) run_bwd<BF16, 128, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 160) run_bwd<BF16, 160, CAUSAL, DROPOUT>(p, stream);   // dedicated tiles (reference hdim160)
  else if (d <= 192) run_bwd<BF16, 192, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 224) run_bwd<BF16, 224, CAUSAL, DROPOUT>(p, stream);   // (reference hdim224)
  else if (d <= 256) run_bwd<BF16, 256, CAUSAL, DROPOUT>(p, stream);
  else throw std::runtime_error("flash_attn_bwd: head dim " + std::to_string(d) + " > 256");
}

void bwd_block_size(int d, int* block_m, int* block_n) {
  *block_m = d <= 128 ? DkdvTile<128>::BQ : DkdvTile<256>::BQ;
  *block_n = d <= 128 ? DkdvTile<128>::BN : DkdvTile<256>::BN;
}

template <bool BF16>
static void launch_bwd_t(const BwdParams& p, hipStream_t stream) {
  if (p.lse_s == nullptr) throw std::runtime_error("flash_attn_bwd: no scratch for the scaled LSE");
  if (!p.fuse_pre) {
    // (assembly dK / dV: also the zero rows up to the last 32-row group)
    const int rows = p.lsed != nullptr ? 32 * p.lsed_ng : p.s.seqlen_q;
    dim3 grid(p.s.b * p.s.h, (rows + 63) / 64);   // 64 rows per block (bwd_pre_kernel kPreRows)
    prof_begin(kTimeBwdPre, stream);
    hipLaunchKernelGGL((bwd_pre_kernel<BF16>), grid, dim3(256), 0, stream, p);
    prof_end(kTimeBwdPre, stream);
  }
  if (p.s.causal) {
    if (p.s.dropout) dispatch_bwd_d<BF16, true, true>(p, stream); else dispatch_bwd_d<BF16, true, false>(p, stream);
  } else {
    if (p.s.dropout) dispatch_bwd_d<BF16, false, true>(p, stream); else dispatch_bwd_d<BF16, false, false>(p, stream);
  }
}

void launch_bwd(const BwdParams& p_in, bool is_bf16, hipStream_t stream) {
  if (p_in.s.b <= 0 || p_in.s.h <= 0 || p_in.s.seqlen_q <= 0) return;
  if ((p_in.s.seqlen_q + 15) / 16 > 65535 ||
      (int64_t)p_in.s.b * p_in.s.h * ((p_in.s.seqlen_q + kDqMinBM - 1) / kDqMinBM) > 0x7fffffff ||
      (int64_t)p_in.s.b * p_in.s.h * p_in.num_n_blocks > 0x7fffffff)
    throw std::runtime_error("flash_attn_bwd: problem too large for the grid");
  BwdParams p = p_in;
  {
    const int bm = p.s.d <= 128 ? DqTile<128>::BM : DqTile<256>::BM;
    p.dq_head_group = xcd_head_group((long long)p.s.b * p.s.h, (p.s.seqlen_q + bm - 1) / bm,
                                     4ll * p.s.b * p.s.seqlen_k * p.s.hk * p.s.d, p.s.causal);
#ifdef FA_FWD_NOGROUP
    p.dq_head_group = 0;
#endif
  }
  // A folding call (attn_folds_q -- a pure function of the call, so it is the forward's decision
  // whatever knobs changed since): its forward scored with Q' = bf16/f16(c Q).  Score the backward
  // with the same Q' so that the recomputed P is the forward's -- S' = Q' K^T is c S in the log2
  // domain (c -> 1), -LSE / scale -> -LSE log2(e) (scale -> ln 2), dK = ln2 dS^T Q',
  // dQ = scale dS K (dq_scale).  Without this the backward's exact scores would disagree with the
  // forward's LSE by the rounding of Q' (e.g. a one-key row's P != 1).  Q' comes from the assembly
  // dQ kernel when it runs first (fused preprocessing: it converts its own Q fragments and stores
  // them for dK/dV), else from q_fold_kernel.
  p.dq_scale = p.s.scale;
  p.qfold = nullptr;
  const bool fold = attn_folds_q(p.s, is_bf16);
  const float fold_c = p.s.scale_log2;
  if (fold) {
    p.s.mask_unscale *= fold_c;   // (dense mask: its term joins the log2-domain scores)
    p.s.scale = kLn2;
    p.s.scale_log2 = 1.0f;
  }
  // the strides the kernels see for Q' (compact, QFoldArgs): the assembly dK/dV kernel reads Q'
  // there on both fold paths, so its 32-bit record limits are checked on these
  BwdParams pq = p;
  if (fold) {
    pq.q_batch = (int64_t)p.s.seqlen_q * p.s.h * p.s.d;
    pq.q_row = (int64_t)p.s.h * p.s.d;
    pq.q_head = p.s.d;
  }
  // softmax_scale == 0 (uniform attention) would make -LSE / scale infinite: a tiny positive scale
  // gives the same P to fp32 precision (P deviates from uniform by 1e-30 |S|) and dQ, dK ~ 1e-30.
  if (p.s.scale == 0.f) { p.s.scale = 1e-30f; p.s.scale_log2 = 1e-30f * kLog2e; }
  // scratch for -LSE / scale (HIP dK/dV): the caller's dq_accum (at least (b, h, seqlen_q_rounded)
  // fp32), else the stream-ordered allocator; the assembly dK/dV's [-LSE / scale | -D] groups
  // (2 x 32-row-rounded rows) always come from the allocator (the caller's buffer size is unknown)
  p.lsed = nullptr;
  p.lsed_ng = (p.s.seqlen_q + 31) / 32;
  const bool asm_dkdv = bwd_asm_applicable(pq);
  StreamScratch ws;
  p.lse_s = p.dq_accum;
  if (p.lse_s == nullptr || asm_dkdv) {
    const size_t bytes = asm_dkdv ? (size_t)p.s.b * p.s.h * p.lsed_ng * 64 * sizeof(float)
                                  : (size_t)p.s.b * p.s.h * p.seqlen_q_rounded * sizeof(float);
    if (!ws.alloc(bytes, stream))
      throw std::runtime_error("flash_attn_bwd: hipMallocAsync of the LSE scratch failed");
    if (asm_dkdv) {
      p.lsed = static_cast<float*>(ws.p);
      if (p.lse_s == nullptr) p.lse_s = p.lsed;   // (not read on this path)
    } else {
      p.lse_s = static_cast<float*>(ws.p);
    }
  }
  // knob 8: the assembly dQ kernel computes D itself and writes softmax_d and the dK/dV scratch
  // (with the fold the dQ kernel also stores Q' in the compact rows: their 256-row records must fit)
  p.fuse_pre = asm_dkdv && knob(kKnobFusePre) != 0 && (p.s.d == 128 || p.s.d == 64) && !p.s.dropout && p.s.mask == nullptr &&
               p.s.fm_lts == nullptr && dq_asm_applicable(p, true) && (!fold || dq_asm_applicable(pq, false));
  StreamScratch qfold;
  if (fold) {
    const int64_t hd = (int64_t)p.s.h * p.s.d;
    const int64_t rows = (int64_t)p.s.b * p.s.seqlen_q;   // varlen: total_q <= b max_seqlen_q
    if (!qfold.alloc((size_t)(rows * hd) * 2, stream))
      throw std::runtime_error("flash_attn_bwd: hipMallocAsync of the prescaled Q failed");
    if (p.fuse_pre) {   // the dQ kernel (first) converts and stores Q'; dK/dV reads it
      p.qfold = qfold.p;
      p.qfold_c = fold_c;
    } else {
      QFoldArgs a;
      a.q = p.q; a.qf = qfold.p;
      a.q_batch = p.q_batch; a.q_row = p.q_row; a.q_head = p.q_head;
      a.cu_seqlens_q = p.s.cu_seqlens_q; a.padded = p.s.varlen_padded_input;
      a.b = p.s.b; a.seqlen_q = p.s.seqlen_q; a.h = p.s.h; a.d = p.s.d;
      a.c = fold_c;
      launch_q_fold(a, is_bf16, stream);
      p.q = qfold.p;
      p.q_batch = pq.q_batch; p.q_row = pq.q_row; p.q_head = pq.q_head;
    }
  }
  if (is_bf16) launch_bwd_t<true>(p, stream); else launch_bwd_t<false>(p, stream);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_bwd launch: ") + hipGetErrorString(e));
}

}  // namespace fa

#ifdef FA_STAMPS
extern "C" int flash_attn_debug_stamps(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(fa::g_fa_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
