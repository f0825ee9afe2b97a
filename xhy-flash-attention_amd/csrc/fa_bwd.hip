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
//   2. bwd_dkdv_kernel  one workgroup (4 waves, one per SIMD, full 512-entry register file) per
//                       128-key block of a (batch, kv-head); each wave's 32 keys of K and V stay in
//                       registers, (Q, dO, LSE, D) slices of 64 query rows arrive by LDS-DMA two
//                       slices ahead into a 3-deep ring; dK^T / dV^T accumulate in registers over
//                       every slice (and, for GQA, every query head of the group) and are written
//                       once: 4 MFMA GEMMs per tile, no atomics.
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
//   * Row constants as the initial accumulator in dkdv: S starts at -LSE/scale and dP at -D.
//   * Slices / tiles that need no mask run a branch-free body (the two 32-row q-tiles of a slice,
//     resp. the S / dP chains of a tile, interleave in one basic block).
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

typedef unsigned short u16;

constexpr int kDkdvWaves = 4;
constexpr int kDkdvBN = 32 * kDkdvWaves;  // keys per dK/dV workgroup
constexpr int kDkdvBQ = 64;               // query rows per sweep step
constexpr int kDqWaves = 8;
constexpr int kDqBM = 32 * kDqWaves;      // query rows per dQ workgroup
constexpr int kDqBN = 64;                 // keys per streamed K/V tile
constexpr int kBwdBufs = 3;

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
  using E = Elt<BF16>;
  const AttnShape s = p.s;
  const int bh = blockIdx.x;
  const int bidb = bh / s.h, head = bh - bidb * s.h;
  const SeqGeom g = seq_geom(p, bidb);
  const int row = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int l16 = threadIdx.x & 15;
  if (row >= g.sq) return;
  const u16* O = (const u16*)p.o + g.o_off + (int64_t)head * p.o_head + (int64_t)row * p.o_row;
  const u16* dO = (const u16*)p.dout + g.do_off + (int64_t)head * p.do_head + (int64_t)row * p.do_row;
  float acc = 0.f;
  for (int c = l16; c < s.d / 8; c += 16) {
    const u32x4_t a = *(const u32x4_t*)(O + 8 * c);
    const u32x4_t b = *(const u32x4_t*)(dO + 8 * c);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      acc += E::to_f32(a[w] & 0xffff) * E::to_f32(b[w] & 0xffff);
      acc += E::to_f32(a[w] >> 16) * E::to_f32(b[w] >> 16);
    }
  }
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 16);
  if (l16 == 0) p.dsum[((int64_t)bidb * s.h + head) * p.seqlen_q_rounded + row] = acc;
}

// ------------------------------------------------------------------------------------------------
// 2. dK / dV
// ------------------------------------------------------------------------------------------------
template <bool BF16, int D, bool CAUSAL>
__global__ void __launch_bounds__(kDkdvWaves * 64, 1) bwd_dkdv_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int NW = kDkdvWaves;
  constexpr int BQ = kDkdvBQ;
  constexpr int KS = D / 16;
  constexpr int NP = D / 32;
  constexpr int QTILE = BQ * D * 2;                 // bytes of a Q or dO slice
  constexpr int SLICE = 2 * QTILE + 2 * BQ * 4;     // Q | dO | lse[BQ] | D[BQ]
  constexpr int PIECES = QTILE / 1024;
  constexpr int PPW = (PIECES + NW - 1) / NW;
  static_assert(QTILE % 1024 == 0, "slice must be whole DMA pieces");
  __shared__ __attribute__((aligned(16))) char smem[kBwdBufs * SLICE];

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const LdsBases lb(lane);
  const int group = s.h / s.hk;

  const int nheads_grid = p.gqa_reduce ? s.hk : s.h;
  const int bidb = blockIdx.x / nheads_grid;
  const int hx = blockIdx.x - bidb * nheads_grid;
  const int kvh = p.gqa_reduce ? hx : hx / group;
  const int h_begin = p.gqa_reduce ? hx * group : hx;
  const int nh = p.gqa_reduce ? group : 1;
  const SeqGeom geo = seq_geom(p, bidb);
  const int sq = geo.sq, sk = geo.sk;
  const int n0 = blockIdx.y * kDkdvBN;
  if (n0 >= sk) return;
  const int dlim = s.d;

  // ---- this wave's 32 keys: K / V fragments (B operands of S = Q K^T and dP = dO V^T) ----
  const int kw0 = n0 + 32 * wave;
  const int key = kw0 + r;
  i16x8_t kf[KS], vf[KS];
  {
    const bool ok = key < sk;
    const u16* krow = (const u16*)p.k + geo.k_off + (int64_t)kvh * p.k_head + (int64_t)(ok ? key : 0) * p.k_row;
    const u16* vrow = (const u16*)p.v + geo.v_off + (int64_t)kvh * p.v_head + (int64_t)(ok ? key : 0) * p.v_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      kf[ks] = __builtin_bit_cast(i16x8_t, ld16(krow + d0, ok && d0 < dlim));
      vf[ks] = __builtin_bit_cast(i16x8_t, ld16(vrow + d0, ok && d0 < dlim));
    }
  }

  // ---- query sweep: (head, BQ-row slice) pairs; causal: queries >= n0 only ----
  const int m_first = CAUSAL ? (n0 / BQ) : 0;
  const int m_count = (sq + BQ - 1) / BQ;
  const int ns = m_count > m_first ? m_count - m_first : 0;
  const int total = ns * nh;

  int voff_q[PPW], voff_o[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    voff_q[j] = dma_voff<BQ>(wave + j * NW, lane, p.q_row, dlim);
    voff_o[j] = dma_voff<BQ>(wave + j * NW, lane, p.do_row, dlim);
  }
  auto issue = [&](int it) {
    const int hq = h_begin + it / ns;
    const int q0 = (m_first + it % ns) * BQ;
    char* dst = smem + (it % kBwdBufs) * SLICE;
    const u16* Qp = (const u16*)p.q + geo.q_off + (int64_t)hq * p.q_head + (int64_t)q0 * p.q_row;
    const u16* Dp = (const u16*)p.dout + geo.do_off + (int64_t)hq * p.do_head + (int64_t)q0 * p.do_row;
    const buf_rsrc_t rq = make_rsrc(Qp, rec_bytes(sq - q0, p.q_row, 2));
    const buf_rsrc_t ro = make_rsrc(Dp, rec_bytes(sq - q0, p.do_row, 2));
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = wave + j * NW;
      if (PIECES % NW == 0 || pc < PIECES) {
        dma16(rq, dst + pc * 1024, voff_q[j]);
        dma16(ro, dst + QTILE + pc * 1024, voff_o[j]);
      }
    }
    if (wave < 2) {   // wave 0: LSE rows, wave 1: D rows (64 x 4 bytes each)
      const int64_t bhi = (int64_t)bidb * s.h + hq;
      const float* src = (wave == 0) ? p.lse + bhi * s.lse_pitch + q0 : p.dsum + bhi * p.seqlen_q_rounded + q0;
      dma4(make_rsrc(src, rec_bytes(sq - q0, 1, 4)), dst + 2 * QTILE + wave * BQ * 4, lane * 4);
    }
  };

  f32x16_t dvt[NP], dkt[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) { dvt[t][g] = 0.f; dkt[t][g] = 0.f; }

  const float inv_scale = 1.f / s.scale;
  const float c = s.scale_log2;

  // one 32-row q-tile QI of the slice at byte offset `so`; MASK adds the causal / bound masks
  auto qtile = [&](auto QIC, auto MASKC, int so, int q0) {
    constexpr int QI = decltype(QIC)::value;
    constexpr bool MASK = decltype(MASKC)::value;
    const int qa = q0 + 32 * QI;
    const TileAddr tq(lb, so), to(lb, so + QTILE);
    const float* lt = (const float*)(smem + so + 2 * QTILE);
    // S' = Q K^T - LSE/scale ; dP' = dO V^T - D      (query on registers, key on lane)
    f32x16_t sacc, pacc;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4_t lv = *(const f32x4_t*)(lt + 32 * QI + 8 * u + 4 * hh);
      const f32x4_t dv = *(const f32x4_t*)(lt + BQ + 32 * QI + 8 * u + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) { sacc[4 * u + j] = -lv[j] * inv_scale; pacc[4 * u + j] = -dv[j]; }
    }
    i16x8_t qa_f[KS], oa_f[KS];
    static_for<0, KS>([&](auto KK) {
      constexpr int ks = decltype(KK)::value;
      qa_f[ks] = row_read_c<BQ, 32 * QI, 2 * ks>(smem, tq);
      oa_f[ks] = row_read_c<BQ, 32 * QI, 2 * ks>(smem, to);
    });
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      sacc = E::mfma(qa_f[ks], kf[ks], sacc);
      pacc = E::mfma(oa_f[ks], vf[ks], pacc);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      float pv = fast_exp2(sacc[g] * c);
      if constexpr (MASK) {
        const int q = qa + acc_row(g, hh);
        if (key >= sk || q >= sq || (CAUSAL && key > q)) pv = 0.f;
      }
      sacc[g] = pv;
      pacc[g] = pv * pacc[g];
    }
    const i16x8_t pf0 = pack_frag<BF16>(sacc, 0), pf1 = pack_frag<BF16>(sacc, 1);
    const i16x8_t df0 = pack_frag<BF16>(pacc, 0), df1 = pack_frag<BF16>(pacc, 1);
    // dV^T += dO^T P ; dK^T += Q^T dS
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      const i16x8_t o0 = tr_frag_c<BQ, 32 * QI, dt>(smem, to);
      const i16x8_t o1 = tr_frag_c<BQ, 32 * QI + 16, dt>(smem, to);
      const i16x8_t q0f = tr_frag_c<BQ, 32 * QI, dt>(smem, tq);
      const i16x8_t q1f = tr_frag_c<BQ, 32 * QI + 16, dt>(smem, tq);
      dvt[dt] = E::mfma(o0, pf0, dvt[dt]);
      dvt[dt] = E::mfma(o1, pf1, dvt[dt]);
      dkt[dt] = E::mfma(q0f, df0, dkt[dt]);
      dkt[dt] = E::mfma(q1f, df1, dkt[dt]);
    });
  };

  // ---- pipelined pieces of the mask-free path ----
  // S' / dP' accumulators of 32-row q-tile QI of the slice at byte offset so
  // raw S = Q K^T and dP = dO V^T (chains start from a zero accumulator: no VALU init)
  auto sdp = [&](auto QIC, int so, f32x16_t& sacc, f32x16_t& pacc) {
    constexpr int QI = decltype(QIC)::value;
    const TileAddr tq(lb, so), to(lb, so + QTILE);
    i16x8_t qa_f[KS], oa_f[KS];
    static_for<0, KS>([&](auto KK) {
      constexpr int ks = decltype(KK)::value;
      qa_f[ks] = row_read_c<BQ, 32 * QI, 2 * ks>(smem, tq);
      oa_f[ks] = row_read_c<BQ, 32 * QI, 2 * ks>(smem, to);
    });
    const f32x16_t zero = {};
    sacc = E::mfma(qa_f[0], kf[0], zero);
    pacc = E::mfma(oa_f[0], vf[0], zero);
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) {
      sacc = E::mfma(qa_f[ks], kf[ks], sacc);
      pacc = E::mfma(oa_f[ks], vf[ks], pacc);
    }
  };
  // P = exp2(c S - LSE log2e), dS = P o (dP - D) -> packed B operands (no masks); the per-row
  // LSE / D of the accumulator rows come from the slice's LDS copy (4 x 16-byte broadcast reads)
  auto finish = [&](auto QIC, int so, f32x16_t& sacc, f32x16_t& pacc, i16x8_t (&fr)[4]) {
    constexpr int QI = decltype(QIC)::value;
    const float* lt = (const float*)(smem + so + 2 * QTILE);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4_t lv = *(const f32x4_t*)(lt + 32 * QI + 8 * u + 4 * hh);
      const f32x4_t dv = *(const f32x4_t*)(lt + BQ + 32 * QI + 8 * u + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int g = 4 * u + j;
        const float pv = fast_exp2(fmaf(sacc[g], c, -lv[j] * kLog2e));
        sacc[g] = pv;
        pacc[g] = pv * (pacc[g] - dv[j]);
      }
    }
    fr[0] = pack_frag<BF16>(sacc, 0); fr[1] = pack_frag<BF16>(sacc, 1);
    fr[2] = pack_frag<BF16>(pacc, 0); fr[3] = pack_frag<BF16>(pacc, 1);
  };
  // dV^T += dO^T P ; dK^T += Q^T dS for q-tile QI of the slice at so
  auto update = [&](auto QIC, int so, const i16x8_t (&fr)[4]) {
    constexpr int QI = decltype(QIC)::value;
    const TileAddr tq(lb, so), to(lb, so + QTILE);
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      const i16x8_t o0 = tr_frag_c<BQ, 32 * QI, dt>(smem, to);
      const i16x8_t o1 = tr_frag_c<BQ, 32 * QI + 16, dt>(smem, to);
      const i16x8_t q0f = tr_frag_c<BQ, 32 * QI, dt>(smem, tq);
      const i16x8_t q1f = tr_frag_c<BQ, 32 * QI + 16, dt>(smem, tq);
      dvt[dt] = E::mfma(o0, fr[0], dvt[dt]);
      dvt[dt] = E::mfma(o1, fr[1], dvt[dt]);
      dkt[dt] = E::mfma(q0f, fr[2], dkt[dt]);
      dkt[dt] = E::mfma(q1f, fr[3], dkt[dt]);
    });
  };
  const std::integral_constant<int, 0> QT0{};
  const std::integral_constant<int, 1> QT1{};
  static_assert(BQ == 64, "the pipelined path assumes two 32-row q-tiles per slice");
  auto is_fast = [&](int it) {
    const int q0 = (m_first + it % ns) * BQ;
    return (q0 + BQ <= sq) && (n0 + kDkdvBN <= sk) && (!CAUSAL || q0 >= n0 + kDkdvBN - 1);
  };

  if (total > 0) issue(0);
  if (total > 1) issue(1);
  wait_dma_and_barrier();

  int it = 0;
  while (it < total) {
    if (is_fast(it)) {
      // run of mask-free slices: S/dP of the next q-tile (MFMA) overlaps this q-tile's exp/pack (VALU)
      int it_end = it + 1;
      while (it_end < total && is_fast(it_end)) ++it_end;
      f32x16_t sa, pa, sb, pb;
      sdp(QT0, (it % kBwdBufs) * SLICE, sa, pa);
      for (; it < it_end; ++it) {
        if (it + 2 < total) issue(it + 2);
        const int so = (it % kBwdBufs) * SLICE;
        const int so_next = ((it + 1) % kBwdBufs) * SLICE;   // resident (or unused garbage at the end)
        i16x8_t fr[4];
        sdp(QT1, so, sb, pb);
        finish(QT0, so, sa, pa, fr);
        update(QT0, so, fr);
        sdp(QT0, so_next, sa, pa);
        finish(QT1, so, sb, pb, fr);
        update(QT1, so, fr);
        wait_dma_and_barrier();
      }
    } else {
      const int q0 = (m_first + it % ns) * BQ;
      if (it + 2 < total) issue(it + 2);
      const int so = (it % kBwdBufs) * SLICE;
      static_for<0, BQ / 32>([&](auto QIC) {
        const int qa = q0 + 32 * decltype(QIC)::value;
        if (qa < sq && !(CAUSAL && kw0 > qa + 31)) qtile(QIC, std::true_type{}, so, q0);
      });
      wait_dma_and_barrier();
      ++it;
    }
  }

  // ---- epilogue: dK = scale * (dK^T)^T, dV = (dV^T)^T ----
  if (key < sk) {
    const int hd = p.gqa_reduce ? kvh : hx;
    u16* dkrow = (u16*)p.dk + geo.dk_off + (int64_t)hd * p.dk_head + (int64_t)key * p.dk_row;
    u16* dvrow = (u16*)p.dv + geo.dv_off + (int64_t)hd * p.dv_head + (int64_t)key * p.dv_row;
    const float sc = s.scale;
#pragma unroll
    for (int dt = 0; dt < NP; ++dt)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int d0 = dt * 32 + 8 * u + 4 * hh;
        if (d0 < dlim) {
          u32x2_t wk, wv;
          wk[0] = E::pack2(dkt[dt][4 * u + 0] * sc, dkt[dt][4 * u + 1] * sc);
          wk[1] = E::pack2(dkt[dt][4 * u + 2] * sc, dkt[dt][4 * u + 3] * sc);
          wv[0] = E::pack2(dvt[dt][4 * u + 0], dvt[dt][4 * u + 1]);
          wv[1] = E::pack2(dvt[dt][4 * u + 2], dvt[dt][4 * u + 3]);
          *(u32x2_t*)(dkrow + d0) = wk;
          *(u32x2_t*)(dvrow + d0) = wv;
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// 3. dQ  (forward-shaped: query on the lane, K/V streamed)
// ------------------------------------------------------------------------------------------------
template <bool BF16, int D, bool CAUSAL>
__global__ void __launch_bounds__(kDqWaves * 64, 2) bwd_dq_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int NW = kDqWaves;
  constexpr int BN = kDqBN;
  constexpr int BM = kDqBM;
  constexpr int KS = D / 16;
  constexpr int NT = BN / 32;
  constexpr int NP = D / 32;
  constexpr int TILE = BN * D * 2;
  constexpr int PIECES = TILE / 1024;
  constexpr int PPW = (PIECES + NW - 1) / NW;
  constexpr int KG = (KS % 4 == 0) ? 4 : ((KS % 3 == 0) ? 3 : 2);
  static_assert(TILE % 1024 == 0 && KS % KG == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[kBwdBufs * 2 * TILE];  // [buffer][K | V]

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const LdsBases lb(lane);
  const int bidb = blockIdx.x / s.h;
  const int head = blockIdx.x - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int num_m = (s.seqlen_q + BM - 1) / BM;
  const int m_block = num_m - 1 - (int)blockIdx.y;   // heaviest causal blocks first
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
  const int nfast = min(nblk, (CAUSAL ? min(sk, m0 + 1) : sk) / BN);

  int voff_k[PPW], voff_v[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    voff_k[j] = dma_voff<BN>(wave + j * NW, lane, p.k_row, dlim);
    voff_v[j] = dma_voff<BN>(wave + j * NW, lane, p.v_row, dlim);
  }
  auto issue = [&](int nb) {
    const int n0 = nb * BN;
    char* dst = smem + (nb % kBwdBufs) * 2 * TILE;
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

  auto tile = [&](auto MASKC, int nb) {
    constexpr bool MASK = decltype(MASKC)::value;
    const int n0 = nb * BN;
    const int kt = (nb % kBwdBufs) * 2 * TILE;
    const TileAddr tk(lb, kt), tv(lb, kt + TILE);
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
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        float pv = fast_exp2(fmaf(st[t][g], c, -lse_l2));
        if constexpr (MASK) {
          const int kk = n0 + t * 32 + acc_row(g, hh);
          if (kk >= sk || (CAUSAL && kk > qi)) pv = 0.f;
        }
        pt[t][g] = pv * pt[t][g];     // dS^T = P^T o (dP^T - D)
      }
    // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
    i16x8_t df[2 * NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      df[2 * t] = pack_frag<BF16>(pt[t], 0);
      df[2 * t + 1] = pack_frag<BF16>(pt[t], 1);
    }
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

  if (nblk > 0) issue(0);
  if (nblk > 1) issue(1);
  wait_dma_and_barrier();
  for (int nb = 0; nb < nfast; ++nb) {
    if (nb + 2 < nblk) issue(nb + 2);
    tile(std::false_type{}, nb);
    wait_dma_and_barrier();
  }
  for (int nb = nfast; nb < nblk; ++nb) {
    if (nb + 2 < nblk) issue(nb + 2);
    if ((wq0 < sq) && (!CAUSAL || nb * BN <= wq0 + 31)) tile(std::true_type{}, nb);
    wait_dma_and_barrier();
  }

  if (q_ok) {
    u16* drow = (u16*)p.dq + geo.dq_off + (int64_t)head * p.dq_head + (int64_t)qi * p.dq_row;
    const float sc = s.scale;
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
template <bool BF16, int D, bool CAUSAL>
static void run_bwd(const BwdParams& p, hipStream_t stream) {
  const int nheads_grid = p.gqa_reduce ? p.s.hk : p.s.h;
  {
    dim3 grid(p.s.b * nheads_grid, p.num_n_blocks);
    prof_begin(kTimeBwdMain, stream);
    hipLaunchKernelGGL((bwd_dkdv_kernel<BF16, D, CAUSAL>), grid, dim3(kDkdvWaves * 64), 0, stream, p);
    prof_end(kTimeBwdMain, stream);
  }
  {
    dim3 grid(p.s.b * p.s.h, (p.s.seqlen_q + kDqBM - 1) / kDqBM);
    prof_begin(kTimeBwdDq, stream);
    hipLaunchKernelGGL((bwd_dq_kernel<BF16, D, CAUSAL>), grid, dim3(kDqWaves * 64), 0, stream, p);
    prof_end(kTimeBwdDq, stream);
  }
}

template <bool BF16, bool CAUSAL>
static void dispatch_bwd_d(const BwdParams& p, hipStream_t stream) {
  const int d = p.s.d;
  if (d <= 32) run_bwd<BF16, 32, CAUSAL>(p, stream);
  else if (d <= 64) run_bwd<BF16, 64, CAUSAL>(p, stream);
  else if (d <= 96) run_bwd<BF16, 96, CAUSAL>(p, stream);
  else if (d <= 128) run_bwd<BF16, 128, CAUSAL>(p, stream);
  else throw std::runtime_error("flash_attn_bwd: head dim " + std::to_string(d) + " > 128 not built yet");
}

void bwd_block_size(int d, int* block_m, int* block_n) {
  *block_m = kDkdvBQ;
  *block_n = kDkdvBN;
  (void)d;
}

template <bool BF16>
static void launch_bwd_t(const BwdParams& p, hipStream_t stream) {
  {
    dim3 grid(p.s.b * p.s.h, (p.s.seqlen_q + 15) / 16);
    prof_begin(kTimeBwdPre, stream);
    hipLaunchKernelGGL((bwd_pre_kernel<BF16>), grid, dim3(256), 0, stream, p);
    prof_end(kTimeBwdPre, stream);
  }
  if (p.s.causal) dispatch_bwd_d<BF16, true>(p, stream); else dispatch_bwd_d<BF16, false>(p, stream);
}

void launch_bwd(const BwdParams& p, bool is_bf16, hipStream_t stream) {
  if (p.s.b <= 0 || p.s.h <= 0 || p.s.seqlen_q <= 0) return;
  if ((p.s.seqlen_q + kDqBM - 1) / kDqBM > 65535 || (p.s.seqlen_q + 15) / 16 > 65535)
    throw std::runtime_error("flash_attn_bwd: seqlen_q too large for the grid");
  if (is_bf16) launch_bwd_t<true>(p, stream); else launch_bwd_t<false>(p, stream);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_bwd launch: ") + hipGetErrorString(e));
}

}  // namespace fa
