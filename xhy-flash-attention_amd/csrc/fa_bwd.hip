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
//   2. bwd_dkdv_kernel  one workgroup per 128-key block of a (batch, kv-head); K and V fragments
//                       live in registers, 64-row (Q, dO) slices stream through LDS; dK^T / dV^T
//                       accumulate in registers over every query slice (and, for GQA, every query
//                       head of the group) and are written once: 4 MFMA GEMMs per tile, no atomics.
//   3. bwd_dq_kernel    one workgroup per 128-row query block, structured like the forward: Q and
//                       dO fragments in registers, K/V tiles streamed through LDS, S^T and dP^T with
//                       the query on the MFMA lane (LSE and D become per-lane scalars), dQ^T += K^T dS^T
//                       with dS^T used in-register as the MFMA B operand; dQ written directly in
//                       bf16/f16 (no fp32 accumulator buffer, no conversion pass).
// Both main kernels are deterministic (no atomics), so dQ is bitwise reproducible too.
//
//   * "Key on the lane" in dkdv: S = Q K^T and dP = dO V^T have the key on the MFMA column, so
//     their accumulators are directly the B operands of dV^T = dO^T P and dK^T = Q^T dS; dO^T and
//     Q^T come from the row-major LDS slice through ds_read_b64_tr_b16.
//   * Row constants as the initial accumulator in dkdv: S starts at -LSE/scale and dP at -D.
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

typedef unsigned short u16;

constexpr int kDkdvWaves = 4;
constexpr int kDkdvBN = 32 * kDkdvWaves;  // keys per dK/dV workgroup
constexpr int kDkdvBQ = 64;               // query rows per sweep step
constexpr int kDqBM = 128;                // query rows per dQ workgroup (4 waves x 32)
constexpr int kDqBN = 64;                 // keys per streamed K/V tile

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
__global__ void __launch_bounds__(256, 1) bwd_dkdv_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int BQ = kDkdvBQ;
  constexpr int KS = D / 16;
  constexpr int NP = D / 32;
  constexpr int QTILE = BQ * D * 2;                 // bytes of a Q or dO slice
  constexpr int SLICE = 2 * QTILE + 2 * BQ * 4;     // Q | dO | lse[BQ] | dsum[BQ]
  constexpr int QPAIR = BQ * NP / 2;                // (2 rows x 64 B) staging units per slice
  constexpr int QLOADS = (QPAIR + 31) / 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * SLICE];

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, i16 = lane & 15;
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

  u32x4_t stq[QLOADS], sto[QLOADS];
  float st_ld = 0.f;
  auto issue = [&](int it) {
    const int hq = h_begin + it / ns;
    const int q0 = (m_first + it % ns) * BQ;
    const u16* Qp = (const u16*)p.q + geo.q_off + (int64_t)hq * p.q_head;
    const u16* Dp = (const u16*)p.dout + geo.do_off + (int64_t)hq * p.do_head;
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      const int panel = pid % NP;
      const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
      const int d0 = panel * 32 + (tid & 3) * 8;
      const int qrow = q0 + row;
      const bool ok = (pid < QPAIR) && qrow < sq && d0 < dlim;
      const int64_t qr = ok ? qrow : 0;
      stq[i] = ld16(Qp + qr * p.q_row + d0, ok);
      sto[i] = ld16(Dp + qr * p.do_row + d0, ok);
    }
    if (tid < 2 * BQ) {   // [0, BQ): lse, [BQ, 2BQ): D
      const int row = tid & (BQ - 1);
      const int qrow = q0 + row;
      const int64_t bhi = (int64_t)bidb * s.h + hq;
      if (qrow < sq) st_ld = (tid < BQ) ? p.lse[bhi * s.lse_pitch + qrow] : p.dsum[bhi * p.seqlen_q_rounded + qrow];
      else st_ld = (tid < BQ) ? __builtin_huge_valf() : 0.f;
    }
  };
  auto commit = [&](int buf) {
    char* qt = smem + buf * SLICE;
    char* ot = qt + QTILE;
    float* lt = (float*)(qt + 2 * QTILE);
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      if (QPAIR % 32 == 0 || pid < QPAIR) {
        const int panel = pid % NP;
        const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
        const int off = panel_off(row, panel * 4 + (tid & 3), BQ);
        *(u32x4_t*)(qt + off) = stq[i];
        *(u32x4_t*)(ot + off) = sto[i];
      }
    }
    if (tid < 2 * BQ) lt[tid] = st_ld;
  };

  f32x16_t dvt[NP], dkt[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) { dvt[t][g] = 0.f; dkt[t][g] = 0.f; }

  const float inv_scale = 1.f / s.scale;
  const float c = s.scale_log2;

  if (total > 0) {
    issue(0);
    commit(0);
  }
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int q0 = (m_first + it % ns) * BQ;
    const bool has_next = it + 1 < total;
    if (has_next) issue(it + 1);

    const char* qt = smem + cur * SLICE;
    const char* ot = qt + QTILE;
    const float* lt = (const float*)(qt + 2 * QTILE);

#pragma unroll
    for (int qi = 0; qi < BQ / 32; ++qi) {
      const int qa = q0 + 32 * qi;   // first query row of this 32-row tile
      const bool skip = (qa >= sq) || (CAUSAL && kw0 > qa + 31);
      if (!skip) {
        // S' = Q K^T - LSE/scale ; dP' = dO V^T - D      (query on registers, key on lane)
        f32x16_t sacc, pacc;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4_t lv = *(const f32x4_t*)(lt + 32 * qi + 8 * u + 4 * hh);
          const f32x4_t dv = *(const f32x4_t*)(lt + BQ + 32 * qi + 8 * u + 4 * hh);
#pragma unroll
          for (int j = 0; j < 4; ++j) { sacc[4 * u + j] = -lv[j] * inv_scale; pacc[4 * u + j] = -dv[j]; }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          sacc = E::mfma(row_read(qt, 32 * qi + r, 2 * ks + hh, BQ), kf[ks], sacc);
          pacc = E::mfma(row_read(ot, 32 * qi + r, 2 * ks + hh, BQ), vf[ks], pacc);
        }
        const bool need_mask = (key >= sk) || (qa + 32 > sq) || (CAUSAL && kw0 + 31 > qa);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          float pv = fast_exp2(sacc[g] * c);
          if (need_mask) {
            const int q = qa + acc_row(g, hh);
            if (key >= sk || q >= sq || (CAUSAL && key > q)) pv = 0.f;
          }
          sacc[g] = pv;
          pacc[g] = pv * pacc[g];
        }
        const i16x8_t pf0 = pack_frag<BF16>(sacc, 0), pf1 = pack_frag<BF16>(sacc, 1);
        const i16x8_t df0 = pack_frag<BF16>(pacc, 0), df1 = pack_frag<BF16>(pacc, 1);
        // dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
        for (int dt = 0; dt < NP; ++dt) {
          const int col0 = dt * 32 + 16 * (r >> 4);
          dvt[dt] = E::mfma(tr_frag(ot, 32 * qi + 4 * hh, col0, BQ, i16), pf0, dvt[dt]);
          dvt[dt] = E::mfma(tr_frag(ot, 32 * qi + 16 + 4 * hh, col0, BQ, i16), pf1, dvt[dt]);
          dkt[dt] = E::mfma(tr_frag(qt, 32 * qi + 4 * hh, col0, BQ, i16), df0, dkt[dt]);
          dkt[dt] = E::mfma(tr_frag(qt, 32 * qi + 16 + 4 * hh, col0, BQ, i16), df1, dkt[dt]);
        }
      }
    }
    if (has_next) commit(cur ^ 1);
    __syncthreads();
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
__global__ void __launch_bounds__(256, 1) bwd_dq_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int BN = kDqBN;
  constexpr int KS = D / 16;
  constexpr int NT = BN / 32;
  constexpr int NP = D / 32;
  constexpr int TILE = BN * D * 2;
  constexpr int NPAIR = BN * NP / 2;
  constexpr int LOADS = (NPAIR + 31) / 32;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buffer][K | V]

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, i16 = lane & 15;
  const int bidb = blockIdx.x / s.h;
  const int head = blockIdx.x - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int num_m = (s.seqlen_q + kDqBM - 1) / kDqBM;
  const int m_block = num_m - 1 - (int)blockIdx.y;   // heaviest causal blocks first
  const SeqGeom geo = seq_geom(p, bidb);
  const int sq = geo.sq, sk = geo.sk;
  const int m0 = m_block * kDqBM;
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

  const int n_end = CAUSAL ? min(sk, m0 + kDqBM) : sk;
  const int nblk = n_end > 0 ? (n_end + BN - 1) / BN : 0;

  u32x4_t stk[LOADS], stv[LOADS];
  auto issue = [&](int n0) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      const int panel = pid % NP;
      const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
      const int d0 = panel * 32 + (tid & 3) * 8;
      const int kr = n0 + row;
      const bool ok = (pid < NPAIR) && kr < sk && d0 < dlim;
      const int64_t rr = ok ? kr : 0;
      stk[i] = ld16(K + rr * p.k_row + d0, ok);
      stv[i] = ld16(V + rr * p.v_row + d0, ok);
    }
  };
  auto commit = [&](int buf) {
    char* kt = smem + buf * 2 * TILE;
    char* vt = kt + TILE;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      if (NPAIR % 32 == 0 || pid < NPAIR) {
        const int panel = pid % NP;
        const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
        const int off = panel_off(row, panel * 4 + (tid & 3), BN);
        *(u32x4_t*)(kt + off) = stk[i];
        *(u32x4_t*)(vt + off) = stv[i];
      }
    }
  };

  f32x16_t dq[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) dq[t][g] = 0.f;

  if (nblk > 0) {
    issue(0);
    commit(0);
    __syncthreads();
  }
  for (int nb = 0; nb < nblk; ++nb) {
    const int n0 = nb * BN;
    const int cur = nb & 1;
    const bool has_next = nb + 1 < nblk;
    if (has_next) issue(n0 + BN);
    const char* kt = smem + cur * 2 * TILE;
    const char* vt = kt + TILE;
    const bool active = (wq0 < sq) && (!CAUSAL || n0 <= wq0 + 31);
    if (active) {
      f32x16_t st[NT], pt[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int g = 0; g < 16; ++g) { st[t][g] = 0.f; pt[t][g] = -dsum_q; }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          st[t] = E::mfma(row_read(kt, t * 32 + r, 2 * ks + hh, BN), qf[ks], st[t]);
          pt[t] = E::mfma(row_read(vt, t * 32 + r, 2 * ks + hh, BN), of[ks], pt[t]);
        }
      }
      const bool need_mask = (n0 + BN > sk) || (CAUSAL && n0 + BN - 1 > wq0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          float pv = fast_exp2(fmaf(st[t][g], c, -lse_l2));
          if (need_mask) {
            const int kk = n0 + t * 32 + acc_row(g, hh);
            if (kk >= sk || (CAUSAL && kk > qi)) pv = 0.f;
          }
          pt[t][g] = pv * pt[t][g];     // dS^T = P^T o (dP^T - D)
        }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const i16x8_t d0f = pack_frag<BF16>(pt[t], 0), d1f = pack_frag<BF16>(pt[t], 1);
#pragma unroll
        for (int dt = 0; dt < NP; ++dt) {
          const int col0 = dt * 32 + 16 * (r >> 4);
          dq[dt] = E::mfma(tr_frag(kt, t * 32 + 4 * hh, col0, BN, i16), d0f, dq[dt]);
          dq[dt] = E::mfma(tr_frag(kt, t * 32 + 16 + 4 * hh, col0, BN, i16), d1f, dq[dt]);
        }
      }
    }
    if (has_next) commit(cur ^ 1);
    __syncthreads();
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
    hipLaunchKernelGGL((bwd_dkdv_kernel<BF16, D, CAUSAL>), grid, dim3(256), 0, stream, p);
    prof_end(kTimeBwdMain, stream);
  }
  {
    dim3 grid(p.s.b * p.s.h, (p.s.seqlen_q + kDqBM - 1) / kDqBM);
    prof_begin(kTimeBwdDq, stream);
    hipLaunchKernelGGL((bwd_dq_kernel<BF16, D, CAUSAL>), grid, dim3(256), 0, stream, p);
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
