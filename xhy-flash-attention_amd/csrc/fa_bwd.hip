// FlashAttention-2 backward for MI355X (gfx950): dQ, dK, dV with the softmax recomputed from LSE.
//
// Algorithm (the reference's seqk-parallel backward, csrc/flash_attn/src/flash_bwd_launch_template.h:49-88):
//   1. bwd_pre_kernel   D[b,h,i] = sum_d dO[i,d] * O[i,d]; clears the fp32 dQ accumulator
//                       (reference compute_dot_do_o, flash_bwd_kernel.h:112-188);
//   2. bwd_main_kernel  per key block: K, V resident; sweep query rows recomputing
//                       P = exp(scale*QK^T - LSE), dP = dO V^T, dS = P o (dP - D);
//                       dV += P^T dO, dK += dS^T Q in registers; dQ += dS K through fp32 atomics
//                       (reference compute_dq_dk_dv_1colblock, flash_bwd_kernel.h:426-1113);
//   3. bwd_dq_kernel    dQ = scale * dQ_accum -> bf16/f16 (reference convert_dQ, :232-310).
//
// MI355X mapping:
//   * 4 waves x 32 keys = 128-key block per workgroup; each wave keeps dK^T and dV^T of its 32 keys
//     in accumulator registers for the whole sweep, so dK / dV are written once, deterministically.
//   * "Key on the lane": S = Q K^T and dP = dO V^T are computed with the key on the MFMA column, so
//     their accumulators are directly the B operands of dV^T = dO^T P and dK^T = Q^T dS (no LDS for
//     P or dS there); dO^T and Q^T come from the row-major LDS tiles via ds_read_b64_tr_b16.
//   * Row constants as the initial accumulator: S starts at -LSE/scale and dP at -D, so
//     p = exp2(scale*log2e * S') and dS = p * dP' need no per-element subtraction.
//   * dS crosses LDS once (as a dS^T image written with 8-byte stores) for dQ = dS K, which the 4
//     waves split by 32-wide d tiles and add into dq_accum with full-row f32 atomics.
//   * GQA: with gqa_reduce the workgroup owns a (batch, kv-head) pair and sweeps every query head of
//     its group, so dK/dV are summed in registers (no expanded buffers, no extra HBM pass).
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

typedef unsigned short u16;

// ------------------------------------------------------------------------------------------------
// 1. D = rowsum(dO * O), dq_accum rows cleared.   One 16-lane group per query row.
// ------------------------------------------------------------------------------------------------
template <bool BF16>
__global__ void __launch_bounds__(256) bwd_pre_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  const AttnShape s = p.s;
  const int bh = blockIdx.x;
  const int bidb = bh / s.h, head = bh - bidb * s.h;
  int sq = s.seqlen_q;
  int64_t o_off = (int64_t)bidb * p.o_batch, do_off = (int64_t)bidb * p.do_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) { o_off = (int64_t)c0 * p.o_row; do_off = (int64_t)c0 * p.do_row; }
  }
  const int row = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int l16 = threadIdx.x & 15;
  if (row >= sq) return;
  const u16* O = (const u16*)p.o + o_off + (int64_t)head * p.o_head + (int64_t)row * p.o_row;
  const u16* dO = (const u16*)p.dout + do_off + (int64_t)head * p.do_head + (int64_t)row * p.do_row;
  float acc = 0.f;
  for (int c = l16; c < s.d / 8; c += 16) {
    const u32x4_t a = *(const u32x4_t*)(O + 8 * c);
    const u32x4_t g = *(const u32x4_t*)(dO + 8 * c);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      acc += E::to_f32(a[w] & 0xffff) * E::to_f32(g[w] & 0xffff);
      acc += E::to_f32(a[w] >> 16) * E::to_f32(g[w] >> 16);
    }
  }
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 16);
  const int64_t bhi = (int64_t)bidb * s.h + head;
  if (l16 == 0) p.dsum[bhi * p.seqlen_q_rounded + row] = acc;
  float* dqa = p.dq_accum + (bhi * p.seqlen_q_rounded + row) * p.d_rounded;
  const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
  for (int c = l16; c < p.d_rounded / 4; c += 16) *(f32x4_t*)(dqa + 4 * c) = z;
}

// ------------------------------------------------------------------------------------------------
// 2. main kernel
// ------------------------------------------------------------------------------------------------
constexpr int kBwdWaves = 4;
constexpr int kBwdBN = 32 * kBwdWaves;  // keys per workgroup
constexpr int kBwdBQ = 32;              // query rows per sweep step

template <bool BF16, int D, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) bwd_main_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  constexpr int KS = D / 16;
  constexpr int NP = D / 32;
  constexpr int QTILE = kBwdBQ * D * 2;           // bytes of a Q or dO slice
  constexpr int KTILE = kBwdBN * D * 2;           // bytes of the K image
  constexpr int SLICE = 2 * QTILE + 2 * kBwdBQ * 4;  // Q | dO | lse | dsum
  constexpr int DST = kBwdBN * kBwdBQ * 2;        // dS^T image [128 keys][32 q]
  constexpr int QPAIR = kBwdBQ * NP / 2;          // staging units of a 32-row slice
  constexpr int QLOADS = (QPAIR + 31) / 32;
  constexpr int KPAIR = kBwdBN * NP / 2;
  constexpr int KLOADS = (KPAIR + 31) / 32;
  __shared__ __attribute__((aligned(16))) char smem[KTILE + 2 * SLICE + DST];
  char* const k_img = smem;
  char* const ds_img = smem + KTILE + 2 * SLICE;

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, i16 = lane & 15;
  const int group = s.h / s.hk;

  const int bx = blockIdx.x;
  const int nheads_grid = p.gqa_reduce ? s.hk : s.h;
  const int bidb = bx / nheads_grid;
  const int hx = bx - bidb * nheads_grid;
  const int kvh = p.gqa_reduce ? hx : hx / group;
  const int h_begin = p.gqa_reduce ? hx * group : hx;
  const int nh = p.gqa_reduce ? group : 1;
  const int n_block = blockIdx.y;

  int sq = s.seqlen_q, sk = s.seqlen_k;
  int64_t q_off = (int64_t)bidb * p.q_batch, do_off = (int64_t)bidb * p.do_batch;
  int64_t k_off = (int64_t)bidb * p.k_batch, v_off = (int64_t)bidb * p.v_batch;
  int64_t dk_off = (int64_t)bidb * p.dk_batch, dv_off = (int64_t)bidb * p.dv_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) { q_off = (int64_t)c0 * p.q_row; do_off = (int64_t)c0 * p.do_row; }
  }
  if (s.cu_seqlens_k) {
    const int c0 = s.cu_seqlens_k[bidb];
    sk = s.cu_seqlens_k[bidb + 1] - c0;
    if (!s.varlen_padded_input) {
      k_off = (int64_t)c0 * p.k_row; v_off = (int64_t)c0 * p.v_row;
      dk_off = (int64_t)c0 * p.dk_row; dv_off = (int64_t)c0 * p.dv_row;
    }
  }
  const int n0 = n_block * kBwdBN;
  if (n0 >= sk) return;
  const int dlim = s.d;

  const u16* __restrict__ Kp = (const u16*)p.k + k_off + (int64_t)kvh * p.k_head;
  const u16* __restrict__ Vp = (const u16*)p.v + v_off + (int64_t)kvh * p.v_head;

  // ---- K image (for dQ) and this wave's K / V fragments (B operands of S and dP) ----
  {
#pragma unroll
    for (int i = 0; i < KLOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      const int panel = pid % NP;
      const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
      const int d0 = panel * 32 + (tid & 3) * 8;
      const bool ok = (pid < KPAIR) && (n0 + row < sk) && d0 < dlim;
      const u32x4_t v = ld16(Kp + (int64_t)(ok ? n0 + row : 0) * p.k_row + d0, ok);
      if (KPAIR % 32 == 0 || pid < KPAIR) *(u32x4_t*)(k_img + panel_off(row, panel * 4 + (tid & 3), kBwdBN)) = v;
    }
  }
  const int key = n0 + 32 * wave + r;  // this lane's key (MFMA column)
  i16x8_t kf[KS], vf[KS];
  {
    const bool ok = key < sk;
    const u16* krow = Kp + (int64_t)(ok ? key : 0) * p.k_row;
    const u16* vrow = Vp + (int64_t)(ok ? key : 0) * p.v_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      kf[ks] = __builtin_bit_cast(i16x8_t, ld16(krow + d0, ok && d0 < dlim));
      vf[ks] = __builtin_bit_cast(i16x8_t, ld16(vrow + d0, ok && d0 < dlim));
    }
  }

  // ---- query sweep: (head, 32-row slice) pairs ----
  const int m_first = CAUSAL ? (n0 / kBwdBQ) : 0;
  const int m_count = (sq + kBwdBQ - 1) / kBwdBQ;
  const int ns = m_count > m_first ? m_count - m_first : 0;
  const int total = ns * nh;

  u32x4_t stq[QLOADS], sto[QLOADS];
  float st_ld = 0.f;
  auto issue = [&](int it) {
    const int hq = h_begin + it / ns;
    const int m = m_first + it % ns;
    const u16* Qp = (const u16*)p.q + q_off + (int64_t)hq * p.q_head;
    const u16* Dp = (const u16*)p.dout + do_off + (int64_t)hq * p.do_head;
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      const int panel = pid % NP;
      const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
      const int d0 = panel * 32 + (tid & 3) * 8;
      const int qrow = m * kBwdBQ + row;
      const bool ok = (pid < QPAIR) && qrow < sq && d0 < dlim;
      const int64_t qr = ok ? qrow : 0;
      stq[i] = ld16(Qp + qr * p.q_row + d0, ok);
      sto[i] = ld16(Dp + qr * p.do_row + d0, ok);
    }
    // lse / dsum: threads 0..31 -> lse[row], 32..63 -> dsum[row]
    if (tid < 64) {
      const int row = tid & 31;
      const int qrow = m * kBwdBQ + row;
      const int64_t bhi = (int64_t)bidb * s.h + hq;
      float v = 0.f;
      if (qrow < sq) v = (tid < 32) ? p.lse[bhi * s.lse_pitch + qrow] : p.dsum[bhi * p.seqlen_q_rounded + qrow];
      else v = (tid < 32) ? __builtin_huge_valf() : 0.f;
      st_ld = v;
    }
  };
  auto commit = [&](int buf) {
    char* qt = smem + KTILE + buf * SLICE;
    char* ot = qt + QTILE;
    float* lt = (float*)(qt + 2 * QTILE);
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      if (QPAIR % 32 == 0 || pid < QPAIR) {
        const int panel = pid % NP;
        const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
        const int off = panel_off(row, panel * 4 + (tid & 3), kBwdBQ);
        *(u32x4_t*)(qt + off) = stq[i];
        *(u32x4_t*)(ot + off) = sto[i];
      }
    }
    if (tid < 64) lt[tid] = st_ld;   // [0,32): lse, [32,64): dsum
  };

  f32x16_t dvt[NP], dkt[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) { dvt[t][g] = 0.f; dkt[t][g] = 0.f; }

  const float inv_scale = 1.f / s.scale;
  const float c = s.scale_log2;

  if (total > 0) issue(0);
  if (total > 0) commit(0);
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int hq = h_begin + it / ns;
    const int m = m_first + it % ns;
    const int q0 = m * kBwdBQ;
    const bool has_next = it + 1 < total;
    if (has_next) issue(it + 1);

    const char* qt = smem + KTILE + cur * SLICE;
    const char* ot = qt + QTILE;
    const float* lt = (const float*)(qt + 2 * QTILE);

    // S' = Q K^T - LSE/scale ; dP' = dO V^T - D    (query rows on registers, key on lane)
    f32x16_t sacc, pacc;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4_t lv = *(const f32x4_t*)(lt + 8 * u + 4 * hh);
      const f32x4_t dv = *(const f32x4_t*)(lt + 32 + 8 * u + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) { sacc[4 * u + j] = -lv[j] * inv_scale; pacc[4 * u + j] = -dv[j]; }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      sacc = E::mfma(row_read(qt, r, 2 * ks + hh, kBwdBQ), kf[ks], sacc);
      pacc = E::mfma(row_read(ot, r, 2 * ks + hh, kBwdBQ), vf[ks], pacc);
    }
    // P, dS
    const bool need_mask = (key >= sk) || (q0 + kBwdBQ > sq) || (CAUSAL && n0 + 32 * wave + 31 > q0);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      float pv = fast_exp2(sacc[g] * c);
      if (need_mask) {
        const int q = q0 + acc_row(g, hh);
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
      dvt[dt] = E::mfma(tr_frag(ot, 4 * hh, col0, kBwdBQ, i16), pf0, dvt[dt]);
      dvt[dt] = E::mfma(tr_frag(ot, 16 + 4 * hh, col0, kBwdBQ, i16), pf1, dvt[dt]);
      dkt[dt] = E::mfma(tr_frag(qt, 4 * hh, col0, kBwdBQ, i16), df0, dkt[dt]);
      dkt[dt] = E::mfma(tr_frag(qt, 16 + 4 * hh, col0, kBwdBQ, i16), df1, dkt[dt]);
    }
    // dS^T image [key][q] (8-byte stores of 4 consecutive q)
    {
      const int krow = 32 * wave + r;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        u32x2_t w;
        w[0] = E::pack2(pacc[4 * u + 0], pacc[4 * u + 1]);
        w[1] = E::pack2(pacc[4 * u + 2], pacc[4 * u + 3]);
        *(u32x2_t*)(ds_img + panel_off(krow, u, kBwdBN) + 8 * hh) = w;
      }
    }
    __syncthreads();
    // dQ[q][d] += dS[q][key] K[key][d]   (waves split the 32-wide d tiles)
    {
      const int64_t bhi = (int64_t)bidb * s.h + hq;
      float* dqa = p.dq_accum + (bhi * p.seqlen_q_rounded + q0) * p.d_rounded;
      for (int dt = wave; dt < NP; dt += kBwdWaves) {
        f32x16_t acc;
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
        for (int ks = 0; ks < kBwdBN / 16; ++ks) {
          const i16x8_t a = tr_frag(ds_img, 16 * ks + 4 * hh, 16 * (r >> 4), kBwdBN, i16);
          const i16x8_t bq = tr_frag(k_img, 16 * ks + 4 * hh, dt * 32 + 16 * (r >> 4), kBwdBN, i16);
          acc = E::mfma(a, bq, acc);
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int q = acc_row(g, hh);
          if (q0 + q < sq) atomicAdd(dqa + (int64_t)q * p.d_rounded + dt * 32 + r, acc[g]);
        }
      }
    }
    if (has_next) commit(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: dK = scale * dK^T^T, dV = dV^T^T ----
  if (key < sk) {
    const int hd = p.gqa_reduce ? kvh : hx;
    u16* dkrow = (u16*)p.dk + dk_off + (int64_t)hd * p.dk_head + (int64_t)key * p.dk_row;
    u16* dvrow = (u16*)p.dv + dv_off + (int64_t)hd * p.dv_head + (int64_t)key * p.dv_row;
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
// 3. dQ = scale * dq_accum  (8 elements per thread)
// ------------------------------------------------------------------------------------------------
template <bool BF16>
__global__ void __launch_bounds__(256) bwd_dq_kernel(const BwdParams p) {
  using E = Elt<BF16>;
  const AttnShape s = p.s;
  const int bh = blockIdx.x;
  const int bidb = bh / s.h, head = bh - bidb * s.h;
  int sq = s.seqlen_q;
  int64_t dq_off = (int64_t)bidb * p.dq_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) dq_off = (int64_t)c0 * p.dq_row;
  }
  const int cpr = s.d / 8;  // 8-element chunks per row
  const int idx = blockIdx.y * 256 + threadIdx.x;
  const int row = idx / cpr, ch = idx - row * cpr;
  if (row >= sq) return;
  const int64_t bhi = (int64_t)bidb * s.h + head;
  const float* src = p.dq_accum + (bhi * p.seqlen_q_rounded + row) * p.d_rounded + 8 * ch;
  const f32x4_t a = *(const f32x4_t*)src;
  const f32x4_t b = *(const f32x4_t*)(src + 4);
  const float sc = s.scale;
  u32x4_t w;
  w[0] = E::pack2(a[0] * sc, a[1] * sc);
  w[1] = E::pack2(a[2] * sc, a[3] * sc);
  w[2] = E::pack2(b[0] * sc, b[1] * sc);
  w[3] = E::pack2(b[2] * sc, b[3] * sc);
  u16* dst = (u16*)p.dq + dq_off + (int64_t)head * p.dq_head + (int64_t)row * p.dq_row + 8 * ch;
  *(u32x4_t*)dst = w;
}

// ------------------------------------------------------------------------------------------------
template <bool BF16, int D, bool CAUSAL>
static void run_bwd(const BwdParams& p, hipStream_t stream) {
  const int nheads_grid = p.gqa_reduce ? p.s.hk : p.s.h;
  dim3 grid(p.s.b * nheads_grid, p.num_n_blocks);
  prof_begin(kTimeBwdMain, stream);
  hipLaunchKernelGGL((bwd_main_kernel<BF16, D, CAUSAL>), grid, dim3(256), 0, stream, p);
  prof_end(kTimeBwdMain, stream);
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
  *block_m = kBwdBQ;
  *block_n = kBwdBN;
  (void)d;
}

template <bool BF16>
static void launch_bwd_t(const BwdParams& p, hipStream_t stream) {
  const int sq = p.s.seqlen_q;
  {
    dim3 grid(p.s.b * p.s.h, (sq + 15) / 16);
    prof_begin(kTimeBwdPre, stream);
    if (grid.y > 0) hipLaunchKernelGGL((bwd_pre_kernel<BF16>), grid, dim3(256), 0, stream, p);
    prof_end(kTimeBwdPre, stream);
  }
  if (p.s.causal) dispatch_bwd_d<BF16, true>(p, stream); else dispatch_bwd_d<BF16, false>(p, stream);
  {
    const int64_t chunks = (int64_t)sq * (p.s.d / 8);
    dim3 grid(p.s.b * p.s.h, (unsigned)((chunks + 255) / 256));
    prof_begin(kTimeBwdDq, stream);
    if (grid.y > 0) hipLaunchKernelGGL((bwd_dq_kernel<BF16>), grid, dim3(256), 0, stream, p);
    prof_end(kTimeBwdDq, stream);
  }
}

void launch_bwd(const BwdParams& p, bool is_bf16, hipStream_t stream) {
  if (p.s.b <= 0 || p.s.h <= 0 || p.s.seqlen_q <= 0) return;
  if (p.d_rounded % 32 != 0 || p.d_rounded < p.s.d) throw std::runtime_error("flash_attn_bwd: bad head_size_rounded");
  if (is_bf16) launch_bwd_t<true>(p, stream); else launch_bwd_t<false>(p, stream);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_bwd launch: ") + hipGetErrorString(e));
}

}  // namespace fa
