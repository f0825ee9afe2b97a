// Forward kernel, one wave per SIMD: 4 waves x 64 query rows (two 32-row q-blocks per wave), the
// whole 512-entry register file per wave.  OPT-IN (FLASH_ATTN_MI355X_FWD_W4=1) for the unmasked,
// dropout-free launches at head dims 64 and 128; fwd_kernel serves everything by default.
// Status: correct (the whole GPU suite passes with it enabled) but 13-20% slower than fwd_kernel on
// this compiler: the O accumulators (128) and Q fragments (64) must sit in AGPRs and the score tiles
// in VGPRs, and hipcc's allocator cannot be told so per MFMA.  Left to its heuristics it put the
// scores in AGPRs (one v_accvgpr_read per score) and spilled; with -mllvm -amdgpu-mfma-vgpr-form
// (Makefile) O moves to VGPRs instead and no register is left to prefetch K/V fragments, so every
// LDS read waits at lgkmcnt(0) before its two MFMAs.  Asm-managed accumulators are the next step.
//
// Why: with 8 waves x 32 rows every K fragment read from LDS feeds one MFMA and the two waves of a
// SIMD share its matrix pipe; at 64 rows per wave each K (b128) and V (tr) fragment feeds two MFMAs
// (q-block a and b), so LDS reads per MFMA halve, and the LDS-DMA pieces per MFMA too (one tile
// per 4 waves).  The one wave on a SIMD hides its own softmax VALU under its MFMAs: per K/V tile
// two 32-MFMA phases, each carrying the softmax of one q-block (~1 v_exp per MFMA gap):
//   phase X:  S(n+1, a), S(n+1, b) = K(n+1) Q^T   ||  P(n, b)   = exp2(c S(n, b) - c m_b)
//   phase Y:  O_a += V(n)^T P(n, a), O_b += ...   ||  P(n+1, a) = exp2(c S(n+1, a) - c m_a)
// Each q-block keeps its own running max / sum, the max-free fast path with the 2^8 guard and the
// refit slow path of fwd_kernel; S(n, b) and P(n, a) are carried across the step (the loop is
// unrolled by two with the carried sets swapping names: no register copies).
// Algorithm reference: compute_attn_1rowblock, flash_fwd_kernel.h:121-583.

#include <cstdlib>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

template <bool BF16, int D, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) fwd_kernel_w4(const FwdParams p) {
  using E = Elt<BF16>;
  constexpr int NW = 4;
  constexpr int BM = 256;
  constexpr int BN = 64;
  constexpr int KS = D / 16;
  constexpr int NT = BN / 32;            // 32-key subtiles per tile
  constexpr int NP = D / 32;             // 32-wide d panels of O
  constexpr int TILE = BN * D * 2;
  constexpr int PIECES = TILE / 1024;
  constexpr int PPW = PIECES / NW;
  constexpr int NB = 4;                  // K ring and V ring depth
  static_assert(PIECES % NW == 0, "whole DMA pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[2 * NB * TILE];
  auto kslot = [&](int pos) { return (pos % NB) * TILE; };
  auto vslot = [&](int pos) { return NB * TILE + (pos % NB) * TILE; };

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const LdsBases lb(lane);

  int bh, m_idx;
  xcd_order_grouped(blockIdx.x, s.b * s.h, p.num_m_blocks, p.head_group, bh, m_idx);
  const int bidb = bh / s.h;
  const int head = bh - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int m_block = p.num_m_blocks - 1 - m_idx;

  int sq = s.seqlen_q, sk = s.seqlen_k;
  int64_t q_off = (int64_t)bidb * p.q_batch, o_off = (int64_t)bidb * p.o_batch;
  int64_t k_off = (int64_t)bidb * p.k_batch, v_off = (int64_t)bidb * p.v_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) { q_off = (int64_t)c0 * p.q_row; o_off = (int64_t)c0 * p.o_row; }
  }
  if (s.cu_seqlens_k) {
    const int c0 = s.cu_seqlens_k[bidb];
    sk = s.cu_seqlens_k[bidb + 1] - c0;
    if (!s.varlen_padded_input) { k_off = (int64_t)c0 * p.k_row; v_off = (int64_t)c0 * p.v_row; }
  }
  if (p.rng_state != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
    p.rng_state[0] = p.seed;
    p.rng_state[1] = p.offset;
  }
  const int m0 = m_block * BM;
  if (m0 >= sq) return;

  typedef unsigned short u16;
  const u16* __restrict__ Q = (const u16*)p.q + q_off + (int64_t)head * p.q_head;
  const u16* __restrict__ K = (const u16*)p.k + k_off + (int64_t)kvh * p.k_head;
  const u16* __restrict__ V = (const u16*)p.v + v_off + (int64_t)kvh * p.v_head;
  u16* __restrict__ O = (u16*)p.o + o_off + (int64_t)head * p.o_head;
  float* __restrict__ LSE = p.lse + ((int64_t)bidb * s.h + head) * s.lse_pitch;

  const int wq0 = m0 + 64 * wave;       // first query row of this wave (q-block a; b = +32)
  const int dlim = s.d;

  // ---- Q fragments of both q-blocks (B operands of S^T = K Q^T) ----
  i16x8_t qf[2][KS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = wq0 + 32 * j + r;
    const bool ok = qi < sq;
    const u16* qrow = Q + (int64_t)(ok ? qi : 0) * p.q_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      qf[j][ks] = __builtin_bit_cast(i16x8_t, ld16(qrow + d0, ok && d0 < dlim));
#ifndef FA_W4_QF_VGPR
      // Q fragments live in the accumulator file (MFMA reads A/B from AGPRs): the VGPRs stay for
      // the score tiles the softmax reads
      asm volatile("" : "+a"(qf[j][ks]));
#endif
    }
  }

  const int n_end = CAUSAL ? min(sk, m0 + BM) : sk;
  const int nblk = n_end > 0 ? (n_end + BN - 1) / BN : 0;
  const int nfast = min(nblk, (CAUSAL ? min(sk, m0 + 1) : sk) / BN);

  // ---- LDS-DMA of K/V tiles (panel layout, see fa_fwd.hip) ----
  // Piece j of this wave is pc = wave + 4 j: rows 16 wave .. +15 of d-panel j, so every piece of a
  // tile shares one per-lane byte offset plus 64 j (s.d == D here: no padded columns).  Only that
  // base is kept live; a per-piece offset array held across the loop was spilled, and its scratch
  // reload (vmcnt(0)) serialised the DMA.
  const int drow = wave * 16 + (lane >> 2);
  const int dcol = ((lane & 3) ^ ((drow >> 2) & 3)) << 3;
  const int vbase_k = (int)(((int64_t)drow * p.k_row + dcol) * 2);
  const int vbase_v = (int)(((int64_t)drow * p.v_row + dcol) * 2);
  auto issue = [&](int nb) {
    const int n0 = nb * BN;
    char* kdst = smem + kslot(nb) + wave * 1024;
    char* vdst = smem + vslot(nb) + wave * 1024;
    const int64_t kb = (int64_t)(sk - n0) * p.k_row * 2, vb = (int64_t)(sk - n0) * p.v_row * 2;
    const buf_rsrc_t rk = make_rsrc(K + (int64_t)n0 * p.k_row, (int)(kb > 0x7fffffff ? 0x7fffffff : kb));
    const buf_rsrc_t rv = make_rsrc(V + (int64_t)n0 * p.v_row, (int)(vb > 0x7fffffff ? 0x7fffffff : vb));
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      dma16(rk, kdst + j * NW * 1024, vbase_k + 64 * j);
      dma16(rv, vdst + j * NW * 1024, vbase_v + 64 * j);
    }
  };
  constexpr int NDMA = 2 * PPW;   // DMA operations one issue() leaves outstanding in this wave
  auto tile_sync = [&](bool ahead) { wait_dma_keep_and_barrier(ahead ? NDMA : 0); };

  // ---- MFMA building blocks ----
  constexpr int KG = (KS % 4 == 0) ? 4 : 2;
  // S^T of both q-blocks for the K tile at kt_off: each K fragment feeds two MFMAs
  auto qk2 = [&](int kt_off, f32x16_t (&sa)[NT], f32x16_t (&sb)[NT]) {
    const TileAddr ta(lb, kt_off);
    static_for<0, NT>([&](auto T) {
      constexpr int t = decltype(T)::value;
#pragma unroll
      for (int g = 0; g < 16; ++g) { sa[t][g] = 0.f; sb[t][g] = 0.f; }
      static_for<0, KS / KG>([&](auto GG) {
        constexpr int g0 = decltype(GG)::value * KG;
        i16x8_t ka[KG];
        static_for<0, KG>([&](auto KK) {
          constexpr int ks = g0 + decltype(KK)::value;
          ka[ks - g0] = row_read_c<BN, t * 32, 2 * ks>(smem, ta);
        });
#pragma unroll
        for (int k = 0; k < KG; ++k) {
          sa[t] = E::mfma(ka[k], qf[0][g0 + k], sa[t]);
          sb[t] = E::mfma(ka[k], qf[1][g0 + k], sb[t]);
        }
      });
    });
  };
  // S^T of one q-block (refit, general path)
  auto qk1 = [&](int kt_off, int j, f32x16_t (&st)[NT]) {
    const TileAddr ta(lb, kt_off);
    static_for<0, NT>([&](auto T) {
      constexpr int t = decltype(T)::value;
#pragma unroll
      for (int g = 0; g < 16; ++g) st[t][g] = 0.f;
      static_for<0, KS / KG>([&](auto GG) {
        constexpr int g0 = decltype(GG)::value * KG;
        i16x8_t ka[KG];
        static_for<0, KG>([&](auto KK) {
          constexpr int ks = g0 + decltype(KK)::value;
          ka[ks - g0] = row_read_c<BN, t * 32, 2 * ks>(smem, ta);
        });
#pragma unroll
        for (int k = 0; k < KG; ++k) st[t] = E::mfma(ka[k], j ? qf[1][g0 + k] : qf[0][g0 + k], st[t]);
      });
    });
  };

  float m_run[2] = {kNegInf, kNegInf}, l_run[2] = {0.f, 0.f};
  f32x16_t o[2][NP];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NP; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) o[j][t][g] = 0.f;
  const float c = s.scale_log2;

  // O^T of both q-blocks += V^T P^T: each V fragment feeds two MFMAs
  auto pv2 = [&](int vt_off, const i16x8_t (&pa)[2 * NT], const i16x8_t (&pb)[2 * NT]) {
    const TileAddr ta(lb, vt_off);
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      i16x8_t a[2 * NT];
      static_for<0, 2 * NT>([&](auto KC) {
        constexpr int kk = decltype(KC)::value;
        a[kk] = tr_frag_c<BN, kk * 16, dt>(smem, ta);
      });
#pragma unroll
      for (int kk = 0; kk < 2 * NT; ++kk) {
        o[0][dt] = E::mfma(a[kk], pa[kk], o[0][dt]);
        o[1][dt] = E::mfma(a[kk], pb[kk], o[1][dt]);
      }
    });
  };
  auto pv1 = [&](int vt_off, int j, const i16x8_t (&pf)[2 * NT]) {
    const TileAddr ta(lb, vt_off);
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      i16x8_t a[2 * NT];
      static_for<0, 2 * NT>([&](auto KC) {
        constexpr int kk = decltype(KC)::value;
        a[kk] = tr_frag_c<BN, kk * 16, dt>(smem, ta);
      });
#pragma unroll
      for (int kk = 0; kk < 2 * NT; ++kk) {
        if (j) o[1][dt] = E::mfma(a[kk], pf[kk], o[1][dt]);
        else o[0][dt] = E::mfma(a[kk], pf[kk], o[0][dt]);
      }
    });
  };

  auto rowmax = [&](const f32x16_t (&st)[NT]) {
    float mx[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) mx[g & 3] = fmaxf(mx[g & 3], st[t][g]);
    return half_swap_max(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
  };
  auto scale_o = [&](int j, float alpha) {
#pragma unroll
    for (int t = 0; t < NP; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        if (j) o[1][t][g] *= alpha;
        else o[0][t][g] *= alpha;
      }
  };
  // deferred-max rescale of q-block j for a tile whose row max is mt (fwd_kernel rescale)
  auto rescale = [&](int j, float mt) {
    const float mr = m_run[j];
    const float m_new = fmaxf(mr, mt);
    if (__any(mr == kNegInf ? m_new != mr : (mt - mr) * c > kFwdRescaleThr)) {
      const float alpha = fast_exp2(mr * c - ((m_new == kNegInf) ? 0.f : m_new * c));
      l_run[j] *= alpha;
      scale_o(j, alpha);
      m_run[j] = m_new;
    }
  };
  // P of q-block j against its running max (general path: the sum goes to l_run)
  auto softmax_pack = [&](int j, f32x16_t (&st)[NT], i16x8_t (&pf)[2 * NT]) {
    const float ms = (m_run[j] == kNegInf) ? 0.f : m_run[j] * c;
    float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float pv = fast_exp2(fmaf(st[t][g], c, -ms));
        ls[g & 3] += pv;
        st[t][g] = pv;
      }
      pf[2 * t] = pack_frag<BF16>(st[t], 0);
      pf[2 * t + 1] = pack_frag<BF16>(st[t], 1);
    }
    l_run[j] += (ls[0] + ls[1]) + (ls[2] + ls[3]);
  };
  // fast path: no max pass, partial sum returned for the guard
  auto softmax_fast = [&](int j, const f32x16_t (&st)[NT], i16x8_t (&pf)[2 * NT]) {
    const float ms = m_run[j] * c;
    float ls[4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x16_t pt;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        pt[g] = fast_exp2(fmaf(st[t][g], c, -ms));
        ls[g & 3] = (t == 0 && g < 4) ? pt[g] : ls[g & 3] + pt[g];
      }
      pf[2 * t] = pack_frag<BF16>(pt, 0);
      pf[2 * t + 1] = pack_frag<BF16>(pt, 1);
    }
    return (ls[0] + ls[1]) + (ls[2] + ls[3]);
  };
  auto guard_ok = [&](float ls) { return !__any(!(ls <= kFwdSumThr)); };
  // slow path: recompute S of q-block j from the resident K tile at kt_off, move the running max to
  // the true max, rescale, redo P (wave-uniform, rare)
  auto refit = [&](int kt_off, int j, i16x8_t (&pf)[2 * NT]) {
    asm volatile("; refit" ::: "memory");
    f32x16_t st[NT];
    qk1(kt_off, j, st);
    const float mt = rowmax(st);
    const float m_new = fmaxf(m_run[j], mt);
    const float alpha = fast_exp2((m_run[j] - m_new) * c);
    l_run[j] *= alpha;
    scale_o(j, alpha);
    m_run[j] = m_new;
    return softmax_fast(j, st, pf);
  };

  // tiles 0, 1, 2 in flight before the loop
  if (nblk > 0) issue(0);
  if (nblk > 1) issue(1);
  wait_vmem_all();   // Q fragments and tiles 0, 1 (compiler-visible)
  if (nblk > 2) issue(2);
  lds_barrier();

  if (nfast > 0) {
    // prologue: S(0, a), S(0, b); explicit max of the first tile; P(0, a)
    f32x16_t s1A[NT], s1B[NT];   // carried S(n, b)
    i16x8_t p0A[2 * NT], p0B[2 * NT];   // carried P(n, a)
    {
      f32x16_t s0[NT];
      qk2(kslot(0), s0, s1A);
      rescale(0, rowmax(s0));
      rescale(1, rowmax(s1A));
      softmax_pack(0, s0, p0A);
    }
    // one K/V step; s1c = S(nb, b), p0c = P(nb, a) in; s1n = S(nb+1, b), p0n = P(nb+1, a) out
    auto body = [&](int nb, const f32x16_t (&s1c)[NT], f32x16_t (&s1n)[NT], const i16x8_t (&p0c)[2 * NT],
                    i16x8_t (&p0n)[2 * NT]) {
      if (nb + 3 < nblk) issue(nb + 3);
      f32x16_t s0n[NT];
      i16x8_t p1[2 * NT];
      // phase X: P(nb, b) || S(nb+1, a), S(nb+1, b)
      float ls1 = softmax_fast(1, s1c, p1);
      qk2(kslot(nb + 1), s0n, s1n);
      if (!guard_ok(ls1)) ls1 = refit(kslot(nb), 1, p1);
      l_run[1] += ls1;
      // phase Y: P(nb+1, a) || O += V(nb)^T P(nb)
      float ls0 = softmax_fast(0, s0n, p0n);
      pv2(vslot(nb), p0c, p1);
      if (!guard_ok(ls0)) ls0 = refit(kslot(nb + 1), 0, p0n);
      l_run[0] += ls0;
      tile_sync(nb + 3 < nblk);
    };
    // the last fast tile: no S / P of the next tile (it belongs to the general path, or is past the end)
    auto body_last = [&](int nb, const f32x16_t (&s1c)[NT], const i16x8_t (&p0c)[2 * NT]) {
      if (nb + 3 < nblk) issue(nb + 3);
      i16x8_t p1[2 * NT];
      float ls1 = softmax_fast(1, s1c, p1);
      if (!guard_ok(ls1)) ls1 = refit(kslot(nb), 1, p1);
      l_run[1] += ls1;
      pv2(vslot(nb), p0c, p1);
      tile_sync(nb + 3 < nblk);
    };
    int nb = 0;
    for (; nb + 2 < nfast; nb += 2) {
      body(nb, s1A, s1B, p0A, p0B);
      body(nb + 1, s1B, s1A, p0B, p0A);
    }
    if (nb + 1 < nfast) {
      body(nb, s1A, s1B, p0A, p0B);
      body_last(nb + 1, s1B, p0B);
    } else {
      body_last(nb, s1A, p0A);
    }
  }

  // ---- general path: causal diagonal / ragged tiles, per q-block ----
  for (int nb = nfast; nb < nblk; ++nb) {
    const int n0 = nb * BN;
    if (nb + 3 < nblk) issue(nb + 3);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int qb0 = wq0 + 32 * j;
      const int qi = qb0 + r;
      if ((qb0 < sq) && (!CAUSAL || n0 <= qb0 + 31)) {
        f32x16_t st[NT];
        qk1(kslot(nb), j, st);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int key = n0 + t * 32 + acc_row(g, hh);
            if ((key >= sk) | (CAUSAL && key > qi)) st[t][g] = kNegInf;
          }
        rescale(j, rowmax(st));
        i16x8_t pf[2 * NT];
        softmax_pack(j, st, pf);
        pv1(vslot(nb), j, pf);
      }
    }
    tile_sync(nb + 3 < nblk);
  }

  // ---- epilogue (fwd_kernel's, per q-block) ----
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = wq0 + 32 * j + r;
    const float l_tot = half_swap_sum(l_run[j]);
    const bool bad = (l_tot == 0.f) || (l_tot != l_tot);
    const float inv = bad ? 1.f : fast_rcp(l_tot);
    const float lse = bad ? __builtin_huge_valf() : m_run[j] * s.scale + __logf(l_tot);
    u16* orow = O + (int64_t)(qi < sq ? qi : 0) * p.o_row;
#pragma unroll
    for (int dt = 0; dt < NP; ++dt)
#pragma unroll
      for (int u = 0; u < 4; u += 2) {
        const f32x16_t& oj = j ? o[1][dt] : o[0][dt];
        unsigned a0 = E::pack2(oj[4 * u + 0] * inv, oj[4 * u + 1] * inv);
        unsigned a1 = E::pack2(oj[4 * u + 2] * inv, oj[4 * u + 3] * inv);
        unsigned b0 = E::pack2(oj[4 * u + 4] * inv, oj[4 * u + 5] * inv);
        unsigned b1 = E::pack2(oj[4 * u + 6] * inv, oj[4 * u + 7] * inv);
        auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        const int col = dt * 32 + 8 * u + 8 * hh;
        if (qi < sq && col < dlim) {
          u32x4_t w = {(unsigned)r0[0], (unsigned)r1[0], (unsigned)r0[1], (unsigned)r1[1]};
          *(u32x4_t*)(orow + col) = w;
        }
      }
    if (qi < sq && hh == 0) LSE[qi] = lse;
  }
}

// Launches fwd_kernel_w4 when it is enabled (FLASH_ATTN_MI355X_FWD_W4=1, read per launch) and covers
// the call (d == 64 or 128, no dropout / mask / split-KV, 256-row blocks); false leaves the launch
// to fwd_kernel.  Opt-in: measured 13-20% slower than fwd_kernel at C3 / C5 ("Tried").
bool launch_fwd_w4(const FwdParams& p, bool is_bf16, hipStream_t stream) {
  const char* e = std::getenv("FLASH_ATTN_MI355X_FWD_W4");
  if (e == nullptr || e[0] != '1') return false;
  const AttnShape& s = p.s;
  if (s.dropout || s.mask != nullptr || s.fm_lts != nullptr || p.n_split != 0 || p.p_out != nullptr) return false;
  if (s.d != 64 && s.d != 128) return false;
  const dim3 grid(s.b * s.h * p.num_m_blocks), block(256);
#define FA_W4_LAUNCH(BF, DD, CA) hipLaunchKernelGGL((fwd_kernel_w4<BF, DD, CA>), grid, block, 0, stream, p)
  if (is_bf16) {
    if (s.d == 64) { if (s.causal) FA_W4_LAUNCH(true, 64, true); else FA_W4_LAUNCH(true, 64, false); }
    else { if (s.causal) FA_W4_LAUNCH(true, 128, true); else FA_W4_LAUNCH(true, 128, false); }
  } else {
    if (s.d == 64) { if (s.causal) FA_W4_LAUNCH(false, 64, true); else FA_W4_LAUNCH(false, 64, false); }
    else { if (s.causal) FA_W4_LAUNCH(false, 128, true); else FA_W4_LAUNCH(false, 128, false); }
  }
#undef FA_W4_LAUNCH
  return true;
}

}  // namespace fa
