// FlashAttention-2 forward for MI355X (gfx950): O = softmax(scale * Q K^T [+ causal mask]) V, LSE.
//
// Algorithm (the reference's compute_attn_1rowblock, csrc/flash_attn/src/flash_fwd_kernel.h:121-583):
// one workgroup per (query block, batch, head); K/V tiles streamed through LDS; online softmax with
// running max / sum; epilogue O /= l, LSE = max * scale + ln(l) (+inf when l == 0 or NaN,
// flash_fwd_kernel.h:509-518); causal mask is top-left aligned (key <= query, softmax.h:143-178).
//
// MI355X mapping (not a translation of the CUDA tiling):
//   * 4 waves x 32 query rows = 128-row query block; BN = 64 keys per K/V tile.
//   * "Swapped" QK^T: each wave computes S^T = K . Q^T with v_mfma_f32_32x32x16, so the query sits on
//     the MFMA column (= lane) and every lane holds 32 scores of ONE query row: the row max / sum are
//     in-lane reductions plus one v_permlane32_swap, with no LDS and no shuffles.
//   * O^T = V^T . P^T: the S^T accumulator, converted to bf16/f16 in registers, is directly the B
//     operand of the PV MFMA (no LDS round trip for P); V^T fragments come from the row-major V tile
//     through ds_read_b64_tr_b16.  O^T keeps the query on the lane, so the online-softmax rescale is
//     a per-lane scalar multiply.
//   * Q lives in registers for the whole K/V sweep.  K and V are register-staged: the global loads of
//     tile n+1 are issued before the MFMAs of tile n and written (XOR-swizzled panel layout, see
//     fa_common.h) into the other LDS buffer afterwards: one barrier per tile.
//   * Heaviest causal query blocks are dispatched first (blockIdx.y reversed) to shorten the tail.
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

constexpr int kFwdWaves = 4;
constexpr int kFwdBM = 32 * kFwdWaves;

template <int D> struct FwdTile { static constexpr int BN = 64; };

template <bool BF16, int D, bool CAUSAL>
__global__ void __launch_bounds__(256, 2) fwd_kernel(const FwdParams p) {
  using E = Elt<BF16>;
  constexpr int BN = FwdTile<D>::BN;
  constexpr int KS = D / 16;            // QK^T k-steps (16 along d)
  constexpr int NT = BN / 32;           // 32-key subtiles per K/V tile
  constexpr int NP = D / 32;            // 32-wide d panels == PV output tiles
  constexpr int TILE = BN * D * 2;      // bytes of one K or V tile
  constexpr int NPAIR = BN * NP / 2;    // (2 rows x 64 B) staging units per tile
  constexpr int LOADS = (NPAIR + 31) / 32;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buffer][K | V]

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, i16 = lane & 15;

  const int bh = blockIdx.x;
  const int bidb = bh / s.h;
  const int head = bh - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int m_block = p.num_m_blocks - 1 - (int)blockIdx.y;

  // ---- sequence geometry (reference BlockInfo, block_info.h:14-31) ----
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
  if (p.rng_state != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    p.rng_state[0] = p.seed;
    p.rng_state[1] = p.offset;
  }
  const int m0 = m_block * kFwdBM;
  if (m0 >= sq) return;

  typedef unsigned short u16;
  const u16* __restrict__ Q = (const u16*)p.q + q_off + (int64_t)head * p.q_head;
  const u16* __restrict__ K = (const u16*)p.k + k_off + (int64_t)kvh * p.k_head;
  const u16* __restrict__ V = (const u16*)p.v + v_off + (int64_t)kvh * p.v_head;
  u16* __restrict__ O = (u16*)p.o + o_off + (int64_t)head * p.o_head;
  float* __restrict__ LSE = p.lse + ((int64_t)bidb * s.h + head) * s.lse_pitch;

  const int wq0 = m0 + 32 * wave;   // first query row of this wave
  const int qi = wq0 + r;           // this lane's query row
  const int dlim = s.d;

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[qi][16ks + 8hh .. +7] ----
  i16x8_t qf[KS];
  {
    const bool ok = qi < sq;
    const u16* qrow = Q + (int64_t)(ok ? qi : 0) * p.q_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      qf[ks] = __builtin_bit_cast(i16x8_t, ld16(qrow + d0, ok && d0 < dlim));
    }
  }

  const int n_end = CAUSAL ? min(sk, m0 + kFwdBM) : sk;
  const int nblk = n_end > 0 ? (n_end + BN - 1) / BN : 0;

  // ---- register staging of K/V tiles ----
  u32x4_t stk[LOADS], stv[LOADS];
  auto issue = [&](int n0) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int pid = i * 32 + (tid >> 3);
      const int panel = pid % NP;
      const int row = 2 * (pid / NP) + ((tid >> 2) & 1);
      const int d0 = panel * 32 + (tid & 3) * 8;
      const int key = n0 + row;
      const bool ok = (pid < NPAIR) && key < sk && d0 < dlim;
      const int64_t kr = ok ? key : 0;
      stk[i] = ld16(K + kr * p.k_row + d0, ok);
      stv[i] = ld16(V + kr * p.v_row + d0, ok);
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

  float m_run = kNegInf, l_run = 0.f;
  f32x16_t o[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) o[t][g] = 0.f;
  const float c = s.scale_log2;

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
      // S^T[key][query] for NT subtiles of 32 keys
      f32x16_t st[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int g = 0; g < 16; ++g) st[t][g] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          st[t] = E::mfma(row_read(kt, t * 32 + r, 2 * ks + hh, BN), qf[ks], st[t]);
      }
      const bool need_mask = (n0 + BN > sk) || (CAUSAL && n0 + BN - 1 > wq0);
      if (need_mask) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int key = n0 + t * 32 + acc_row(g, hh);
            if (key >= sk || (CAUSAL && key > qi)) st[t][g] = kNegInf;
          }
      }
      float mt = kNegInf;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) mt = fmaxf(mt, st[t][g]);
      mt = half_swap_max(mt);
      const float m_new = fmaxf(m_run, mt);
      const float ms = (m_new == kNegInf) ? 0.f : m_new * c;
      const float alpha = fast_exp2(m_run * c - ms);
      float ls = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float pv = fast_exp2(fmaf(st[t][g], c, -ms));
          st[t][g] = pv;
          ls += pv;
        }
      l_run = l_run * alpha + ls;
      m_run = m_new;
#pragma unroll
      for (int t = 0; t < NP; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) o[t][g] *= alpha;

      i16x8_t pf[2 * NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        pf[2 * t] = pack_frag<BF16>(st[t], 0);
        pf[2 * t + 1] = pack_frag<BF16>(st[t], 1);
      }
      // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
      for (int dt = 0; dt < NP; ++dt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const i16x8_t a = tr_frag(vt, t * 32 + 16 * s2 + 4 * hh, dt * 32 + 16 * (r >> 4), BN, i16);
            o[dt] = E::mfma(a, pf[2 * t + s2], o[dt]);
          }
    }
    if (has_next) commit(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const float l_tot = half_swap_sum(l_run);
  const bool bad = (l_tot == 0.f) || (l_tot != l_tot);
  const float inv = bad ? 1.f : 1.f / l_tot;
  const float lse = bad ? __builtin_huge_valf() : m_run * s.scale + __logf(l_tot);
  if (qi < sq) {
    u16* orow = O + (int64_t)qi * p.o_row;
#pragma unroll
    for (int dt = 0; dt < NP; ++dt)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int d0 = dt * 32 + 8 * u + 4 * hh;
        if (d0 < dlim) {
          u32x2_t w;
          w[0] = E::pack2(o[dt][4 * u + 0] * inv, o[dt][4 * u + 1] * inv);
          w[1] = E::pack2(o[dt][4 * u + 2] * inv, o[dt][4 * u + 3] * inv);
          *(u32x2_t*)(orow + d0) = w;
        }
      }
    if (hh == 0) LSE[qi] = lse;
  }
}

template <bool BF16, int D, bool CAUSAL>
static void run_fwd(const FwdParams& p, hipStream_t stream) {
  dim3 grid(p.s.b * p.s.h, p.num_m_blocks);
  prof_begin(kTimeFwd, stream);
  hipLaunchKernelGGL((fwd_kernel<BF16, D, CAUSAL>), grid, dim3(256), 0, stream, p);
  prof_end(kTimeFwd, stream);
}

template <bool BF16, bool CAUSAL>
static void dispatch_d(const FwdParams& p, hipStream_t stream) {
  const int d = p.s.d;
  if (d <= 32) run_fwd<BF16, 32, CAUSAL>(p, stream);
  else if (d <= 64) run_fwd<BF16, 64, CAUSAL>(p, stream);
  else if (d <= 96) run_fwd<BF16, 96, CAUSAL>(p, stream);
  else if (d <= 128) run_fwd<BF16, 128, CAUSAL>(p, stream);
  else throw std::runtime_error("flash_attn_fwd: head dim " + std::to_string(d) + " > 128 not built yet");
}

void fwd_block_size(int d, int* block_m, int* block_n) {
  *block_m = kFwdBM;
  *block_n = 64;
  (void)d;
}

void launch_fwd(const FwdParams& p, bool is_bf16, hipStream_t stream) {
  if (p.s.b <= 0 || p.s.h <= 0) return;
  if (p.num_m_blocks <= 0) return;
  if (p.num_m_blocks > 65535) throw std::runtime_error("flash_attn_fwd: seqlen_q too large for grid.y");
  if (is_bf16) {
    if (p.s.causal) dispatch_d<true, true>(p, stream); else dispatch_d<true, false>(p, stream);
  } else {
    if (p.s.causal) dispatch_d<false, true>(p, stream); else dispatch_d<false, false>(p, stream);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_fwd launch: ") + hipGetErrorString(e));
}

}  // namespace fa
