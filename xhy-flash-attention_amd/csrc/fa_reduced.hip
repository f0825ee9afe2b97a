// calc_reduced_attn_scores for MI355X (gfx950): column sums of the attention probabilities.
//
// Reference: csrc/flash_attn/src/calc_reduced_attn_scores_kernel.h:119-307 (C ABI
// csrc/capi/flash_attn.cu:1107-1201).  For every (batch, head, key k):
//     reduced_scores[b][h][k] = sum_q exp(scale * q . k - LSE[b][h][q])
// over all queries (non-causal, no mask, no dropout), with LSE the forward's softmax_lse; optionally
// the probabilities themselves, softmax_ptr[b][h][q][k] (fp32, seqlen_q x seqlen_k).  The reference
// adds each CTA's partial column sums into reduced_scores with atomicAdd (so it expects a zeroed
// buffer); here one workgroup owns a 128-key column block over ALL queries and stores its sums, which
// is the same result with no atomics and no zeroing requirement.
//
// MI355X mapping: 4 waves x 32 keys.  "Key on the lane": S = Q K^T with v_mfma_f32_32x32x16 where
// the B operand is this wave's K fragments held in registers for the whole sweep and the A operand is
// the 32-row Q tile read straight from global memory (16 B per lane; the four waves share it through
// L1/L2), so the accumulator column is the lane's key and its 16 elements are 16 query rows: the
// column sum is a per-lane add chain plus one v_permlane32_swap at the end.  No LDS, no barriers.
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

template <bool BF16, int D>
__global__ void __launch_bounds__(256) reduced_scores_kernel(const ReducedParams p) {
  using E = Elt<BF16>;
  typedef unsigned short u16;
  constexpr int KS = D / 16;
  const int lane = threadIdx.x & 63, wave = wave_uniform(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int bh = blockIdx.x;
  const int bidb = bh / p.h, head = bh - bidb * p.h;
  const int kvh = head / (p.h / p.hk);
  const int key = blockIdx.y * 128 + wave * 32 + r;
  const bool key_ok = key < p.sk;

  const u16* Q = (const u16*)p.q + (int64_t)bidb * p.q_batch + (int64_t)head * p.q_head;
  const u16* K = (const u16*)p.k + (int64_t)bidb * p.k_batch + (int64_t)kvh * p.k_head;
  const float* LSE = p.lse + (int64_t)bh * p.sq;

  i16x8_t kf[KS];   // B operand: lane holds K[key][16 ks + 8 hh .. +7]
  {
    const u16* krow = K + (int64_t)(key_ok ? key : 0) * p.k_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      kf[ks] = __builtin_bit_cast(i16x8_t, ld16(krow + d0, key_ok && d0 < p.d));
    }
  }
  const float c = p.scale * kLog2e;
  float colsum = 0.f;
  for (int q0 = 0; q0 < p.sq; q0 += 32) {
    // A operand: lane holds Q[q0 + r][16 ks + 8 hh .. +7]
    const int qa = q0 + r;
    const u16* qrow = Q + (int64_t)(qa < p.sq ? qa : 0) * p.q_row;
    f32x16_t s;
#pragma unroll
    for (int g = 0; g < 16; ++g) s[g] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      const i16x8_t qf = __builtin_bit_cast(i16x8_t, ld16(qrow + d0, qa < p.sq && d0 < p.d));
      s = E::mfma(qf, kf[ks], s);
    }
    // element g: query q0 + acc_row(g, hh), key = this lane's key
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qb = q0 + 8 * u + 4 * hh;
      float pv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qq = qb + j;
        // rows past seqlen_q count as LSE = +inf (reference calc_reduced_attn_scores_kernel.h:237)
        const float lse = qq < p.sq ? LSE[qq] : __builtin_huge_valf();
        pv[j] = fast_exp2(s[4 * u + j] * c - lse * kLog2e);
        colsum += pv[j];
      }
      if (p.p_out != nullptr && key_ok) {
        float* prow = p.p_out + ((int64_t)bh * p.sq + qb) * p.sk + key;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (qb + j < p.sq) prow[(int64_t)j * p.sk] = pv[j];
      }
    }
  }
  colsum = half_swap_sum(colsum);
  if (key_ok && hh == 0) p.reduced[(int64_t)bh * p.sk + key] = colsum;
}

template <bool BF16>
static void dispatch_reduced(const ReducedParams& p, hipStream_t stream) {
  dim3 grid(p.b * p.h, (p.sk + 127) / 128);
  const int d = p.d;
  if (d <= 32) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 32>), grid, dim3(256), 0, stream, p);
  else if (d <= 64) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 64>), grid, dim3(256), 0, stream, p);
  else if (d <= 96) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 96>), grid, dim3(256), 0, stream, p);
  else if (d <= 128) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 128>), grid, dim3(256), 0, stream, p);
  else if (d <= 160) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 160>), grid, dim3(256), 0, stream, p);
  else if (d <= 192) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 192>), grid, dim3(256), 0, stream, p);
  else if (d <= 224) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 224>), grid, dim3(256), 0, stream, p);
  else if (d <= 256) hipLaunchKernelGGL((reduced_scores_kernel<BF16, 256>), grid, dim3(256), 0, stream, p);
  else throw std::runtime_error("calc_reduced_attn_scores: head dim " + std::to_string(d) + " > 256");
}

void launch_reduced_scores(const ReducedParams& p, bool is_bf16, hipStream_t stream) {
  if (p.b <= 0 || p.h <= 0 || p.sk <= 0) return;
  if ((p.sk + 127) / 128 > 65535) throw std::runtime_error("calc_reduced_attn_scores: seqlen_k too large for grid.y");
  if (is_bf16) dispatch_reduced<true>(p, stream); else dispatch_reduced<false>(p, stream);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("calc_reduced_attn_scores launch: ") + hipGetErrorString(e));
}

}  // namespace fa
