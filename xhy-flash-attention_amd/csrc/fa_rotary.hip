// Rotary position embedding for MI355X (gfx950): the caller-side op of the attention modules
// (MHA rotary).
//
// Reference: csrc/rotary/rotary.cpp:16-37 + rotary_cuda.cu:9-45 (`rotary_emb.apply_rotary`), driven
// by flash_attn/layers/rotary.py:35-196.  For each (batch, row, head) and pair i < rotary_dim / 2:
//     x1 = x[i], x2 = x[i + rotary_dim / 2]          (GPT-NeoX halves)   or
//     x1 = x[2 i], x2 = x[2 i + 1]                   (interleaved, GPT-J pairs)
//     out1 = x1 cos - x2 sin,  out2 = x1 sin + x2 cos   (conj: sin -> -sin, the backward)
// with cos / sin[row][i] in the input dtype, arithmetic in fp32 and one rounding per output, as the
// reference's elementwise kernel does.  Columns past rotary_dim are not touched (the Python layer
// copies them for out-of-place calls, as the reference does).  out may alias x.
//
// HBM-bound elementwise work (2 x 2 bytes read and written per pair plus the cos/sin row, which
// stays in L2): one thread per pair, consecutive threads on consecutive pairs of a row, so both
// halves (or the interleaved pairs) are read and written coalesced.
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_params.h"

namespace fa {

template <bool BF16, bool INTERLEAVED, bool CONJ>
__global__ void __launch_bounds__(256) rotary_kernel(const RotaryParams p) {
  using E = Elt<BF16>;
  typedef unsigned short u16;
  const int half = p.rotary_dim / 2;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)p.b * p.seqlen * p.h * half;
  if (idx >= total) return;
  const int i = (int)(idx % half);
  int64_t rest = idx / half;
  const int head = (int)(rest % p.h);
  rest /= p.h;
  const int row = (int)(rest % p.seqlen);
  const int bidb = (int)(rest / p.seqlen);
  const int i1 = INTERLEAVED ? 2 * i : i;
  const int i2 = INTERLEAVED ? 2 * i + 1 : i + half;
  const u16* x = (const u16*)p.x + (int64_t)bidb * p.x_batch + (int64_t)row * p.x_row + (int64_t)head * p.x_head;
  u16* o = (u16*)p.out + (int64_t)bidb * p.o_batch + (int64_t)row * p.o_row + (int64_t)head * p.o_head;
  const float x1 = E::to_f32(x[i1]), x2 = E::to_f32(x[i2]);
  const float c = E::to_f32(((const u16*)p.cos)[(int64_t)row * p.cs_row + i]);
  float sn = E::to_f32(((const u16*)p.sin)[(int64_t)row * p.cs_row + i]);
  if (CONJ) sn = -sn;
  const float o1 = x1 * c - x2 * sn;
  const float o2 = x1 * sn + x2 * c;
  o[i1] = (u16)(E::pack2(o1, 0.f) & 0xffffu);
  o[i2] = (u16)(E::pack2(o2, 0.f) & 0xffffu);
}

template <bool BF16>
static void dispatch_rotary(const RotaryParams& p, bool interleaved, bool conj, hipStream_t stream) {
  const int64_t total = (int64_t)p.b * p.seqlen * p.h * (p.rotary_dim / 2);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (interleaved) {
    if (conj) hipLaunchKernelGGL((rotary_kernel<BF16, true, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((rotary_kernel<BF16, true, false>), grid, dim3(256), 0, stream, p);
  } else {
    if (conj) hipLaunchKernelGGL((rotary_kernel<BF16, false, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((rotary_kernel<BF16, false, false>), grid, dim3(256), 0, stream, p);
  }
}

void launch_rotary(const RotaryParams& p, bool interleaved, bool conj, bool is_bf16, hipStream_t stream) {
  const int64_t total = (int64_t)p.b * p.seqlen * p.h * (p.rotary_dim / 2);
  if (total <= 0) return;
  if ((total + 255) / 256 > 0x7fffffff) throw std::runtime_error("rotary: too many elements for one launch");
  if (is_bf16) dispatch_rotary<true>(p, interleaved, conj, stream);
  else dispatch_rotary<false>(p, interleaved, conj, stream);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("rotary launch: ") + hipGetErrorString(e));
}

}  // namespace fa
