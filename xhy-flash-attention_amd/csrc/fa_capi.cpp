// C ABI of libflash_attn_mi355x.so (declarations: include/flash_attn.h).
//
// Mirrors the reference's Paddle C ABI (reference csrc/capi/flash_attn.cu): bool return + a
// thread-local error string (flash_attn.cu:45-67), argument checks of CHECK_FWD_EXECTUABLE /
// CHECK_BWD_EXECTUABLE (:69-90), strided parameter set-up (set_params_fprop_strided :98-229,
// set_params_dgrad_strided :413-533) and the four entry points (:576-1105).  The arch check is
// gfx950 (MI355X) instead of sm80/sm90.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "../../include/flash_attn.h"
#include "fa_params.h"

namespace {

thread_local std::unique_ptr<char[]> g_err;

void set_error(const char* msg) {
  if (msg == nullptr || *msg == '\0') msg = "unknown error";
  const size_t n = std::strlen(msg);
  std::unique_ptr<char[]> m(new char[n + 1]);
  std::memcpy(m.get(), msg, n + 1);
  g_err = std::move(m);
}

#define FA_CHECK(cond)                                                                          \
  do {                                                                                          \
    if (!(cond))                                                                                \
      throw std::runtime_error(std::string("`") + #cond + "` check failed at " + __FILE__ + ":" + \
                               std::to_string(__LINE__));                                       \
  } while (0)

#define FA_BEGIN try {
#define FA_END                                  \
  }                                             \
  catch (const std::exception& e) {             \
    set_error(e.what());                        \
    return false;                               \
  }                                             \
  catch (...) {                                 \
    set_error(nullptr);                         \
    return false;                               \
  }

// gfx950 only: this library carries no other code objects.
void check_device() {
  static thread_local int checked_dev = -1;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("hipGetDevice failed");
  if (dev == checked_dev) return;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) throw std::runtime_error("hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    throw std::runtime_error(std::string("FlashAttention MI355X build requires gfx950, got ") + prop.gcnArchName);
  checked_dev = dev;
}

// FlashMask column-range mask arguments of the reference C ABI (capi/flash_attn.h:38-43); the
// reference takes the FlashMask path iff downstart is non-null (flash_attn.cu:540, 795).
struct FlashMaskArgs {
  const void* downstart;        // LTStart
  const int64_t* dims;          // dims[1] = heads of the mask (reference mask_head_mod_size)
  const void* upend;            // UTEnd
  const void* downend;          // LTEnd
  const void* upstart;          // UTStart
};

void check_common(int batch_size, int num_heads, int num_heads_k, int head_size,
                  int head_size_rounded, float p_dropout, const void* attn_mask,
                  const FlashMaskArgs* flashmask) {
  check_device();
  FA_CHECK(batch_size > 0);
  FA_CHECK(num_heads > 0 && num_heads_k > 0);
  FA_CHECK(head_size % 8 == 0);
  FA_CHECK(head_size <= 256);
  FA_CHECK(num_heads % num_heads_k == 0);
  FA_CHECK(head_size_rounded >= head_size);
  if (attn_mask != nullptr && flashmask != nullptr && flashmask->downstart != nullptr)
    throw std::runtime_error("attn_mask and FlashMask cannot be combined");
  FA_CHECK(p_dropout >= 0.f && p_dropout < 1.f);
}

fa::AttnShape make_shape(int b, int h, int hk, int sq, int sk, int d, float scale, bool causal,
                         const int* cu_q, const int* cu_k, bool padded, float p_dropout,
                         uint64_t seed, uint64_t offset) {
  fa::AttnShape s;
  std::memset(&s, 0, sizeof(s));
  s.b = b; s.h = h; s.hk = hk; s.seqlen_q = sq; s.seqlen_k = sk; s.d = d;
  s.lse_pitch = sq;
  s.cu_seqlens_q = cu_q; s.cu_seqlens_k = cu_k; s.varlen_padded_input = padded;
  s.causal = causal;
  s.scale = scale;
  s.scale_log2 = scale * 1.4426950408889634f;
  // reference set_params_fprop (flash_api.cpp:94-100): keep prob, its uint8 threshold, 1 / keep prob
  s.dropout = p_dropout > 0.f;
  s.p_keep = 1.f - p_dropout;
  s.keep_u8 = (unsigned)(uint8_t)std::floor(s.p_keep * 255.0);
  s.rp_dropout = 1.f / s.p_keep;
  s.philox_seed = seed;
  s.philox_offset = offset;
  return s;
}

// Dense additive mask (reference capi flash_attn.cu:623-624: mask_head_mod_size = mask_dims[1],
// mask_seq_q_mod_size = mask_dims[2]; the kernels index rows with seqlen_k as the stride,
// flash_fwd_kernel.h:640-643).  mask_dims = {batch, heads or a divisor pattern, rows, seqlen_k}.
void set_mask(fa::AttnShape& s, const void* attn_mask, const int64_t* mask_dims, float unscale) {
  if (attn_mask == nullptr) return;
  FA_CHECK(mask_dims != nullptr);
  if (mask_dims[0] != s.b || mask_dims[1] < 1 || mask_dims[2] < 1 || mask_dims[3] != s.seqlen_k)
    throw std::runtime_error("attn_mask: mask_dims must be {batch, heads_mod >= 1, rows_mod >= 1, seqlen_k}");
  s.mask = attn_mask;
  s.mask_h = (int)mask_dims[1];
  s.mask_sq = (int)mask_dims[2];
  s.mask_row = mask_dims[3];
  s.mask_unscale = unscale;
}

// FlashMask (reference capi flash_attn.cu:204-209, mask.h, flash_fwd_kernel.h:1055-1700): int32
// row bounds per key column, (batch, mask heads, seqlen_k) each, head index head / (h / mask_heads).
// The reference's caller-provided maxmin scratch feeds its tile-skip scan; the MI355X kernels
// classify tiles themselves and do not need it.
void set_flashmask(fa::AttnShape& s, const FlashMaskArgs* fm) {
  if (fm == nullptr || fm->downstart == nullptr) return;
  if (fm->dims == nullptr || fm->dims[1] < 1 || s.h % fm->dims[1] != 0)
    throw std::runtime_error("FlashMask: flashmask_dims[1] must divide num_heads");
  if (!s.causal && fm->upend == nullptr)
    throw std::runtime_error("FlashMask: non-causal attention needs flashmask_upend_ptr");
  if (!s.causal && fm->upstart != nullptr && fm->downend == nullptr)
    throw std::runtime_error("FlashMask: flashmask_upstart_ptr needs flashmask_downend_ptr");
  s.fm_lts = static_cast<const int*>(fm->downstart);
  s.fm_lte = static_cast<const int*>(fm->downend);
  s.fm_uts = s.causal ? nullptr : static_cast<const int*>(fm->upstart);
  s.fm_ute = s.causal ? nullptr : static_cast<const int*>(fm->upend);
  s.fm_h = (int)fm->dims[1];
}

bool fwd_impl(const void* q, const void* k, const void* v, const int32_t* cu_q, const int32_t* cu_k,
              void* rng_state, void* out, void* softmax_ptr, void* lse, int b, int sq, int sk,
              int sq_r, int sk_r,
              int h, int hk, int d, int d_r, float p_dropout, float scale, bool causal,
              bool return_softmax, bool is_bf16, hipStream_t stream, uint64_t seed, uint64_t offset,
              const void* attn_mask, const FlashMaskArgs* flashmask, int q_row, int k_row, int v_row,
              int q_head, int k_head, int v_head, int o_row, int o_head, int q_batch, int k_batch,
              int v_batch, int o_batch, bool padded, const int64_t* mask_dims = nullptr,
              float unscale = 1.f) {
  FA_BEGIN
  check_common(b, h, hk, d, d_r, p_dropout, attn_mask, flashmask);
  // return_softmax is accepted with or without dropout, as the reference C ABI passes softmax_ptr
  // whenever it is set (capi/flash_attn.cu:641, 747); the "p_dropout > 0" rule is the torch
  // binding's (flash_api.cpp:276-279) and lives in flash_attn_2_cuda.py.  The probabilities come
  // from the same scores as O and LSE (on a folding call: from Q', attn_folds_q).
  FA_CHECK(q && k && v && out && lse);
  fa::FwdParams p;
  std::memset(&p, 0, sizeof(p));
  p.s = make_shape(b, h, hk, sq, sk, d, scale, causal, cu_q, cu_k, padded, p_dropout, seed, offset);
  set_mask(p.s, attn_mask, mask_dims, unscale);
  set_flashmask(p.s, flashmask);
  if (return_softmax) {
    FA_CHECK(softmax_ptr != nullptr && sq_r >= sq && sk_r >= sk);
    p.p_out = softmax_ptr;
    p.p_rows = sq_r;
    p.p_cols = sk_r;
  }
  p.q = q; p.k = k; p.v = v; p.o = out; p.lse = static_cast<float*>(lse);
  p.q_batch = q_batch; p.q_row = q_row; p.q_head = q_head;
  p.k_batch = k_batch; p.k_row = k_row; p.k_head = k_head;
  p.v_batch = v_batch; p.v_row = v_row; p.v_head = v_head;
  p.o_batch = o_batch; p.o_row = o_row; p.o_head = o_head;
  int bm, bn;
  fa::fwd_block_size(d, &bm, &bn);
  p.num_m_blocks = (sq + bm - 1) / bm;
  p.rng_state = static_cast<uint64_t*>(rng_state);
  p.seed = seed; p.offset = offset;
  fa::launch_fwd(p, is_bf16, stream);
  return true;
  FA_END
}

bool bwd_impl(const void* dout, const void* q, const void* k, const void* v, const void* out,
              const void* softmax_d, const void* lse, const int32_t* cu_q, const int32_t* cu_k,
              void* dq, void* dk, void* dv, void* dq_accum, int b, int sq, int sk, int sq_r,
              int h, int hk, int d, int d_r, float p_dropout, float scale, bool causal,
              bool is_bf16, hipStream_t stream, const void* attn_mask, const FlashMaskArgs* flashmask,
              int q_row, int k_row, int v_row, int q_head, int k_head, int v_head, int o_row,
              int o_head, int q_batch, int k_batch, int v_batch, int o_batch, int dq_row,
              int dk_row, int dv_row, int dq_head, int dk_head, int dv_head, int do_row,
              int do_head, int dq_batch, int dk_batch, int dv_batch, int do_batch, bool padded,
              bool gqa_reduce, void* rng_state, uint64_t seed, uint64_t offset,
              const int64_t* mask_dims = nullptr, float unscale = 1.f) {
  FA_BEGIN
  check_common(b, h, hk, d, d_r, p_dropout, attn_mask, flashmask);
  FA_CHECK(dout && q && k && v && out && softmax_d && lse && dq && dk && dv);
  FA_CHECK(d_r % 32 == 0);
  FA_CHECK(sq_r >= sq);
  fa::BwdParams p;
  std::memset(&p, 0, sizeof(p));
  p.s = make_shape(b, h, hk, sq, sk, d, scale, causal, cu_q, cu_k, padded, p_dropout, seed, offset);
  set_mask(p.s, attn_mask, mask_dims, unscale);
  set_flashmask(p.s, flashmask);
  p.s.lse_pitch = sq;
  if (p.s.dropout && rng_state != nullptr) {
    if (gqa_reduce) {
      // MI355X entry points (*_bwd_gqa): rng_state is the forward's record and the kernels read
      // (seed, offset) from it on the device, as the reference's torch op does with rng_state
      // (flash_api.cpp:669-670, flash_bwd_kernel.h:783-784); seed / offset are ignored.
      p.s.philox_dev = static_cast<const uint64_t*>(rng_state);
    } else {
      // reference capi flash_attn.cu:943-947: {seed, offset} is written into rng_state
      const uint64_t st[2] = {seed, offset};
      if (hipMemcpyAsync(rng_state, st, sizeof(st), hipMemcpyHostToDevice, stream) != hipSuccess)
        throw std::runtime_error("flash_attn_bwd: rng_state copy failed");
    }
  }  // softmax_lse is (b, h, seqlen_q) as written by the forward
  p.q = q; p.k = k; p.v = v; p.o = out; p.dout = dout;
  p.dq = dq; p.dk = dk; p.dv = dv;
  p.lse = static_cast<const float*>(lse);
  p.dsum = static_cast<float*>(const_cast<void*>(softmax_d));
  p.dq_accum = static_cast<float*>(dq_accum);
  p.q_batch = q_batch; p.q_row = q_row; p.q_head = q_head;
  p.k_batch = k_batch; p.k_row = k_row; p.k_head = k_head;
  p.v_batch = v_batch; p.v_row = v_row; p.v_head = v_head;
  p.o_batch = o_batch; p.o_row = o_row; p.o_head = o_head;
  p.do_batch = do_batch; p.do_row = do_row; p.do_head = do_head;
  p.dq_batch = dq_batch; p.dq_row = dq_row; p.dq_head = dq_head;
  p.dk_batch = dk_batch; p.dk_row = dk_row; p.dk_head = dk_head;
  p.dv_batch = dv_batch; p.dv_row = dv_row; p.dv_head = dv_head;
  p.seqlen_q_rounded = sq_r;
  p.d_rounded = d_r;
  p.gqa_reduce = gqa_reduce && (h != hk);
  int bm, bn;
  fa::bwd_block_size(d, &bm, &bn);
  p.num_n_blocks = (sk + bn - 1) / bn;
  fa::launch_bwd(p, is_bf16, stream);
  return true;
  FA_END
}

}  // namespace

extern "C" {

// reference csrc/capi/flash_attn.h:313-315 (flash_attn.cu:47-60)
void flash_attn_set_error(const char* msg) { set_error(msg); }
const char* flash_attn_error() { return g_err.get(); }

void flash_attn_block_size(int head_size, int is_backward, int* block_m, int* block_n) {
  if (is_backward) fa::bwd_block_size(head_size, block_m, block_n);
  else fa::fwd_block_size(head_size, block_m, block_n);
}

bool flash_attn_fwd(const void* const q, const void* const k, const void* const v,
                    void* const rng_state, void* const out, void* const softmax_ptr,
                    void* const softmax_lse_ptr, const int batch_size, const int seqlen_q,
                    const int seqlen_k, const int seqlen_q_rounded, const int seqlen_k_rounded,
                    const int num_heads, const int num_heads_k, const int head_size,
                    const int head_size_rounded, const float p_dropout, const float softmax_scale,
                    const float softmax_unscale, const bool is_causal, const bool return_softmax,
                    const bool is_bf16, hipStream_t stream, uint64_t seed, uint64_t offset,
                    const void* const attn_mask, const int64_t* const mask_dims,
                    const void* const flashmask_downstart_ptr, const int64_t* const flashmask_dims,
                    const void* const flashmask_upend_ptr, const void* const flashmask_downend_ptr,
                    const void* const flashmask_upstart_ptr, const void* const flashmask_maxmin_ptr,
                    const int q_row_stride, const int k_row_stride, const int v_row_stride,
                    const int q_head_stride, const int k_head_stride, const int v_head_stride,
                    const int o_row_stride, const int o_head_stride, const int q_batch_stride,
                    const int k_batch_stride, const int v_batch_stride, const int o_batch_stride) {
  (void)flashmask_maxmin_ptr;
  const FlashMaskArgs fm = {flashmask_downstart_ptr, flashmask_dims, flashmask_upend_ptr,
                            flashmask_downend_ptr, flashmask_upstart_ptr};
  return fwd_impl(q, k, v, nullptr, nullptr, rng_state, out, softmax_ptr, softmax_lse_ptr,
                  batch_size, seqlen_q, seqlen_k, seqlen_q_rounded, seqlen_k_rounded,
                  num_heads, num_heads_k, head_size,
                  head_size_rounded, p_dropout, softmax_scale, is_causal, return_softmax, is_bf16,
                  stream, seed, offset, attn_mask, &fm, q_row_stride,
                  k_row_stride, v_row_stride, q_head_stride, k_head_stride, v_head_stride,
                  o_row_stride, o_head_stride, q_batch_stride, k_batch_stride, v_batch_stride,
                  o_batch_stride, false, mask_dims, softmax_unscale);
}

bool flash_attn_varlen_fwd(const void* const q, const void* const k, const void* const v,
                           const int32_t* const cu_seqlens_q, const int32_t* const cu_seqlens_k,
                           void* const rng_state, void* const out, void* const softmax_ptr,
                           void* const softmax_lse_ptr, const int batch_size,
                           const int max_seqlen_q, const int max_seqlen_k,
                           const int seqlen_q_rounded, const int seqlen_k_rounded,
                           const int num_heads, const int num_heads_k, const int head_size,
                           const int head_size_rounded, const float p_dropout,
                           const float softmax_scale, const float softmax_unscale,
                           const bool is_causal, const bool return_softmax, const bool is_bf16,
                           hipStream_t stream, uint64_t seed, uint64_t offset,
                           const void* const attn_mask, const void* const mask_dims,
                           const int q_row_stride, const int k_row_stride, const int v_row_stride,
                           const int q_head_stride, const int k_head_stride,
                           const int v_head_stride, const int o_row_stride,
                           const int o_head_stride, const int q_batch_stride,
                           const int k_batch_stride, const int v_batch_stride,
                           const int o_batch_stride, bool varlen_padded_input) {
  if (cu_seqlens_q == nullptr || cu_seqlens_k == nullptr) {
    set_error("flash_attn_varlen_fwd: cu_seqlens_q / cu_seqlens_k must not be null");
    return false;
  }
  return fwd_impl(q, k, v, cu_seqlens_q, cu_seqlens_k, rng_state, out, softmax_ptr,
                  softmax_lse_ptr, batch_size, max_seqlen_q, max_seqlen_k, seqlen_q_rounded,
                  seqlen_k_rounded, num_heads, num_heads_k,
                  head_size, head_size_rounded, p_dropout, softmax_scale, is_causal,
                  return_softmax, is_bf16, stream, seed, offset, attn_mask, nullptr, q_row_stride,
                  k_row_stride, v_row_stride, q_head_stride, k_head_stride, v_head_stride,
                  o_row_stride, o_head_stride, q_batch_stride, k_batch_stride, v_batch_stride,
                  o_batch_stride, varlen_padded_input, static_cast<const int64_t*>(mask_dims),
                  softmax_unscale);
}

#define FA_BWD_ARGS                                                                               \
  const void *const dout, const void *const q, const void *const k, const void *const v,          \
      const void *const out, const void *const softmax_d, const void *const softmax_lse,          \
      void *const rng_state, void *const dq, void *const dk, void *const dv,                       \
      void *const dq_accum, const int batch_size, const int seqlen_q, const int seqlen_k,          \
      const int seqlen_q_rounded, const int seqlen_k_rounded, const int num_heads,                 \
      const int num_heads_k, const int head_size, const int head_size_rounded,                     \
      const float p_dropout, const float softmax_scale, const float softmax_unscale,               \
      const bool is_causal, const bool is_bf16, const int num_splits, hipStream_t stream,          \
      uint64_t seed, uint64_t offset, const void *const attn_mask,                                 \
      const int64_t *const mask_dims, const void *const flashmask_downstart_ptr,                   \
      const int64_t *const flashmask_dims, const void *const flashmask_upend_ptr,                  \
      const void *const flashmask_downend_ptr, const void *const flashmask_upstart_ptr,            \
      const void *const flashmask_maxmin_ptr, const int q_row_stride, const int k_row_stride,      \
      const int v_row_stride, const int q_head_stride, const int k_head_stride,                    \
      const int v_head_stride, const int o_row_stride, const int o_head_stride,                    \
      const int q_batch_stride, const int k_batch_stride, const int v_batch_stride,                \
      const int o_batch_stride, const int dq_row_stride, const int dk_row_stride,                  \
      const int dv_row_stride, const int dq_head_stride, const int dk_head_stride,                 \
      const int dv_head_stride, const int do_row_stride, const int do_head_stride,                 \
      const int dq_batch_stride, const int dk_batch_stride, const int dv_batch_stride,             \
      const int do_batch_stride

#define FA_BWD_CALL(GQA)                                                                          \
  (void)seqlen_k_rounded; (void)num_splits;                                                       \
  (void)flashmask_maxmin_ptr;                                                                      \
  const FlashMaskArgs fm = {flashmask_downstart_ptr, flashmask_dims, flashmask_upend_ptr,          \
                            flashmask_downend_ptr, flashmask_upstart_ptr};                         \
  return bwd_impl(dout, q, k, v, out, softmax_d, softmax_lse, nullptr, nullptr, dq, dk, dv,        \
                  dq_accum, batch_size, seqlen_q, seqlen_k, seqlen_q_rounded, num_heads,           \
                  num_heads_k, head_size, head_size_rounded, p_dropout, softmax_scale, is_causal,  \
                  is_bf16, stream, attn_mask, &fm, q_row_stride, k_row_stride,                     \
                  v_row_stride, q_head_stride, k_head_stride, v_head_stride, o_row_stride,         \
                  o_head_stride, q_batch_stride, k_batch_stride, v_batch_stride, o_batch_stride,   \
                  dq_row_stride, dk_row_stride, dv_row_stride, dq_head_stride, dk_head_stride,     \
                  dv_head_stride, do_row_stride, do_head_stride, dq_batch_stride, dk_batch_stride, \
                  dv_batch_stride, do_batch_stride, false, GQA, rng_state, seed, offset,         \
                  mask_dims, softmax_unscale)

bool flash_attn_bwd(FA_BWD_ARGS) { FA_BWD_CALL(false); }
bool flash_attn_bwd_gqa(FA_BWD_ARGS) { FA_BWD_CALL(true); }

#define FA_VARLEN_BWD_ARGS                                                                        \
  const void *const dout, const void *const q, const void *const k, const void *const v,          \
      const void *const out, const void *const softmax_d, const void *const softmax_lse,          \
      const int32_t *const cu_seqlens_q, const int32_t *const cu_seqlens_k,                        \
      void *const rng_state, void *const dq, void *const dk, void *const dv,                       \
      void *const dq_accum, const int batch_size, const int max_seqlen_q,                          \
      const int max_seqlen_k, const int seqlen_q_rounded, const int seqlen_k_rounded,              \
      const int num_heads, const int num_heads_k, const int head_size,                             \
      const int head_size_rounded, const float p_dropout, const float softmax_scale,               \
      const float softmax_unscale, const bool is_causal, const bool is_bf16,                       \
      const int num_splits, hipStream_t stream, uint64_t seed, uint64_t offset,                    \
      const void *attn_mask, const int64_t *const mask_dims, const int q_row_stride,               \
      const int k_row_stride, const int v_row_stride, const int q_head_stride,                     \
      const int k_head_stride, const int v_head_stride, const int o_row_stride,                    \
      const int o_head_stride, const int q_batch_stride, const int k_batch_stride,                 \
      const int v_batch_stride, const int o_batch_stride, const int dq_row_stride,                 \
      const int dk_row_stride, const int dv_row_stride, const int dq_head_stride,                  \
      const int dk_head_stride, const int dv_head_stride, const int do_row_stride,                 \
      const int do_head_stride, const int dq_batch_stride, const int dk_batch_stride,              \
      const int dv_batch_stride, const int do_batch_stride, const bool varlen_padded_input

#define FA_VARLEN_BWD_CALL(GQA)                                                                   \
  (void)seqlen_k_rounded; (void)num_splits;                                                       \
  if (cu_seqlens_q == nullptr || cu_seqlens_k == nullptr) {                                        \
    set_error("flash_attn_varlen_bwd: cu_seqlens_q / cu_seqlens_k must not be null");             \
    return false;                                                                                  \
  }                                                                                                \
  return bwd_impl(dout, q, k, v, out, softmax_d, softmax_lse, cu_seqlens_q, cu_seqlens_k, dq, dk,  \
                  dv, dq_accum, batch_size, max_seqlen_q, max_seqlen_k, seqlen_q_rounded,          \
                  num_heads, num_heads_k, head_size, head_size_rounded, p_dropout, softmax_scale,  \
                  is_causal, is_bf16, stream, attn_mask, nullptr, q_row_stride, k_row_stride,      \
                  v_row_stride, q_head_stride, k_head_stride, v_head_stride, o_row_stride,         \
                  o_head_stride, q_batch_stride, k_batch_stride, v_batch_stride, o_batch_stride,   \
                  dq_row_stride, dk_row_stride, dv_row_stride, dq_head_stride, dk_head_stride,     \
                  dv_head_stride, do_row_stride, do_head_stride, dq_batch_stride, dk_batch_stride, \
                  dv_batch_stride, do_batch_stride, varlen_padded_input, GQA, rng_state, seed,     \
                  offset, mask_dims, softmax_unscale)

bool flash_attn_varlen_bwd(FA_VARLEN_BWD_ARGS) { FA_VARLEN_BWD_CALL(false); }

// reference csrc/capi/flash_attn.cu:1107-1201 (o_* strides are accepted and unused there too)
bool calc_reduced_attn_scores(const void* const q, const void* const k, const void* const softmax_lse,
                              void* const reduced_scores, void* const softmax_ptr, const int batch_size,
                              const int seqlen_q, const int seqlen_k, const int num_heads,
                              const int num_heads_k, const int head_size, const float softmax_scale,
                              const bool return_softmax, const bool is_bf16, const int num_splits,
                              hipStream_t stream, const int q_row_stride, const int k_row_stride,
                              const int o_row_stride, const int q_head_stride, const int k_head_stride,
                              const int o_head_stride, const int q_batch_stride, const int k_batch_stride,
                              const int o_batch_stride) {
  (void)num_splits; (void)o_row_stride; (void)o_head_stride; (void)o_batch_stride;
  FA_BEGIN
  check_common(batch_size, num_heads, num_heads_k, head_size, head_size, 0.f, nullptr, nullptr);
  FA_CHECK(q && k && softmax_lse && reduced_scores);
  FA_CHECK(seqlen_q > 0 && seqlen_k > 0);
  if (return_softmax) FA_CHECK(softmax_ptr != nullptr);
  fa::ReducedParams p;
  std::memset(&p, 0, sizeof(p));
  p.q = q; p.k = k;
  p.lse = static_cast<const float*>(softmax_lse);
  p.reduced = static_cast<float*>(reduced_scores);
  p.p_out = return_softmax ? static_cast<float*>(softmax_ptr) : nullptr;
  p.b = batch_size; p.h = num_heads; p.hk = num_heads_k;
  p.sq = seqlen_q; p.sk = seqlen_k; p.d = head_size;
  p.scale = softmax_scale;
  p.q_batch = q_batch_stride; p.q_row = q_row_stride; p.q_head = q_head_stride;
  p.k_batch = k_batch_stride; p.k_row = k_row_stride; p.k_head = k_head_stride;
  fa::launch_reduced_scores(p, is_bf16, stream);
  return true;
  FA_END
}
bool flash_attn_varlen_bwd_gqa(FA_VARLEN_BWD_ARGS) { FA_VARLEN_BWD_CALL(true); }

// reference csrc/rotary/rotary.cpp:16-37 (apply_rotary on the x1 / x2 halves, conj for the
// backward); here on the whole (b, seqlen, h, d) view, rotary_dim leading columns.
bool flash_attn_rotary_apply(const void* const x, void* const out, const void* const cos,
                             const void* const sin, const int batch_size, const int seqlen,
                             const int num_heads, const int rotary_dim, const int64_t x_batch_stride,
                             const int64_t x_row_stride, const int64_t x_head_stride,
                             const int64_t out_batch_stride, const int64_t out_row_stride,
                             const int64_t out_head_stride, const int64_t cos_row_stride,
                             const bool interleaved, const bool conj, const bool is_bf16,
                             hipStream_t stream) {
  FA_BEGIN
  check_device();
  FA_CHECK(x && out && cos && sin);
  FA_CHECK(batch_size >= 0 && seqlen >= 0 && num_heads >= 0);
  FA_CHECK(rotary_dim > 0 && rotary_dim % 2 == 0);
  fa::RotaryParams p;
  std::memset(&p, 0, sizeof(p));
  p.x = x; p.out = out; p.cos = cos; p.sin = sin;
  p.b = batch_size; p.seqlen = seqlen; p.h = num_heads; p.rotary_dim = rotary_dim;
  p.x_batch = x_batch_stride; p.x_row = x_row_stride; p.x_head = x_head_stride;
  p.o_batch = out_batch_stride; p.o_row = out_row_stride; p.o_head = out_head_stride;
  p.cs_row = cos_row_stride;
  fa::launch_rotary(p, interleaved, conj, is_bf16, stream);
  return true;
  FA_END
}

}  // extern "C"
