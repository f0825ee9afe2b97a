/*
 * C ABI of the MI355X-native FlashAttention-2 library (libflash_attn_mi355x.so).
 *
 * This is the drop-in boundary for the hot path.  Each entry point replaces the
 * entry of the same name in the reference's Paddle C ABI (reference
 * csrc/capi/flash_attn.h) with an identical argument list, except that the
 * stream is a hipStream_t instead of a cudaStream_t:
 *
 *   flash_attn_fwd         <- reference csrc/capi/flash_attn.h:11-55
 *   flash_attn_varlen_fwd  <- reference csrc/capi/flash_attn.h:57-98
 *   flash_attn_bwd         <- reference csrc/capi/flash_attn.h:100-161
 *   flash_attn_varlen_bwd  <- reference csrc/capi/flash_attn.h:163-221
 *   flash_attn_set_error   <- reference csrc/capi/flash_attn.h:313
 *   flash_attn_error       <- reference csrc/capi/flash_attn.h:315
 *   calc_reduced_attn_scores <- reference csrc/capi/flash_attn.h:223-247
 *
 * Conventions (reference csrc/capi/flash_attn.cu:29-96, 576-1105):
 *   - every buffer is a caller-owned device pointer; strides are in ELEMENTS;
 *   - calls are stream-ordered and never synchronise;
 *   - a call returns false on error and leaves a thread-local message readable
 *     through flash_attn_error();
 *   - head_size % 8 == 0, head_size <= 256, num_heads % num_heads_k == 0;
 *   - attn_mask (dense additive Paddle mask, input dtype) is supported in the
 *     forward and backward entry points: raw scores QK^T get
 *     attn_mask[b][h % mask_dims[1]][q % mask_dims[2]][k] * softmax_unscale
 *     added before the softmax scale (reference flash_fwd_kernel.h:640-660,
 *     softmax.h:361-379); mask_dims = {batch, head modulus, row modulus,
 *     seqlen_k} (host int64[4], reference flash_attn.cu:623-624); with
 *     return_softmax the S_dmask probabilities include the mask;
 *   - FlashMask (flash_attn_fwd / flash_attn_bwd*, not varlen, reference
 *     flash_attn.cu:204-209): active iff flashmask_downstart_ptr != NULL.
 *     int32 row bounds of shape (batch, flashmask_dims[1], seqlen_k) each;
 *     attention head h uses mask head h / (num_heads / flashmask_dims[1]).
 *     Causal: key k is hidden from rows in [downstart[k], downend[k]) (downend
 *     NULL: to the end).  Non-causal: rows in [downstart, downend) and
 *     [upstart, upend) when upstart is given, else rows >= downstart or
 *     < upend; upend is required (reference softmax.h:180-298).  Pass the same
 *     pointers to the backward.  flashmask_maxmin_ptr (the reference's
 *     tile-scan scratch) is accepted and not used.  Not combined with attn_mask;
 *     with return_softmax the S_dmask zeroes the hidden entries.  Rows that see
 *     no key give out = 0, LSE = +inf;
 *   - backward: softmax_d (b, h, seqlen_q_rounded) fp32 is a caller-owned
 *     output (D = rowsum(dO * O)); dq_accum is caller-owned fp32 SCRATCH of at
 *     least batch * num_heads * seqlen_q_rounded floats (the reference's
 *     (b, h, sq_r, d_r) dq_accum always qualifies).  The MI355X backward needs
 *     no fp32 dQ accumulator (dQ has its own kernel, no atomics); it stores
 *     -LSE / softmax_scale per query row there.  dq_accum may be NULL: the
 *     library then takes the scratch from the stream-ordered allocator
 *     (hipMallocAsync / hipFreeAsync on `stream`); for MQA/GQA the caller passes dk/dv
 *     with num_heads heads ("expanded", reference flash_api.cpp:628-635) and
 *     sums the groups itself;
 *   - num_splits is accepted and ignored: the MI355X backward uses no atomics,
 *     so dQ, dK and dV are bitwise deterministic for every value;
 *   - return_softmax is honoured with or without dropout (reference
 *     flash_attn.cu:641, 747); the probabilities come from the scores O and LSE
 *     were computed from.
 *
 * MI355X extensions (no reference counterpart):
 *   flash_attn_bwd_gqa / flash_attn_varlen_bwd_gqa take the same arguments as
 *   the reference entries but write dk/dv with num_heads_k heads, summing each
 *   query-head group inside the kernel (no expanded buffers, no extra HBM pass:
 *   replaces the at::sum_out of reference flash_api.cpp:682-686, 900-904).
 *   With dropout, their rng_state (when non-NULL) is an INPUT: the forward's
 *   {seed, offset} record, read by the kernels on the device (as the
 *   reference's torch op reads rng_state, flash_api.cpp:669-670 /
 *   flash_bwd_kernel.h:783-784), and the seed / offset arguments are ignored;
 *   the reference-shaped entries keep the Paddle C ABI behaviour of writing
 *   {seed, offset} into rng_state (flash_attn.cu:943-947).
 *   flash_attn_block_size reports the tile sizes the launchers use.
 */
#ifndef FLASH_ATTN_MI355X_H_
#define FLASH_ATTN_MI355X_H_

#include <hip/hip_runtime.h>
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

bool flash_attn_fwd(const void * const q,
                    const void * const k,
                    const void * const v,
                    void * const rng_state,
                    void * const out,
                    void * const softmax_ptr,
                    void * const softmax_lse_ptr,
                    const int batch_size,
                    const int seqlen_q,
                    const int seqlen_k,
                    const int seqlen_q_rounded,
                    const int seqlen_k_rounded,
                    const int num_heads,
                    const int num_heads_k,
                    const int head_size,
                    const int head_size_rounded,
                    const float p_dropout,
                    const float softmax_scale,
                    const float softmax_unscale,
                    const bool is_causal,
                    const bool return_softmax,
                    const bool is_bf16,
                    hipStream_t stream,
                    uint64_t seed,
                    uint64_t offset,
                    const void * const attn_mask,
                    const int64_t * const mask_dims,
                    const void * const flashmask_downstart_ptr,
                    const int64_t * const flashmask_dims,
                    const void * const flashmask_upend_ptr,
                    const void * const flashmask_downend_ptr,
                    const void * const flashmask_upstart_ptr,
                    const void * const flashmask_maxmin_ptr,
                    const int q_row_stride,
                    const int k_row_stride,
                    const int v_row_stride,
                    const int q_head_stride,
                    const int k_head_stride,
                    const int v_head_stride,
                    const int o_row_stride,
                    const int o_head_stride,
                    const int q_batch_stride,
                    const int k_batch_stride,
                    const int v_batch_stride,
                    const int o_batch_stride);

bool flash_attn_varlen_fwd(const void * const q,
                           const void * const k,
                           const void * const v,
                           const int32_t * const cu_seqlens_q,
                           const int32_t * const cu_seqlens_k,
                           void * const rng_state,
                           void * const out,
                           void * const softmax_ptr,
                           void * const softmax_lse_ptr,
                           const int batch_size,
                           const int max_seqlen_q,
                           const int max_seqlen_k,
                           const int seqlen_q_rounded,
                           const int seqlen_k_rounded,
                           const int num_heads,
                           const int num_heads_k,
                           const int head_size,
                           const int head_size_rounded,
                           const float p_dropout,
                           const float softmax_scale,
                           const float softmax_unscale,
                           const bool is_causal,
                           const bool return_softmax,
                           const bool is_bf16,
                           hipStream_t stream,
                           uint64_t seed,
                           uint64_t offset,
                           const void * const attn_mask,
                           const void * const mask_dims,
                           const int q_row_stride,
                           const int k_row_stride,
                           const int v_row_stride,
                           const int q_head_stride,
                           const int k_head_stride,
                           const int v_head_stride,
                           const int o_row_stride,
                           const int o_head_stride,
                           const int q_batch_stride,
                           const int k_batch_stride,
                           const int v_batch_stride,
                           const int o_batch_stride,
                           bool varlen_padded_input);

bool flash_attn_bwd(const void * const dout,
                    const void * const q,
                    const void * const k,
                    const void * const v,
                    const void * const out,
                    const void * const softmax_d,
                    const void * const softmax_lse,
                    void * const rng_state,
                    void * const dq,
                    void * const dk,
                    void * const dv,
                    void * const dq_accum,
                    const int batch_size,
                    const int seqlen_q,
                    const int seqlen_k,
                    const int seqlen_q_rounded,
                    const int seqlen_k_rounded,
                    const int num_heads,
                    const int num_heads_k,
                    const int head_size,
                    const int head_size_rounded,
                    const float p_dropout,
                    const float softmax_scale,
                    const float softmax_unscale,
                    const bool is_causal,
                    const bool is_bf16,
                    const int num_splits,
                    hipStream_t stream,
                    uint64_t seed,
                    uint64_t offset,
                    const void * const attn_mask,
                    const int64_t * const mask_dims,
                    const void * const flashmask_downstart_ptr,
                    const int64_t * const flashmask_dims,
                    const void * const flashmask_upend_ptr,
                    const void * const flashmask_downend_ptr,
                    const void * const flashmask_upstart_ptr,
                    const void * const flashmask_maxmin_ptr,
                    const int q_row_stride,
                    const int k_row_stride,
                    const int v_row_stride,
                    const int q_head_stride,
                    const int k_head_stride,
                    const int v_head_stride,
                    const int o_row_stride,
                    const int o_head_stride,
                    const int q_batch_stride,
                    const int k_batch_stride,
                    const int v_batch_stride,
                    const int o_batch_stride,
                    const int dq_row_stride,
                    const int dk_row_stride,
                    const int dv_row_stride,
                    const int dq_head_stride,
                    const int dk_head_stride,
                    const int dv_head_stride,
                    const int do_row_stride,
                    const int do_head_stride,
                    const int dq_batch_stride,
                    const int dk_batch_stride,
                    const int dv_batch_stride,
                    const int do_batch_stride);

bool flash_attn_varlen_bwd(const void * const dout,
                           const void * const q,
                           const void * const k,
                           const void * const v,
                           const void * const out,
                           const void * const softmax_d,
                           const void * const softmax_lse,
                           const int32_t * const cu_seqlens_q,
                           const int32_t * const cu_seqlens_k,
                           void * const rng_state,
                           void * const dq,
                           void * const dk,
                           void * const dv,
                           void * const dq_accum,
                           const int batch_size,
                           const int max_seqlen_q,
                           const int max_seqlen_k,
                           const int seqlen_q_rounded,
                           const int seqlen_k_rounded,
                           const int num_heads,
                           const int num_heads_k,
                           const int head_size,
                           const int head_size_rounded,
                           const float p_dropout,
                           const float softmax_scale,
                           const float softmax_unscale,
                           const bool is_causal,
                           const bool is_bf16,
                           const int num_splits,
                           hipStream_t stream,
                           uint64_t seed,
                           uint64_t offset,
                           const void * attn_mask,
                           const int64_t * const mask_dims,
                           const int q_row_stride,
                           const int k_row_stride,
                           const int v_row_stride,
                           const int q_head_stride,
                           const int k_head_stride,
                           const int v_head_stride,
                           const int o_row_stride,
                           const int o_head_stride,
                           const int q_batch_stride,
                           const int k_batch_stride,
                           const int v_batch_stride,
                           const int o_batch_stride,
                           const int dq_row_stride,
                           const int dk_row_stride,
                           const int dv_row_stride,
                           const int dq_head_stride,
                           const int dk_head_stride,
                           const int dv_head_stride,
                           const int do_row_stride,
                           const int do_head_stride,
                           const int dq_batch_stride,
                           const int dk_batch_stride,
                           const int dv_batch_stride,
                           const int do_batch_stride,
                           const bool varlen_padded_input);

/* reference csrc/capi/flash_attn.h:223-247 (calc_reduced_attn_scores): for every (batch, head,
 * key) the column sum over all queries of exp(softmax_scale * q.k - softmax_lse[q]) into
 * reduced_scores (fp32, batch x num_heads x seqlen_k; written, so it needs no zeroing -- the
 * reference atomically adds into a zeroed buffer), and with return_softmax the probabilities into
 * softmax_ptr (fp32, batch x num_heads x seqlen_q x seqlen_k).  Non-causal, no mask (as the
 * reference); MQA/GQA through num_heads_k.  num_splits and the o_* strides are accepted and unused. */
bool calc_reduced_attn_scores(const void * const q,
                              const void * const k,
                              const void * const softmax_lse,
                              void * const reduced_scores,
                              void * const softmax_ptr,
                              const int batch_size,
                              const int seqlen_q,
                              const int seqlen_k,
                              const int num_heads,
                              const int num_heads_k,
                              const int head_size,
                              const float softmax_scale,
                              const bool return_softmax,
                              const bool is_bf16,
                              const int num_splits,
                              hipStream_t stream,
                              const int q_row_stride,
                              const int k_row_stride,
                              const int o_row_stride,
                              const int q_head_stride,
                              const int k_head_stride,
                              const int o_head_stride,
                              const int q_batch_stride,
                              const int k_batch_stride,
                              const int o_batch_stride);

void flash_attn_set_error(const char *msg);

const char *flash_attn_error();

/* ---- MI355X extensions ---- */

/* Same arguments as flash_attn_bwd; dk/dv have num_heads_k heads (group-summed in kernel). */
bool flash_attn_bwd_gqa(const void * const dout, const void * const q, const void * const k,
                        const void * const v, const void * const out,
                        const void * const softmax_d, const void * const softmax_lse,
                        void * const rng_state, void * const dq, void * const dk,
                        void * const dv, void * const dq_accum,
                        const int batch_size, const int seqlen_q, const int seqlen_k,
                        const int seqlen_q_rounded, const int seqlen_k_rounded,
                        const int num_heads, const int num_heads_k,
                        const int head_size, const int head_size_rounded,
                        const float p_dropout, const float softmax_scale,
                        const float softmax_unscale, const bool is_causal, const bool is_bf16,
                        const int num_splits, hipStream_t stream, uint64_t seed, uint64_t offset,
                        const void * const attn_mask, const int64_t * const mask_dims,
                        const void * const flashmask_downstart_ptr,
                        const int64_t * const flashmask_dims,
                        const void * const flashmask_upend_ptr,
                        const void * const flashmask_downend_ptr,
                        const void * const flashmask_upstart_ptr,
                        const void * const flashmask_maxmin_ptr,
                        const int q_row_stride, const int k_row_stride, const int v_row_stride,
                        const int q_head_stride, const int k_head_stride, const int v_head_stride,
                        const int o_row_stride, const int o_head_stride,
                        const int q_batch_stride, const int k_batch_stride,
                        const int v_batch_stride, const int o_batch_stride,
                        const int dq_row_stride, const int dk_row_stride, const int dv_row_stride,
                        const int dq_head_stride, const int dk_head_stride,
                        const int dv_head_stride, const int do_row_stride,
                        const int do_head_stride, const int dq_batch_stride,
                        const int dk_batch_stride, const int dv_batch_stride,
                        const int do_batch_stride);

/* Same arguments as flash_attn_varlen_bwd; dk/dv have num_heads_k heads. */
bool flash_attn_varlen_bwd_gqa(const void * const dout, const void * const q,
                               const void * const k, const void * const v,
                               const void * const out, const void * const softmax_d,
                               const void * const softmax_lse,
                               const int32_t * const cu_seqlens_q,
                               const int32_t * const cu_seqlens_k, void * const rng_state,
                               void * const dq, void * const dk, void * const dv,
                               void * const dq_accum, const int batch_size,
                               const int max_seqlen_q, const int max_seqlen_k,
                               const int seqlen_q_rounded, const int seqlen_k_rounded,
                               const int num_heads, const int num_heads_k,
                               const int head_size, const int head_size_rounded,
                               const float p_dropout, const float softmax_scale,
                               const float softmax_unscale, const bool is_causal,
                               const bool is_bf16, const int num_splits, hipStream_t stream,
                               uint64_t seed, uint64_t offset, const void * attn_mask,
                               const int64_t * const mask_dims,
                               const int q_row_stride, const int k_row_stride,
                               const int v_row_stride, const int q_head_stride,
                               const int k_head_stride, const int v_head_stride,
                               const int o_row_stride, const int o_head_stride,
                               const int q_batch_stride, const int k_batch_stride,
                               const int v_batch_stride, const int o_batch_stride,
                               const int dq_row_stride, const int dk_row_stride,
                               const int dv_row_stride, const int dq_head_stride,
                               const int dk_head_stride, const int dv_head_stride,
                               const int do_row_stride, const int do_head_stride,
                               const int dq_batch_stride, const int dk_batch_stride,
                               const int dv_batch_stride, const int do_batch_stride,
                               const bool varlen_padded_input);

/* Rotary position embedding of the attention modules; replaces the reference's torch extension
 * op rotary_emb.apply_rotary (csrc/rotary/rotary.cpp:16-37, rotary_cuda.cu:9-45) as used by
 * flash_attn/layers/rotary.py:35-196.  x, out: (batch, seqlen, num_heads, >= rotary_dim) with
 * ELEMENT strides and a contiguous last dim (out may alias x); cos, sin: (seqlen, rotary_dim / 2)
 * with row stride cos_row_stride, input dtype.  For each pair (x1, x2) -- the two halves of the
 * first rotary_dim columns, or (even, odd) columns when interleaved -- writes
 * x1 cos - x2 sin, x1 sin + x2 cos (conj: with -sin, the backward), fp32 arithmetic.  Columns
 * past rotary_dim are not written. */
bool flash_attn_rotary_apply(const void * const x, void * const out, const void * const cos,
                             const void * const sin, const int batch_size, const int seqlen,
                             const int num_heads, const int rotary_dim,
                             const int64_t x_batch_stride, const int64_t x_row_stride,
                             const int64_t x_head_stride, const int64_t out_batch_stride,
                             const int64_t out_row_stride, const int64_t out_head_stride,
                             const int64_t cos_row_stride, const bool interleaved, const bool conj,
                             const bool is_bf16, hipStream_t stream);

/* Tile sizes (block_m x block_n) of the forward / backward launchers for head_size. */
void flash_attn_block_size(int head_size, int is_backward, int * block_m, int * block_n);

/* Per-kernel device timing with HIP events on the launch stream (benchmarking only; not under
 * graph capture).  enable != 0 clears the totals and starts recording.  Kernel ids: 0 forward,
 * 1 backward preprocess (D = rowsum(dO*O)), 2 backward dK/dV, 3 backward dQ, 4 the window from
 * the dK/dV launch to the end of dQ (the two may overlap on two streams). */
void flash_attn_timing_enable(int enable);
void flash_attn_timing_read(int kernel_id, double * total_ms, long * count);

/* Test / A-B switches (no reference counterpart).  Knob ids: 0 never split K/V in the forward
 * (FLASH_ATTN_MI355X_NO_SPLITKV), 1 head-fastest work order (FLASH_ATTN_MI355X_NO_XCD_GROUP),
 * 2 XCD head-grouping threshold in MiB of streamed K/V (FLASH_ATTN_MI355X_XCD_GROUP_MIN_MIB,
 * default 256), 3 / 4 assembly dK/dV / dQ kernels (FLASH_ATTN_MI355X_BWD_ASM / _DQ_ASM, default 1),
 * 5 persistent assembly forward, one workgroup per CU walking the item list
 * (FLASH_ATTN_MI355X_FWD_PERSIST, default 1; 0 = one workgroup per item), 6 the same for the
 * assembly dK/dV and dQ kernels, fixed-length launches (FLASH_ATTN_MI355X_BWD_PERSIST, default 1), 7 knob 2's threshold
 * for the persistent assembly forward and dQ (FLASH_ATTN_MI355X_ASM_XCD_GROUP_MIN_MIB, default 0:
 * heads grouped per XCD whenever the shape allows), 8 the backward preprocessing fused into the
 * assembly dQ kernel (FLASH_ATTN_MI355X_FUSE_PRE, default 1: D = rowsum(dO o O), softmax_d and the
 * dK/dV kernel's scratch are written by dQ, which then runs before dK/dV; 0 launches the separate
 * preprocessing kernel), 9 items per workgroup of the assembly dK/dV kernel on varlen calls
 * (FLASH_ATTN_MI355X_VARLEN_ROUNDS, default 2, in snake-paired rounds; 1: one workgroup per item).
 * Knob 6 = 2 also runs varlen dK/dV persistent, from a device-built work list.  10 the assembly
 * dK/dV kernel with two waves per SIMD, specialised by role (FLASH_ATTN_MI355X_BWD_2W, default 0 =
 * the one-wave-per-SIMD kernel; 1 gives bitwise the same results, measured 7-8 % slower).  11 items
 * per workgroup of the assembly forward on varlen calls that are not persistent
 * (FLASH_ATTN_MI355X_FWD_VARLEN_ROUNDS, snake-paired rounds; 1 = one workgroup per item).  Each is
 * read from its environment variable once, at first use. */
void flash_attn_set_knob(int id, int value);
int flash_attn_get_knob(int id);
/* (FLASH_ATTN_MI355X_NO_QFOLD=1 in the environment, read once per process, makes attn_folds_q false for
 * every call: scores from the exact Q, the unfolded assembly forward fa_fwdnf_asm_*.)
 * 0 routes every forward to the HIP kernel, 1 (default) lets head dim 128 and 64 take the assembly
 * kernel (FLASH_ATTN_MI355X_FWD_ASM=0 sets 0).  Neither this nor any knob changes a call's
 * numerics contract: whether a call scores from Q' = bf16/f16(scale log2(e) Q) (head dim 64 / 128,
 * no dropout; fp16 only with |scale log2(e)| <= 1) is decided by the call alone, the HIP forward
 * scores from a materialised Q' then, and a backward may run under other settings than its
 * forward. */
void flash_attn_fwd_use_asm(int on);
/* Backward dQ / dK-dV stream overlap: 0 (default) serial on the caller's stream, 1 dQ on a second
 * stream, 2 dQ on a lowest-priority stream, 3 dK/dV on a highest-priority stream
 * (FLASH_ATTN_MI355X_BWD_OVERLAP).  Launches whose dQ kernel computes D itself (knob 8) run dQ then
 * dK/dV on the caller's stream whatever the mode: dK/dV reads what dQ writes. */
void flash_attn_bwd_overlap(int mode);

#ifdef __cplusplus
}
#endif

#endif  /* FLASH_ATTN_MI355X_H_ */
