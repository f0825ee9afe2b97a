// Kernel parameter blocks (passed by value to the kernels) and launcher declarations.
//
// Semantics follow the reference's Qkv_params / Flash_fwd_params / Flash_bwd_params
// (reference csrc/flash_attn/src/flash.h:30-168): element strides, h % h_k == 0 grouping, the
// varlen cu_seqlens convention of BlockInfo (reference block_info.h:11-38) and the padded LSE /
// softmax_d row pitch.  Unlike the reference, every stride and offset is 64-bit (the reference's
// uint32 element offsets are flagged "won't work for arrays > 2GB", flash.h:150-151) so a 288 GB
// HBM3E device can take arbitrarily large shards.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>

namespace fa {

struct AttnShape {
  int b;            // batch (number of sequences for varlen)
  int h;            // query heads
  int hk;           // key/value heads (h % hk == 0)
  int seqlen_q;     // fixed-length seqlen, or max_seqlen_q for varlen
  int seqlen_k;
  int d;            // head dim actually stored (multiple of 8, <= 256)
  int lse_pitch;    // row pitch of softmax_lse / softmax_d per (b, h): seqlen_q (fwd) / rounded (bwd)
  const int* cu_seqlens_q;  // nullptr for fixed-length
  const int* cu_seqlens_k;
  bool varlen_padded_input;  // cu_seqlens give lengths only; rows addressed with batch strides
  bool causal;
  float scale;      // softmax scale
  float scale_log2; // scale * log2(e)
  // dropout (reference Flash_fwd_params p_dropout / p_dropout_in_uint8_t / rp_dropout, flash.h:88-95)
  bool dropout;             // p_dropout > 0
  unsigned keep_u8;         // floor(keep_prob * 255): an element is kept iff its random byte <= this
  float p_keep;             // keep probability 1 - p_dropout
  float rp_dropout;         // 1 / p_keep
  uint64_t philox_seed, philox_offset;   // the reference's (seed, offset) pair (rng_state)
  // backward only: when set, the kernels read (seed, offset) from this device buffer (the rng_state
  // the forward recorded), as the reference's kernels read params.rng_state[0..1]
  // (flash_bwd_kernel.h:783-784) -- no host round trip
  const uint64_t* philox_dev;
  // Paddle dense additive mask (reference Flash_fwd_params attn_mask_ptr / mask_head_mod_size /
  // mask_seq_q_mod_size / unscale_softmax, flash.h; applied in softmax.h:361-379): raw scores
  // QK^T += mask[b][h % mask_h][q % mask_sq][k] * mask_unscale, in the input dtype, row stride
  // mask_row (= seqlen_k).  nullptr: no mask.
  const void* mask;
  int mask_h, mask_sq;
  int64_t mask_row;
  float mask_unscale;
  // FlashMask column-range mask (reference Flash_fwd_params flashmask_*_ptr / h_sparsemask, flash.h;
  // applied in softmax.h:180-298): per (batch, mask head, key) int32 row bounds; fm_lts == nullptr:
  // none.  Causal: LT range [lts, lte) (lte nullptr = to the end).  Non-causal: [lts, lte) and
  // [uts, ute) when uts is given, else rows >= lts or < ute.  See fm_masked (fa_common.h).
  const int* fm_lts;
  const int* fm_lte;
  const int* fm_uts;
  const int* fm_ute;
  int fm_h;
};

struct FwdParams {
  AttnShape s;
  const void* q; const void* k; const void* v; void* o;
  float* lse;
  uint64_t* rng_state;      // if non-null, {seed, offset} is recorded here (reference
  uint64_t seed, offset;    // flash_fwd_kernel.h:321-324 writes it unconditionally)
  int64_t q_batch, q_row, q_head;
  int64_t k_batch, k_row, k_head;
  int64_t v_batch, v_row, v_head;
  int64_t o_batch, o_row, o_head;
  int num_m_blocks;
  int head_group;           // xcd_order_grouped heads per group (0: head-fastest order); launch_fwd
  void* p_out;              // return_softmax (dropout only): S_dmask (b, h, sq_rounded, sk_rounded)
  int p_rows, p_cols;       // sq_rounded, sk_rounded
  // split-KV (launch_fwd decides; decode-shaped calls): workgroup (., split) covers key tiles
  // [split * split_tiles, +split_tiles) and writes fp32 O_i / LSE_i partials, merged by a combine
  // kernel.  o_acc: (n_split, b, h, seqlen_q, acc_d), lse_acc: (n_split, b, h, seqlen_q).
  int n_split, split_tiles, acc_d;
  float* o_acc;
  float* lse_acc;
  // GQA packing on the split-KV path: the pack_g query heads of a kv head become pack_g rows per
  // query (s.h = kv heads, s.seqlen_q = seqlen_q * pack_g), so K/V stream once per kv head.  1: off.
  int pack_g;
};

struct BwdParams {
  AttnShape s;
  const void* q; const void* k; const void* v; const void* o; const void* dout;
  void* dq; void* dk; void* dv;
  const float* lse;
  float* dsum;      // softmax_d: (b, h, seqlen_q_rounded) fp32, D = rowsum(dO * O)
  float* dq_accum;  // caller scratch (reference: (b, h, seqlen_q_rounded, d_rounded) fp32)
  float* lse_s;     // scratch (b, h, seqlen_q_rounded) fp32: -LSE / scale, written by bwd_pre_kernel
                    // (dq_accum when given, else stream-ordered allocation in launch_bwd)
  int64_t q_batch, q_row, q_head;
  int64_t k_batch, k_row, k_head;
  int64_t v_batch, v_row, v_head;
  int64_t o_batch, o_row, o_head;
  int64_t do_batch, do_row, do_head;
  int64_t dq_batch, dq_row, dq_head;
  int64_t dk_batch, dk_row, dk_head;
  int64_t dv_batch, dv_row, dv_head;
  int seqlen_q_rounded;   // pitch of dsum / dq_accum rows
  int d_rounded;          // pitch of dq_accum columns (multiple of 32)
  bool gqa_reduce;        // true: dk/dv have hk heads and the kernel sums the group in-register;
                          // false: dk/dv have h heads (reference "expanded" contract)
  int num_n_blocks;
  int dq_head_group;        // dQ kernel: xcd_order_grouped heads per group (0: head-fastest)
  // assembly dK / dV path (fa_bwd_asm.cpp): (b, h, lsed_ng, 64) fp32 scratch of 32-row groups
  // [-LSE / scale x 32 | -D x 32] written by bwd_pre_kernel instead of lse_s; nullptr: HIP path
  float* lsed;
  int lsed_ng;
  bool fuse_pre;          // (knob 8) the assembly dQ kernel writes D, softmax_d and lsed; dQ before dK/dV
  // dQ = dq_scale dS K.  launch_bwd sets it to the softmax scale, then -- when the call folds
  // (attn_folds_q: the forward held Q as bf16/f16(c Q)) -- scores the backward with that same rounded
  // Q' (q / q_* strides -> a prescaled copy), c -> 1 and scale -> ln 2 (dK = ln2 dS^T Q'), so the
  // recomputed P is the forward's P.
  float dq_scale;
  // (the fold with the fused preprocessing) the assembly dQ kernel, which runs first, converts its Q
  // fragments to bf16/f16(qfold_c Q) itself and stores them here (compact (b | padded rows,
  // seqlen_q, h, d)); the assembly dK/dV kernel then reads Q' from here.  nullptr otherwise.
  void* qfold;
  float qfold_c;
};

// calc_reduced_attn_scores (fa_reduced.hip; reference reduced_scores::Params,
// calc_reduced_attn_scores_kernel.h:14-40): column sums of exp(scale q.k - LSE) per (b, h, key).
struct ReducedParams {
  const void* q; const void* k;
  const float* lse;        // (b, h, sq) fp32
  float* reduced;          // (b, h, sk) fp32, written (not accumulated)
  float* p_out;            // optional (b, h, sq, sk) fp32 probabilities
  int b, h, hk, sq, sk, d;
  float scale;
  int64_t q_batch, q_row, q_head;
  int64_t k_batch, k_row, k_head;
};

// Rotary embedding (fa_rotary.hip; reference csrc/rotary): x, out (b, seqlen, h, >= rotary_dim)
// with element strides and a contiguous last dim; cos / sin (seqlen, rotary_dim / 2), row stride
// cs_row, in the input dtype.
struct RotaryParams {
  const void* x;
  void* out;
  const void* cos;
  const void* sin;
  int b, seqlen, h, rotary_dim;
  int64_t x_batch, x_row, x_head;
  int64_t o_batch, o_row, o_head;
  int64_t cs_row;
};

// Q' = bf16/f16(c Q) in the compact layout (b | padded rows, seqlen_q, h, d): rows at the sequence
// offsets the kernels use (batch b at b seqlen_q h d; varlen at cu_seqlens_q[b] h d), so the
// consumers address it with q_batch = seqlen_q h d, q_row = h d, q_head = d (fa_bwd.hip
// q_fold_kernel; HBM-bound elementwise pass, 16 bytes per thread).
struct QFoldArgs {
  const void* q;
  void* qf;
  int64_t q_batch, q_row, q_head;   // elements
  const int* cu_seqlens_q;
  bool padded;                      // varlen_padded_input
  int b, seqlen_q, h, d;
  float c;
};
void launch_q_fold(const QFoldArgs& a, bool is_bf16, hipStream_t stream);

// The Q fold.  A call "folds" when its scores are computed from Q' = bf16/f16(c Q), c = scale
// log2(e), in the log2 domain (c -> 1, scale -> ln 2): the assembly forward holds Q that way
// (gen_fwd.py FA_GEN_FOLD), and the backward must recompute P from the same Q' or a one-key row's
// P would not be 1.  The decision is a PURE function of the call -- head dim, dtype, scale, dropout,
// masks -- and never of a runtime knob, a stride or the kernel launch_fwd happens to pick: a forward
// that folds but cannot take the assembly kernel (knobs, split-KV, return_softmax, 32-bit record
// limits) runs the HIP kernels on a materialised Q' (launch_q_fold), so forward and backward agree
// whatever switches are flipped between them.  The one process-wide input is
// FLASH_ATTN_MI355X_NO_QFOLD=1, read once at the first call: no call folds, the forward runs the
// unfolded assembly kernels (gen_fwdnf.py) and the backward its c != 1 kernels.
bool attn_folds_q(const AttnShape& s, bool is_bf16);                 // fa_fwd.hip

// Host launchers (fa_fwd.hip / fa_bwd.hip).  Throw std::runtime_error on invalid configuration.
void launch_fwd(const FwdParams& p, bool is_bf16, hipStream_t stream);
// fa_fwd_asm.cpp: the assembly forward (d = 128 or 64, no dropout / mask / split-KV); false when it
// does not apply
bool launch_fwd_asm(const FwdParams& p, bool is_bf16, hipStream_t stream);
bool fwd_asm_applicable(const FwdParams& p, bool is_bf16);           // fa_fwd_asm.cpp
void fwd_asm_enable(int on);
void launch_bwd(const BwdParams& p, bool is_bf16, hipStream_t stream);
void bwd_overlap_enable(int mode);                                  // fa_bwd.hip: dQ / dK-dV stream overlap mode (default 0: off)
bool bwd_asm_applicable(const BwdParams& p);                        // fa_bwd_asm.cpp
void launch_bwd_dkdv_asm(const BwdParams& p, bool is_bf16, hipStream_t stream);
bool dq_asm_applicable(const BwdParams& p, bool fused);                         // fa_bwd_asm.cpp
void launch_bwd_dq_asm(const BwdParams& p, bool is_bf16, hipStream_t stream);
void launch_reduced_scores(const ReducedParams& p, bool is_bf16, hipStream_t stream);
void launch_rotary(const RotaryParams& p, bool interleaved, bool conj, bool is_bf16, hipStream_t stream);

// Tile sizes the launchers use for a given head dim (reported by _get_block_size in Python).
void fwd_block_size(int d, int* block_m, int* block_n);
void bwd_block_size(int d, int* block_m, int* block_n);

// Optional HIP-event timing around each kernel launch (fa_timing.cpp).
enum TimedKernel { kTimeFwd = 0, kTimeBwdPre = 1, kTimeBwdMain = 2 /* dK/dV */, kTimeBwdDq = 3,
                   kTimeBwdBoth = 4 /* dK/dV + dQ window */, kTimeQFold = 5 /* prescaled Q' (launch_bwd) */,
                   kNumTimedKernels = 6 };
void prof_begin(int id, hipStream_t s);
void prof_end(int id, hipStream_t s);

// Test / A-B switches of the launchers (fa_timing.cpp): each is read from its environment variable
// once, at its first use, and can be set later through flash_attn_set_knob (not per launch).
enum Knob { kKnobNoSplitKv = 0 /* FLASH_ATTN_MI355X_NO_SPLITKV: 1 = never split K/V */,
            kKnobNoXcdGroup = 1 /* FLASH_ATTN_MI355X_NO_XCD_GROUP: 1 = head-fastest order */,
            kKnobXcdGroupMinMiB = 2 /* FLASH_ATTN_MI355X_XCD_GROUP_MIN_MIB: grouping threshold */,
            kKnobBwdAsm = 3 /* FLASH_ATTN_MI355X_BWD_ASM: 0 = HIP dK/dV kernel for every call */,
            kKnobDqAsm = 4 /* FLASH_ATTN_MI355X_DQ_ASM: 0 = HIP dQ kernel for every call */,
            kKnobFwdPersist = 5 /* FLASH_ATTN_MI355X_FWD_PERSIST: 0 = assembly forward with one
                                   workgroup per item, 1 = one persistent workgroup per CU */,
            kKnobBwdPersist = 6 /* FLASH_ATTN_MI355X_BWD_PERSIST: the same for the assembly dK/dV and
                                   dQ kernels, fixed length; 2 also varlen dK/dV (device-built list) */,
            kKnobAsmXcdGroupMinMiB = 7 /* FLASH_ATTN_MI355X_ASM_XCD_GROUP_MIN_MIB: knob 2's threshold
                                          for the persistent assembly forward / dQ (default 0) */,
            kKnobFusePre = 8 /* FLASH_ATTN_MI355X_FUSE_PRE: 1 (default) = the assembly dQ kernel computes
                                D and writes softmax_d and the dK/dV scratch itself (no bwd_pre_kernel);
                                dQ runs first.  0 = bwd_pre_kernel, then dK/dV and dQ */,
            kKnobVarlenRounds = 9 /* FLASH_ATTN_MI355X_VARLEN_ROUNDS: items per workgroup of the assembly
                                     dK/dV kernel on varlen calls (default 2, snake-paired
                                     rounds; 1 = one workgroup per item, the dispatcher balancing) */,
            kKnobBwd2W = 10 /* FLASH_ATTN_MI355X_BWD_2W: 1 = the assembly dK/dV kernel with two waves per SIMD
                               (gen_bwd2.py, 8 waves by role; bitwise the same results, 7-8 % slower at C3,
                               DESIGN.md round 6); 0 (default) = one wave per SIMD (gen_bwd.py) */,
            kKnobFwdVarlenRounds = 11 /* FLASH_ATTN_MI355X_FWD_VARLEN_ROUNDS: items per workgroup of the
                                         assembly forward on varlen calls that do not run persistent
                                         (snake-paired rounds: the next item's Q / K / V are issued
                                         under the current one's last steps); 1 = one per item */,
            kNumKnobs = 12 };
int knob(int id);
void set_knob(int id, int value);

// Work order of the assembly kernels, computed in the kernel from the workgroup's item index L (no
// table, no host->device copy, nothing cached per shape: graph-capturable, the reference's launch
// path makes no copies either, flash_bwd_launch_template.h:49-88).  The orders are fa_common.h's:
//   i = L >> xs, lo = L & (2^xs - 1);  gi = i / PG, r = i % PG;  blk = r / HP, hr = r % HP;
//   bh = ((gi HP + hr) << xs) + lo;  bidb = bh / H, head = bh % H;  kvh = head / G
// forward / dQ (xcd_order_grouped, heaviest causal block first): xs = 3, PG = hp nblk, HP = hp when
// the heads group per XCD, else xs = 0, PG = 2^31 - 1, HP = b h (block-major, heads fastest); the
// query block is nblk - 1 - blk.  dK / dV (xcd_order: the key blocks of a head on one XCD):
// xs = 3, PG = nblk, HP = 1 when b h % 8 == 0, else as the forward's head-fastest form; block = blk.
// Each division is a multiply-high by a host-computed magic number, exact for 0 <= n < 2^31
// (Granlund-Montgomery): q = (n * mag) >> sh with sh = 31 + ceil(log2 d), mag = 2^sh / d + 1.
struct MagicDiv {
  uint32_t mag, sh;
};
inline MagicDiv magic_div(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  return {(uint32_t)((1ull << (31 + l)) / d + 1), 31 + l};
}
// kernarg tail of the three assembly kernels (40 bytes; gen_*.py item_decode_ops)
struct ItemDecode {
  uint32_t mag[4];   // PG, HP, H, G
  uint32_t div[4];
  uint32_t shifts;   // sh(PG) | sh(HP) << 8 | sh(H) << 16 | sh(G) << 24
  uint32_t xs_nb1;   // xs | (nblk - 1) << 8
};
static_assert(sizeof(ItemDecode) == 40, "ItemDecode layout");
inline ItemDecode make_item_decode(int xs, uint32_t pg, uint32_t hp, uint32_t h, uint32_t g, int nblk) {
  ItemDecode d;
  const uint32_t dv[4] = {pg, hp, h, g};
  d.shifts = 0;
  for (int i = 0; i < 4; ++i) {
    const MagicDiv m = magic_div(dv[i]);
    d.mag[i] = m.mag;
    d.div[i] = dv[i];
    d.shifts |= m.sh << (8 * i);
  }
  d.xs_nb1 = (uint32_t)xs | ((uint32_t)(nblk - 1) << 8);
  return d;
}
// the forward / dQ order over nbh = b h (query) heads and nblk query blocks, hp heads per XCD group
// (0: head-fastest); the dK / dV order over nbh = b heads_grid and nblk key blocks
inline ItemDecode fwd_item_decode(int nbh, int h, int g, int nblk, int hp) {
  if ((nbh & 7) == 0 && hp > 0 && ((nbh >> 3) % hp) == 0)
    return make_item_decode(3, (uint32_t)hp * (uint32_t)nblk, (uint32_t)hp, (uint32_t)h, (uint32_t)g, nblk);
  return make_item_decode(0, 0x7fffffffu, (uint32_t)nbh, (uint32_t)h, (uint32_t)g, nblk);
}
inline ItemDecode dkdv_item_decode(int nbh, int h_grid, int g, int nblk) {
  if ((nbh & 7) == 0) return make_item_decode(3, (uint32_t)nblk, 1u, (uint32_t)h_grid, (uint32_t)g, nblk);
  return make_item_decode(0, 0x7fffffffu, (uint32_t)nbh, (uint32_t)h_grid, (uint32_t)g, nblk);
}

// Keep blocks freed by hipFreeAsync in the device's default pool across synchronisations, so the
// launchers' per-call scratch (split-KV partials, backward LSE rows, varlen work lists) does not hit
// the driver (once per device).
inline void keep_pool_memory() {
  // (launchers on several host threads: one relaxed flag per device; the attribute set is
  // idempotent, so two threads racing past the check both set the same value)
  static std::atomic<bool> done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || done[dev].load(std::memory_order_relaxed)) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
    uint64_t thr = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  done[dev].store(true, std::memory_order_relaxed);
}

// A stream-ordered scratch allocation, freed on its stream when it leaves scope -- also when a
// launch in between throws.
struct StreamScratch {
  void* p = nullptr;
  hipStream_t s = nullptr;
  StreamScratch() = default;
  StreamScratch(const StreamScratch&) = delete;
  StreamScratch& operator=(const StreamScratch&) = delete;
  ~StreamScratch() {
    if (p != nullptr) (void)hipFreeAsync(p, s);
  }
  // allocates `bytes` on `stream`; false on failure (the caller throws)
  bool alloc(size_t bytes, hipStream_t stream) {
    keep_pool_memory();
    s = stream;
    return hipMallocAsync(&p, bytes, stream) == hipSuccess;
  }
};

// Varlen work lists built on the device (fa_fwd_asm.cpp varlen_items_kernel): stream-ordered
// allocation (in `buf`, freed when it leaves scope) of 2 max_items + 2 dwords, [count, 0, entries...].
bool varlen_items_fit(int b, int nlev);
uint32_t* build_varlen_items(StreamScratch& buf, const int* cu, int b, int nh, int gdiv, int rows, int nlev,
                             bool reverse, long long max_items, hipStream_t stream);

}  // namespace fa
