// Host side of the hand-scheduled assembly backward kernels (csrc/asm/gen_bwd.py -> fa_bwd_asm.s for
// dK / dV, csrc/asm/gen_dq.py -> fa_dq_asm.s for dQ; assembled for gfx950 and embedded in this
// library as code objects).
//
// The kernel covers the headline backward: head dim 128, bf16 / fp16, causal or not, fixed length
// or varlen, MHA / GQA (reduced in-kernel over the group, or expanded per query head), no dropout /
// mask / FlashMask.  Head dim 64 has its own dK / dV kernels (round 6, gen_bwd64.py: 4 waves x 64
// keys, each A fragment feeding both 32-key groups' MFMAs, 256-key blocks; C2-class / d64 dK/dV
// -33 to -41 % against bwd_dkdv_kernel, profiles/r06/ab_d64_*_r06g.txt), and so does dQ (gen_dq64.py:
// gen_dq.py's kernel at d = 64, 24 MFMAs a phase, one K and one V DMA piece a wave per subtile).
// It replaces bwd_dkdv_kernel for those calls; bwd_pre_kernel then writes the
// per-row chain starts it streams (-LSE / scale and -D, 32 rows per 256-byte group: the "lsed"
// scratch), and the dQ kernel is unchanged.  Everything else -- and this path when it is switched
// off (FLASH_ATTN_MI355X_BWD_ASM=0 or knob 3) -- runs bwd_dkdv_kernel (fa_bwd.hip).
//
// Work order: each workgroup computes its (batch, head, kv head, 128-key block) from its index in the
// HIP kernel's xcd_order (heaviest causal key block first, the blocks of one head on one XCD) with
// the magic-number divisions of fa_params.h ItemDecode: no table, no host->device copy, nothing
// cached per shape, so a launch is graph-capturable and varlen shapes cost nothing new.
//
// The dQ kernel (same operand coverage; K and V must share their row and batch strides) replaces
// bwd_dq_kernel: 256-row query blocks in the forward's work order (xcd_order_grouped with the
// launcher's dq_head_group, computed in the kernel as above), reading LSE and D (softmax_d) directly.  FLASH_ATTN_MI355X_DQ_ASM=0 (or
// knob 4) keeps bwd_dq_kernel.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "fa_params.h"

extern "C" const unsigned char fa_bwd_asm_co[];
extern "C" const unsigned long fa_bwd_asm_co_size;
extern "C" const unsigned char fa_dq_asm_co[];
extern "C" const unsigned long fa_dq_asm_co_size;
extern "C" const unsigned char fa_dq64_asm_co[];
extern "C" const unsigned long fa_dq64_asm_co_size;
extern "C" const unsigned char fa_bwd2_asm_co[];
extern "C" const unsigned long fa_bwd2_asm_co_size;
extern "C" const unsigned char fa_bwd64_asm_co[];
extern "C" const unsigned long fa_bwd64_asm_co_size;

namespace fa {
namespace {

// must match the kernarg loads of gen_bwd.py (K.prologue) and KARG_SIZE
struct BwdAsmArgs {
  const void* q; const void* k; const void* v; const void* dout; void* dk; void* dv;
  const float* lsed; const uint32_t* sched; const int* cu_q; const int* cu_k;
  int64_t q_batch, k_batch, v_batch, do_batch, dk_batch, dv_batch;     // bytes
  int32_t q_row, k_row, v_row, do_row, dk_row, dv_row;                 // bytes
  int32_t q_head, k_head, v_head, do_head, dk_head, dv_head;           // bytes
  int32_t sq, sk, h, ng, nh, group;
  float c, scale;
  int32_t flags;    // bit 0: varlen_padded_input, bit 1: dK / dV reduced over the GQA group, bit 2: the
                    // items come from the device-built list at sched (count first, entries 8 bytes in)
  int32_t pad;
  void* stamps;     // dev timeline buffer (a generator build with FA_GBW_STAMP=1 writes it), else unused
  ItemDecode dec;   // the work order, computed in the kernel from the item index
  int32_t n_items;  // items (batch x heads x key blocks)
  int32_t grid;     // workgroups: workgroup w runs items r G + (r odd ? rev(w) : w), r = 0, 1, ...
};
static_assert(sizeof(BwdAsmArgs) == 272 && offsetof(BwdAsmArgs, dec) == 224, "BwdAsmArgs layout");

// must match the kernarg loads of gen_dq.py (K.prologue) and KARG_SIZE
struct DqAsmArgs {
  const void* q; const void* k; const void* v; const void* dout; void* dq;
  const float* lse; const float* dsum; const uint32_t* sched; const int* cu_q; const int* cu_k;
  int64_t q_batch, kv_batch, do_batch, dq_batch;                    // bytes
  int32_t q_row, kv_row, do_row, dq_row;                            // bytes
  int32_t q_head, k_head, v_head, do_head, dq_head;                 // bytes
  int32_t sq, sk, lse_pitch, dsum_pitch, h, hk;
  int32_t flags;    // bit 0: varlen_padded_input
  float c, scale;
  ItemDecode dec;   // the work order, computed in the kernel from the item index
  int32_t n_items;  // items (batch x heads x query blocks)
  int32_t grid;     // workgroups (persistent item loop, as BwdAsmArgs)
  // flags bit 1 (BwdParams::fuse_pre): D = rowsum(dO o O) in the kernel, written to dsum and with
  // -LSE / scale to the dK/dV scratch lsed (bwd_pre_kernel's outputs)
  const void* o; int64_t o_batch;                                   // bytes
  int32_t o_row, o_head;                                            // bytes
  float* lsed; int32_t lsed_ng; float nrscale;                      // -1 / scale
  // flags bit 2 (BwdParams::qfold): the kernel converts its Q fragments to bf16/f16(qc Q) -- the
  // forward's rounded Q' -- and stores them to qf (compact rows) for the dK/dV kernel
  void* qf; int64_t qf_batch;                                       // bytes
  int32_t qf_row, qf_head;                                          // bytes
  float qc; int32_t pad2;
};
static_assert(sizeof(DqAsmArgs) == 304 && offsetof(DqAsmArgs, dec) == 184 && offsetof(DqAsmArgs, o) == 232 &&
              offsetof(DqAsmArgs, qf) == 272, "DqAsmArgs layout");

constexpr int kMaxDev = 64;
constexpr int kBkn = 128;   // keys per workgroup (head dim 128)
constexpr int kBkn64 = 256; // head dim 64: 4 waves x 64 keys (gen_bwd64.py)
int bkn_of(int d) { return d == 64 ? kBkn64 : kBkn; }
struct DevModule {
  hipModule_t mod = nullptr, mod_dq = nullptr, mod2 = nullptr, mod64 = nullptr, mod_dq64 = nullptr;
  hipFunction_t fn64[8] = {};    // head dim 64, the order of fn
  hipFunction_t fn[8] = {};      // dK/dV [bf16 causal, bf16 full, f16 causal, f16 full], then the same with c = 1
  hipFunction_t fn2[8] = {};     // the same, two waves per SIMD (gen_bwd2.py, 512 threads)
  hipFunction_t fn_dq[4] = {};   // dQ, the same order
  hipFunction_t fn_dq64[8] = {}; // dQ, head dim 64 (gen_dq64.py): the order of fn (c = 1 kernels last)
  int cus = 0;
};
std::mutex g_mu;
DevModule g_dev[kMaxDev];

// (_c1: P = exp2(S') with no multiply, for launches with c = scale log2(e) = 1 -- the backward of a
// forward that held Q as bf16/f16(c Q), which launch_bwd scores with that Q', c = 1)
const char* kNames[8] = {"fa_bwd_dkdv_asm_d128_bf16_causal", "fa_bwd_dkdv_asm_d128_bf16_full",
                         "fa_bwd_dkdv_asm_d128_f16_causal", "fa_bwd_dkdv_asm_d128_f16_full",
                         "fa_bwd_dkdv_asm_d128_bf16_causal_c1", "fa_bwd_dkdv_asm_d128_bf16_full_c1",
                         "fa_bwd_dkdv_asm_d128_f16_causal_c1", "fa_bwd_dkdv_asm_d128_f16_full_c1"};
const char* kNames2[8] = {"fa_bwd2_dkdv_asm_d128_bf16_causal", "fa_bwd2_dkdv_asm_d128_bf16_full",
                          "fa_bwd2_dkdv_asm_d128_f16_causal", "fa_bwd2_dkdv_asm_d128_f16_full",
                          "fa_bwd2_dkdv_asm_d128_bf16_causal_c1", "fa_bwd2_dkdv_asm_d128_bf16_full_c1",
                          "fa_bwd2_dkdv_asm_d128_f16_causal_c1", "fa_bwd2_dkdv_asm_d128_f16_full_c1"};
const char* kNames64[8] = {"fa_bwd_dkdv_asm_d64_bf16_causal", "fa_bwd_dkdv_asm_d64_bf16_full",
                           "fa_bwd_dkdv_asm_d64_f16_causal", "fa_bwd_dkdv_asm_d64_f16_full",
                           "fa_bwd_dkdv_asm_d64_bf16_causal_c1", "fa_bwd_dkdv_asm_d64_bf16_full_c1",
                           "fa_bwd_dkdv_asm_d64_f16_causal_c1", "fa_bwd_dkdv_asm_d64_f16_full_c1"};
const char* kDqNames[4] = {"fa_bwd_dq_asm_d128_bf16_causal", "fa_bwd_dq_asm_d128_bf16_full",
                           "fa_bwd_dq_asm_d128_f16_causal", "fa_bwd_dq_asm_d128_f16_full"};
const char* kDq64Names[8] = {"fa_bwd_dq_asm_d64_bf16_causal", "fa_bwd_dq_asm_d64_bf16_full",
                             "fa_bwd_dq_asm_d64_f16_causal", "fa_bwd_dq_asm_d64_f16_full",
                             "fa_bwd_dq_asm_d64_bf16_causal_c1", "fa_bwd_dq_asm_d64_bf16_full_c1",
                             "fa_bwd_dq_asm_d64_f16_causal_c1", "fa_bwd_dq_asm_d64_f16_full_c1"};

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_bwd (asm dK/dV): ") + what + ": " + hipGetErrorString(e));
}

DevModule& module_for(int dev) {
  if (dev < 0 || dev >= kMaxDev) throw std::runtime_error("flash_attn_bwd (asm dK/dV): device index out of range");
  DevModule& m = g_dev[dev];
  if (m.mod == nullptr) {
    check(hipModuleLoadData(&m.mod, fa_bwd_asm_co), "hipModuleLoadData");
    for (int i = 0; i < 8; ++i) check(hipModuleGetFunction(&m.fn[i], m.mod, kNames[i]), kNames[i]);
    check(hipModuleLoadData(&m.mod_dq, fa_dq_asm_co), "hipModuleLoadData (dQ)");
    for (int i = 0; i < 4; ++i) check(hipModuleGetFunction(&m.fn_dq[i], m.mod_dq, kDqNames[i]), kDqNames[i]);
    check(hipModuleLoadData(&m.mod_dq64, fa_dq64_asm_co), "hipModuleLoadData (dQ, head dim 64)");
    for (int i = 0; i < 8; ++i) check(hipModuleGetFunction(&m.fn_dq64[i], m.mod_dq64, kDq64Names[i]), kDq64Names[i]);
    check(hipModuleLoadData(&m.mod2, fa_bwd2_asm_co), "hipModuleLoadData (dK/dV, two waves per SIMD)");
    for (int i = 0; i < 8; ++i) check(hipModuleGetFunction(&m.fn2[i], m.mod2, kNames2[i]), kNames2[i]);
    check(hipModuleLoadData(&m.mod64, fa_bwd64_asm_co), "hipModuleLoadData (dK/dV, head dim 64)");
    for (int i = 0; i < 8; ++i) check(hipModuleGetFunction(&m.fn64[i], m.mod64, kNames64[i]), kNames64[i]);
    check(hipDeviceGetAttribute(&m.cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  }
  return m;
}

bool fits32(int64_t x) { return x >= 0 && x < (1ll << 31); }

void* g_stamps = nullptr;   // flash_attn_debug_bwd_stamps

}  // namespace

bool bwd_asm_applicable(const BwdParams& p) {
  const AttnShape& s = p.s;
  if (knob(kKnobBwdAsm) == 0) return false;
  if ((s.d != 128 && s.d != 64) || s.dropout || s.mask != nullptr || s.fm_lts != nullptr) return false;
  if (s.hk <= 0 || s.h % s.hk != 0 || s.b > 65535 || s.h > 65535) return false;
  const int bkn = bkn_of(s.d);
  const int nblk = (s.seqlen_k + bkn - 1) / bkn;
  if (nblk > 65535 || (long long)s.b * s.h * nblk > 0x7fffffffll) return false;
  if ((32ll * ((s.seqlen_q + 31) / 32) + 15) / 16 > 65535) return false;   // bwd_pre_kernel's grid
  for (int64_t x : {p.q_row, p.k_row, p.v_row, p.do_row, p.dk_row, p.dv_row,
                    p.q_head, p.k_head, p.v_head, p.do_head, p.dk_head, p.dv_head})
    if (!fits32(2 * x)) return false;
  // records of one (sequence, head) and the 32-row cursor steps stay below 2^31 bytes
  const int64_t sq = s.seqlen_q + 64, sk = s.seqlen_k + bkn;
  for (int64_t x : {sq * 2 * p.q_row, sq * 2 * p.do_row, sk * 2 * p.k_row, sk * 2 * p.v_row, sk * 2 * p.dk_row,
                    sk * 2 * p.dv_row})
    if (!fits32(x)) return false;
  return true;
}

void launch_bwd_dkdv_asm(const BwdParams& p, bool is_bf16, hipStream_t stream) {
  const AttnShape& s = p.s;
  if (p.lsed == nullptr) throw std::runtime_error("flash_attn_bwd (asm dK/dV): no LSE / D scratch");
  const int nh_grid = p.gqa_reduce ? s.hk : s.h;
  const int bkn = bkn_of(s.d);
  const int nblk = (s.seqlen_k + bkn - 1) / bkn;
  const long long nwg = (long long)s.b * nh_grid * nblk;
  if (nwg <= 0) return;
  int dev = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  hipFunction_t fn;
  int cus = 0;
  // knob 10 (default 0): the kernel with two waves per SIMD, specialised by role (gen_bwd2.py: 8
  // waves, the P waves accumulate dV, the dS waves dK; P crosses in LDS) -- bitwise the same dK / dV,
  // 7-8 % slower at C3 on two boxes; the P exchange costs ~11 % (ablation), its barriers ~2 %
  // (profiles/r06/ab_bwd2_*_r06*.txt)
  const bool two_waves = s.d == 128 && knob(kKnobBwd2W) != 0;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    DevModule& m = module_for(dev);
    const int v = (s.scale_log2 == 1.0f ? 4 : 0) + (is_bf16 ? 0 : 2) + (s.causal ? 0 : 1);
    fn = s.d == 64 ? m.fn64[v] : two_waves ? m.fn2[v] : m.fn[v];
    cus = m.cus;
  }
  // persistent grid (knob 6, default on): one workgroup per CU (151 KiB of LDS allows one) walking the
  // heaviest-first item list in snake order -- no workgroup dispatch between items.  Fixed length;
  // varlen only with knob 6 = 2, from a device-built list (varlen_items_kernel, as the forward: the
  // key blocks of every sequence, heaviest level first, none past a sequence's end).  The
  // dispatcher's dynamic balance over the decoded order (a head's key blocks on one XCD) beats it:
  // C4 dK/dV 2.89 ms one workgroup per item, 3.23 from the list, 3.48 walking the decoded order
  // (profiles/r05/ab_list_c4_r05h.txt, r04/ab_bwd_persist_c4_r04l.txt)
  const bool varlen = s.cu_seqlens_q != nullptr || s.cu_seqlens_k != nullptr;
  const bool dev_list = varlen && knob(kKnobBwdPersist) >= 2 && s.cu_seqlens_k != nullptr &&
                        varlen_items_fit(s.b, nblk) && nwg <= (1ll << 28);
  const bool persist = knob(kKnobBwdPersist) != 0 && (!varlen || dev_list);
  long long grid = (persist && cus > 0 && nwg > cus) ? cus : nwg;
  StreamScratch vbuf;          // device-built varlen work list (stream-ordered allocation)
  uint32_t* vtab = dev_list ? build_varlen_items(vbuf, s.cu_seqlens_k, s.b, nh_grid, p.gqa_reduce ? 1 : s.h / s.hk,
                                                 bkn, nblk, true, nwg, stream)
                            : nullptr;
  // varlen, one workgroup per item: R items per workgroup instead (knob 9, default 2) in snake-paired
  // rounds (item w, then the mirror of w, ...), the dispatcher still balancing the workgroups; G a
  // multiple of 8 keeps each on its XCD's items.  C4 dK/dV -2 % at R = 2
  // (profiles/r05/ab_rounds_c4_r05h.txt)
  const int rounds = knob(kKnobVarlenRounds);
  if (!persist && varlen && rounds > 1 && nwg > 8ll * rounds) grid = ((nwg + rounds - 1) / rounds + 7) / 8 * 8;
  BwdAsmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.q = p.q; a.k = p.k; a.v = p.v; a.dout = p.dout; a.dk = p.dk; a.dv = p.dv;
  a.lsed = p.lsed; a.sched = vtab; a.cu_q = s.cu_seqlens_q; a.cu_k = s.cu_seqlens_k;
  a.q_batch = 2 * p.q_batch; a.k_batch = 2 * p.k_batch; a.v_batch = 2 * p.v_batch;
  int64_t q_row = p.q_row, q_head = p.q_head;
  if (p.qfold != nullptr) {   // the Q' the dQ kernel wrote (it ran first: fused preprocessing)
    a.q = p.qfold;
    a.q_batch = 2ll * s.seqlen_q * s.h * s.d;
    q_row = (int64_t)s.h * s.d; q_head = s.d;
  }
  a.do_batch = 2 * p.do_batch; a.dk_batch = 2 * p.dk_batch; a.dv_batch = 2 * p.dv_batch;
  a.q_row = (int32_t)(2 * q_row); a.k_row = (int32_t)(2 * p.k_row); a.v_row = (int32_t)(2 * p.v_row);
  a.do_row = (int32_t)(2 * p.do_row); a.dk_row = (int32_t)(2 * p.dk_row); a.dv_row = (int32_t)(2 * p.dv_row);
  a.q_head = (int32_t)(2 * q_head); a.k_head = (int32_t)(2 * p.k_head); a.v_head = (int32_t)(2 * p.v_head);
  a.do_head = (int32_t)(2 * p.do_head); a.dk_head = (int32_t)(2 * p.dk_head); a.dv_head = (int32_t)(2 * p.dv_head);
  a.sq = s.seqlen_q; a.sk = s.seqlen_k; a.h = s.h; a.ng = p.lsed_ng;
  a.group = s.h / s.hk;
  a.nh = p.gqa_reduce ? a.group : 1;
  a.c = s.scale_log2; a.scale = s.scale;
  a.flags = (s.varlen_padded_input ? 1 : 0) | (p.gqa_reduce ? 2 : 0) | (vtab != nullptr ? 4 : 0);
  a.stamps = g_stamps;
  a.dec = dkdv_item_decode(s.b * nh_grid, nh_grid, p.gqa_reduce ? 1 : s.h / s.hk, nblk);
  a.n_items = (int32_t)nwg;
  a.grid = (int32_t)grid;
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  check(hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, two_waves ? 512 : 256, 1, 1, 0, stream, nullptr, cfg),
        "hipModuleLaunchKernel");
}

// fused: the kernel also reads O (the fused preprocessing, knob 8): its strides and 256-row records
// must fit as well -- checked only then, so an O layout the kernel never reads does not turn it off
bool dq_asm_applicable(const BwdParams& p, bool fused) {
  const AttnShape& s = p.s;
  if (knob(kKnobDqAsm) == 0) return false;
  if ((s.d != 128 && s.d != 64) || s.dropout || s.mask != nullptr || s.fm_lts != nullptr) return false;
  if (s.hk <= 0 || s.h % s.hk != 0 || s.b > 65535 || s.h > 65535) return false;
  if (p.k_row != p.v_row || p.k_batch != p.v_batch) return false;   // K / V share the DMA offsets
  const int nmb = (s.seqlen_q + 255) / 256;
  if (nmb > 65535 || (long long)s.b * s.h * nmb > 0x7fffffffll) return false;
  for (int64_t x : {p.q_row, p.k_row, p.do_row, p.dq_row, p.q_head, p.k_head, p.v_head, p.do_head, p.dq_head})
    if (!fits32(2 * x)) return false;
  if (fused && (!fits32(2 * p.o_row) || !fits32(2 * p.o_head) || !fits32(256 * 2 * p.o_row))) return false;
  const int64_t sk = s.seqlen_k + 64;
  for (int64_t x : {256 * 2 * p.q_row, 256 * 2 * p.do_row, 256 * 2 * p.dq_row, sk * 2 * p.k_row})
    if (!fits32(x)) return false;
  return true;
}

void launch_bwd_dq_asm(const BwdParams& p, bool is_bf16, hipStream_t stream) {
  const AttnShape& s = p.s;
  const int nmb = (s.seqlen_q + 255) / 256;
  const long long nwg = (long long)s.b * s.h * nmb;
  if (nwg <= 0) return;
  int dev = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  hipFunction_t fn;
  int cus = 0;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    DevModule& m = module_for(dev);
    const int v = (is_bf16 ? 0 : 2) + (s.causal ? 0 : 1);
    fn = s.d == 64 ? m.fn_dq64[v + (s.scale_log2 == 1.0f ? 4 : 0)] : m.fn_dq[v];
    cus = m.cus;
  }
  // persistent grid (knob 6): one workgroup per CU walking the item list in snake order (fixed
  // length only, as dK/dV)
  const bool persist = knob(kKnobBwdPersist) != 0 && s.cu_seqlens_q == nullptr && s.cu_seqlens_k == nullptr;
  // (varlen: one workgroup per query block -- two per workgroup as dK/dV's knob 9 measured C4 dQ
  // 2.151 vs 2.140 ms, profiles/r05/ab_rounds2_c4_r05h.txt)
  const long long grid = (persist && cus > 0 && nwg > cus) ? cus : nwg;
  DqAsmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.q = p.q; a.k = p.k; a.v = p.v; a.dout = p.dout; a.dq = p.dq;
  a.lse = p.lse; a.dsum = p.dsum; a.sched = nullptr; a.cu_q = s.cu_seqlens_q; a.cu_k = s.cu_seqlens_k;
  a.q_batch = 2 * p.q_batch; a.kv_batch = 2 * p.k_batch; a.do_batch = 2 * p.do_batch; a.dq_batch = 2 * p.dq_batch;
  a.q_row = (int32_t)(2 * p.q_row); a.kv_row = (int32_t)(2 * p.k_row); a.do_row = (int32_t)(2 * p.do_row);
  a.dq_row = (int32_t)(2 * p.dq_row);
  a.q_head = (int32_t)(2 * p.q_head); a.k_head = (int32_t)(2 * p.k_head); a.v_head = (int32_t)(2 * p.v_head);
  a.do_head = (int32_t)(2 * p.do_head); a.dq_head = (int32_t)(2 * p.dq_head);
  a.sq = s.seqlen_q; a.sk = s.seqlen_k; a.lse_pitch = s.lse_pitch; a.dsum_pitch = p.seqlen_q_rounded;
  a.h = s.h; a.hk = s.hk;
  a.flags = (s.varlen_padded_input ? 1 : 0) | (p.fuse_pre ? 2 : 0) | (p.qfold != nullptr ? 4 : 0);
  a.c = s.scale_log2; a.scale = p.dq_scale;
  if (p.qfold != nullptr) {
    a.qf = p.qfold;
    a.qf_batch = 2ll * s.seqlen_q * s.h * s.d; a.qf_row = 2 * s.h * s.d; a.qf_head = 2 * s.d;
    a.qc = p.qfold_c;
  }
  a.o = p.o; a.o_batch = 2 * p.o_batch; a.o_row = (int32_t)(2 * p.o_row); a.o_head = (int32_t)(2 * p.o_head);
  a.lsed = p.lsed; a.lsed_ng = p.lsed_ng; a.nrscale = -1.0f / s.scale;
  a.dec = fwd_item_decode(s.b * s.h, s.h, s.h / s.hk, nmb, p.dq_head_group);
  a.n_items = (int32_t)nwg;
  a.grid = (int32_t)grid;
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  check(hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg), "hipModuleLaunchKernel (dQ)");
}

}  // namespace fa

// Dev hook: the timeline buffer of a stamp build of the dK/dV kernel (tools/bwd_stamps.py); NULL off.
extern "C" void flash_attn_debug_bwd_stamps(void* buf) { fa::g_stamps = buf; }
