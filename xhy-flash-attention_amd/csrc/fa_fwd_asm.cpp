// Host side of the hand-scheduled assembly forward (csrc/asm/gen_fwd.py -> fa_fwd_asm.s, assembled
// for gfx950 and embedded in this library as a code object).
//
// The kernels cover the headline path: head dim 128 (and 64: C2), bf16 / fp16, causal or not, fixed
// length or varlen (cu_seqlens, varlen_padded_input), GQA, no dropout / mask / return_softmax /
// split-KV.
// Everything else -- and this path when it is switched off -- goes to fwd_kernel (fa_fwd.hip).
//
// Loading: the embedded code object is loaded with hipModuleLoadData once per device (first call),
// and its four kernels are launched with hipModuleLaunchKernel on the caller's stream; kernel
// arguments are one packed struct (FwdAsmArgs, the layout gen_fwd.py's prologue reads).
//
// Work order: the kernel computes each item (batch, head, kv head, query block) from its index in the
// HIP kernel's order (heaviest causal block first, heads fastest, xcd_order_grouped for K/V streams
// beyond the Infinity Cache) with the magic-number divisions of fa_params.h ItemDecode -- no table,
// no host->device copy, nothing cached per shape.  Varlen launches take a list built on the device
// (varlen_items_kernel, below).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "fa_params.h"

extern "C" const unsigned char fa_fwd_asm_co[];
extern "C" const unsigned long fa_fwd_asm_co_size;
extern "C" const unsigned char fa_fwdnf_asm_co[];
extern "C" const unsigned long fa_fwdnf_asm_co_size;

namespace fa {
namespace {

// must match the kernarg loads of gen_fwd.py (K.prologue) and KARG_SIZE
struct FwdAsmArgs {
  const void* q; const void* k; const void* v; void* o; float* lse;
  const uint32_t* sched; const int* cu_q; const int* cu_k;
  uint64_t* rng; uint64_t seed, offset;
  int64_t q_batch, k_batch, v_batch, o_batch;                       // bytes
  int32_t q_row, kv_row, o_row, q_head, k_head, v_head, o_head;    // bytes
  int32_t sq, sk, lse_pitch, h;
  float c;
  int32_t flags;    // bit 0: varlen_padded_input
  int32_t n_items;  // entries of the work table
  int32_t grid;     // workgroups: workgroup w runs items r G + (r odd ? rev(w) : w), r = 0, 1, ...; rev
                    // reverses groups of 8 workgroups when G % 8 == 0 (w keeps its XCD), else G - 1 - w
  int32_t pad;
  ItemDecode dec;   // the work order, computed in the kernel from the item index (flags bit 1 clear)
};
static_assert(sizeof(FwdAsmArgs) == 224 && offsetof(FwdAsmArgs, dec) == 184, "FwdAsmArgs layout");

constexpr int kMaxDev = 64;
struct DevModule {
  hipModule_t mod = nullptr, mod_nf = nullptr;
  hipFunction_t fn[8] = {};   // d 128 then d 64: [bf16 causal, bf16 full, f16 causal, f16 full]
  hipFunction_t fn_nf[8] = {};   // the same without the Q fold (gen_fwdnf.py)
  int cus = 0;
};
std::mutex g_mu;
DevModule g_dev[kMaxDev];
int g_enabled = -1;   // -1: not read yet
void* g_stamps = nullptr;   // flash_attn_debug_fwd_stamps (a generator build with FA_GEN_STAMP=1 writes it)

const char* kNames[8] = {"fa_fwd_asm_d128_bf16_causal", "fa_fwd_asm_d128_bf16_full",
                         "fa_fwd_asm_d128_f16_causal", "fa_fwd_asm_d128_f16_full",
                         "fa_fwd_asm_d64_bf16_causal", "fa_fwd_asm_d64_bf16_full",
                         "fa_fwd_asm_d64_f16_causal", "fa_fwd_asm_d64_f16_full"};
const char* kNamesNf[8] = {"fa_fwdnf_asm_d128_bf16_causal", "fa_fwdnf_asm_d128_bf16_full",
                           "fa_fwdnf_asm_d128_f16_causal", "fa_fwdnf_asm_d128_f16_full",
                           "fa_fwdnf_asm_d64_bf16_causal", "fa_fwdnf_asm_d64_bf16_full",
                           "fa_fwdnf_asm_d64_f16_causal", "fa_fwdnf_asm_d64_f16_full"};

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_fwd (asm path): ") + what + ": " + hipGetErrorString(e));
}

DevModule& module_for(int dev) {
  if (dev < 0 || dev >= kMaxDev) throw std::runtime_error("flash_attn_fwd (asm path): device index out of range");
  DevModule& m = g_dev[dev];
  if (m.mod == nullptr) {
    check(hipModuleLoadData(&m.mod, fa_fwd_asm_co), "hipModuleLoadData");
    for (int i = 0; i < 8; ++i) check(hipModuleGetFunction(&m.fn[i], m.mod, kNames[i]), kNames[i]);
    check(hipModuleLoadData(&m.mod_nf, fa_fwdnf_asm_co), "hipModuleLoadData (no Q fold)");
    for (int i = 0; i < 8; ++i) check(hipModuleGetFunction(&m.fn_nf[i], m.mod_nf, kNamesNf[i]), kNamesNf[i]);
    check(hipDeviceGetAttribute(&m.cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  }
  return m;
}

bool fits32(int64_t x) { return x >= 0 && x < (1ll << 31); }

constexpr int kVarlenMaxSeqs = 4096, kVarlenMaxBlocks = 2048;

// Varlen work lists, built on the device (the host cannot list the items without reading
// cu_seqlens back): the (sequence, block, head) items that hold rows or keys, heaviest first.
// A sequence of len rows has n = ceil(len / rows_per_block) blocks; item levels lev = n-1 .. 0 go
// in descending order across all sequences (the forward / dQ: block = lev, whose causal work grows
// with it; dK / dV (reverse): block = n - 1 - lev, whose causal sweep shrinks with the block index);
// within a level, sequences by block count descending, heads fastest.  out[0] = item count,
// entry i at out[2 + 2 i] = (seq | head << 16, head / gdiv | block << 16) -- the host tables'
// format (the kernels read the count from the first dword, the entries 8 bytes in).
// Shared memory: nb[b] | order[b] | start[nlev + 1] | cur[nlev + 1] | level offset[nlev].
__global__ void __launch_bounds__(1024) varlen_items_kernel(const int* cu, int b, int nh, int gdiv, int rows,
                                                            int nlev, int reverse, uint32_t* out) {
  extern __shared__ int sm[];
  int* nb = sm;
  int* order = nb + b;
  int* start = order + b;
  int* cur = start + nlev + 1;
  int* off = cur + nlev + 1;
  const int t = threadIdx.x, T = blockDim.x;
  for (int i = t; i <= nlev; i += T) start[i] = 0;
  __syncthreads();
  for (int s = t; s < b; s += T) {
    const int len = cu[s + 1] - cu[s];
    int n = len > 0 ? (len + rows - 1) / rows : 0;
    n = n > nlev ? nlev : n;
    nb[s] = n;
    atomicAdd(&start[n], 1);
  }
  __syncthreads();
  if (t == 0) {
    // start[n] = first sorted position of the sequences with nb == n (larger nb first), which is
    // also #{s : nb[s] > n}: the number of sequences present at level n
    int acc = 0;
    for (int n = nlev; n >= 0; --n) { const int c = start[n]; start[n] = acc; cur[n] = acc; acc += c; }
    int total = 0;
    for (int lv = nlev - 1; lv >= 0; --lv) { off[lv] = total; total += nh * start[lv]; }
    out[0] = (uint32_t)total;
    out[1] = 0;
  }
  __syncthreads();
  for (int s = t; s < b; s += T) order[atomicAdd(&cur[nb[s]], 1)] = s;
  __syncthreads();
  const int total = (int)out[0];
  for (int p = t; p < total; p += T) {
    int lo = 0, hi = nlev - 1;      // smallest level with off[level] <= p (off falls as the level grows)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (off[mid] <= p) hi = mid; else lo = mid + 1;
    }
    const int lv = lo, r = p - off[lv], rank = r / nh, head = r - rank * nh;
    const int s = order[rank];
    const int blk = reverse ? nb[s] - 1 - lv : lv;
    out[2 + 2 * p] = (uint32_t)s | ((uint32_t)head << 16);
    out[3 + 2 * p] = (uint32_t)(head / gdiv) | ((uint32_t)blk << 16);
  }
}

}  // namespace

// its shared memory (2 b + 3 (nlev + 1) ints) must stay within the 64 KiB a HIP kernel gets without
// an opt-in attribute
bool varlen_items_fit(int b, int nlev) {
  return b > 0 && nlev > 0 && b <= kVarlenMaxSeqs && nlev <= kVarlenMaxBlocks &&
         (2ll * b + 3ll * (nlev + 1)) * (long long)sizeof(int) <= 65536;
}

uint32_t* build_varlen_items(StreamScratch& buf, const int* cu, int b, int nh, int gdiv, int rows, int nlev,
                             bool reverse, long long max_items, hipStream_t stream) {
  if (!buf.alloc((size_t)(2 * max_items + 2) * sizeof(uint32_t), stream))
    throw std::runtime_error("flash_attn_fwd (asm path): hipMallocAsync (varlen work list) failed");
  uint32_t* tab = static_cast<uint32_t*>(buf.p);
  const size_t shm = (size_t)(2 * b + 3 * (nlev + 1)) * sizeof(int);
  hipLaunchKernelGGL(varlen_items_kernel, dim3(1), dim3(1024), shm, stream, cu, b, nh, gdiv, rows, nlev,
                     reverse ? 1 : 0, tab);
  check(hipGetLastError(), "varlen_items_kernel");
  return tab;
}

void fwd_asm_enable(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_enabled = on ? 1 : 0;
}

// Whether launch_fwd_asm takes a launch (after launch_fwd's split-KV plan).  Also asked by the
// backward (fwd_folds_q): the assembly forward holds Q as bf16/f16(c Q), and a backward of its
// output must compute its scores from the same rounded Q.
bool fwd_asm_applicable(const FwdParams& p, bool is_bf16) {
  const AttnShape& s = p.s;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_enabled < 0) {   // FLASH_ATTN_MI355X_FWD_ASM=0 switches the path off (read once)
      const char* e = std::getenv("FLASH_ATTN_MI355X_FWD_ASM");
      g_enabled = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    if (!g_enabled) return false;
  }
  if ((s.d != 128 && s.d != 64) || s.dropout || s.mask != nullptr || s.fm_lts != nullptr || p.p_out != nullptr ||
      p.n_split != 0 || p.pack_g != 1)
    return false;
  if (p.k_row != p.v_row) return false;   // the K and V DMA share per-lane offsets
  // (the folding kernels hold Q as f16/bf16(c Q), c = scale * log2(e), gen_fwd.py FA_GEN_FOLD; a call
  // attn_folds_q does not fold -- fp16 with |c| > 1, where c Q could overflow, or
  // FLASH_ATTN_MI355X_NO_QFOLD=1 -- takes the unfolded kernels, gen_fwdnf.py: fp32 scores from Q)
  if (s.b > 65535 || s.h > 65535 || p.num_m_blocks > 65535 || s.h % s.hk != 0) return false;
  const int64_t q_row = 2 * p.q_row, kv_row = 2 * p.k_row, o_row = 2 * p.o_row;
  const int64_t q_head = 2 * p.q_head, k_head = 2 * p.k_head, v_head = 2 * p.v_head, o_head = 2 * p.o_head;
  for (int64_t x : {q_row, kv_row, o_row, q_head, k_head, v_head, o_head})
    if (!fits32(x)) return false;
  // K / V records of one (sequence, kv head) and the per-tile offsets must stay below 2^31 bytes
  if (!fits32(((int64_t)s.seqlen_k + 64) * kv_row)) return false;
  if (!fits32((int64_t)256 * (q_row > o_row ? q_row : o_row))) return false;
  const long long nwg = (long long)s.b * s.h * p.num_m_blocks;
  return nwg <= 0x7fffffff;
}

bool launch_fwd_asm(const FwdParams& p, bool is_bf16, hipStream_t stream) {
  if (!fwd_asm_applicable(p, is_bf16)) return false;
  const AttnShape& s = p.s;
  const int64_t q_row = 2 * p.q_row, kv_row = 2 * p.k_row, o_row = 2 * p.o_row;
  const int64_t q_head = 2 * p.q_head, k_head = 2 * p.k_head, v_head = 2 * p.v_head, o_head = 2 * p.o_head;
  int dev = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  const long long nwg = (long long)s.b * s.h * p.num_m_blocks;
  if (nwg <= 0) return true;
  // Persistent grid (knob 5, default on): one workgroup per CU (the kernel's 160 KiB of LDS allows
  // one), each walking the heaviest-first item list in snake order, so the rounds pair heavy and
  // light causal blocks and every item after the first starts with its K/V tiles and Q already
  // issued by its predecessor.  Varlen launches take their list from the device
  // (varlen_items_kernel: the host cannot see cu_seqlens, and a host table would hold the empty
  // blocks past each sequence).  The XCD-grouped order (head_group > 0: a few heads per XCD, their
  // query blocks level by level) runs persistent as well for fixed-length launches.
  hipFunction_t fn;
  int cus = 0;
  const bool persist = knob(kKnobFwdPersist) != 0 && (p.head_group == 0 || s.cu_seqlens_q == nullptr);
  // (the list kernel indexes its entries with int: at most 2^28 items)
  const bool dev_list = persist && s.cu_seqlens_q != nullptr && varlen_items_fit(s.b, p.num_m_blocks) &&
                        nwg <= (1ll << 28);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    DevModule& m = module_for(dev);
    fn = (attn_folds_q(s, is_bf16) ? m.fn : m.fn_nf)[(s.d == 64 ? 4 : 0) + (is_bf16 ? 0 : 2) + (s.causal ? 0 : 1)];
    cus = m.cus;
  }
  StreamScratch vbuf;          // device-built varlen work list (stream-ordered allocation)
  uint32_t* vtab = dev_list ? build_varlen_items(vbuf, s.cu_seqlens_q, s.b, s.h, s.h / s.hk, 256, p.num_m_blocks,
                                                 false, nwg, stream)
                            : nullptr;
  long long grid = nwg;
  if (persist && cus > 0 && nwg > cus && (dev_list || s.cu_seqlens_q == nullptr)) grid = cus;
  // varlen launches that stay one workgroup per item (the XCD-grouped order has no device list):
  // R items per workgroup instead (knob 11) in snake-paired rounds over the decoded order, the
  // dispatcher still balancing the workgroups; G a multiple of 8 keeps each on its XCD's items
  const int rounds = knob(kKnobFwdVarlenRounds);
  if (s.cu_seqlens_q != nullptr && grid == nwg && rounds > 1 && nwg > 8ll * rounds)
    grid = ((nwg + rounds - 1) / rounds + 7) / 8 * 8;
  FwdAsmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.q = p.q; a.k = p.k; a.v = p.v; a.o = p.o; a.lse = p.lse;
  a.sched = vtab;
  a.cu_q = s.cu_seqlens_q; a.cu_k = s.cu_seqlens_k;
  a.rng = p.rng_state; a.seed = p.seed; a.offset = p.offset;
  if (g_stamps != nullptr) a.seed = (uint64_t)(uintptr_t)g_stamps;   // dev stamp build only
  a.q_batch = 2 * p.q_batch; a.k_batch = 2 * p.k_batch; a.v_batch = 2 * p.v_batch; a.o_batch = 2 * p.o_batch;
  a.q_row = (int32_t)q_row; a.kv_row = (int32_t)kv_row; a.o_row = (int32_t)o_row;
  a.q_head = (int32_t)q_head; a.k_head = (int32_t)k_head; a.v_head = (int32_t)v_head; a.o_head = (int32_t)o_head;
  a.sq = s.seqlen_q; a.sk = s.seqlen_k; a.lse_pitch = s.lse_pitch; a.h = s.h;
  a.c = s.scale_log2;
  a.flags = (s.varlen_padded_input ? 1 : 0) | (vtab != nullptr ? 2 : 0);
  a.n_items = (int32_t)nwg;
  a.grid = (int32_t)grid;
  a.dec = fwd_item_decode(s.b * s.h, s.h, s.h / s.hk, p.num_m_blocks, p.head_group);
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  check(hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg), "hipModuleLaunchKernel");
  return true;
}

}  // namespace fa

// Test / A-B hook: 0 routes every forward to fwd_kernel (HIP), 1 lets launch_fwd use the assembly
// kernel where it applies (the default; FLASH_ATTN_MI355X_FWD_ASM=0 sets 0 at the first launch).
extern "C" void flash_attn_fwd_use_asm(int on) { fa::fwd_asm_enable(on); }
// Dev hook: the clock / cycle stamp buffer of a stamp build of the forward (tools/fwd_stamps.py);
// NULL off.  It travels in the `seed` kernarg (the assembly path has no dropout).
extern "C" void flash_attn_debug_fwd_stamps(void* buf) { fa::g_stamps = buf; }
// Test / A-B hook: 0 (default) runs the backward's dQ kernel after dK/dV on the caller's stream,
// 1..3 overlap them on two streams (fa_bwd.hip run_bwd lists the modes).
extern "C" void flash_attn_bwd_overlap(int mode) { fa::bwd_overlap_enable(mode); }
