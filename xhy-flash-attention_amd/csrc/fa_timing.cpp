// Optional per-kernel timing with HIP events recorded on the launch stream.
//
// Off by default (one branch per launch).  bench.py enables it around its timed region and reads
// the average device duration of each kernel, so the roofline numbers it reports come from the
// kernels themselves rather than from host wall time.  Not for use under graph capture.
#include <hip/hip_runtime.h>

#include <atomic>
#include <climits>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "fa_params.h"

namespace fa {
namespace {

struct Pending { hipEvent_t a, b; int id; };

std::mutex g_mu;
bool g_on = false;
std::vector<Pending> g_pending;
std::vector<hipEvent_t> g_pool;
double g_ms[kNumTimedKernels] = {};
long g_count[kNumTimedKernels] = {};
thread_local hipEvent_t t_start[kNumTimedKernels] = {};   // per id: windows may overlap

hipEvent_t take() {
  if (!g_pool.empty()) { hipEvent_t e = g_pool.back(); g_pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void drain_locked() {
  for (auto& p : g_pending) {
    float ms = 0.f;
    (void)hipEventSynchronize(p.b);
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) { g_ms[p.id] += ms; g_count[p.id] += 1; }
    g_pool.push_back(p.a);
    g_pool.push_back(p.b);
  }
  g_pending.clear();
}

}  // namespace

void prof_begin(int id, hipStream_t s) {
  (void)id;
  if (!g_on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (id < 0 || id >= kNumTimedKernels) return;
  t_start[id] = take();
  (void)hipEventRecord(t_start[id], s);
}

void prof_end(int id, hipStream_t s) {
  if (!g_on || id < 0 || id >= kNumTimedKernels || t_start[id] == nullptr) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e = take();
  (void)hipEventRecord(e, s);
  g_pending.push_back({t_start[id], e, id});
  t_start[id] = nullptr;
  if (g_pending.size() > 4096) drain_locked();
}

}  // namespace fa

extern "C" {

// enable != 0 starts recording (and clears accumulated totals); 0 stops.
void flash_attn_timing_enable(int enable) {
  std::lock_guard<std::mutex> lk(fa::g_mu);
  fa::drain_locked();
  if (enable) {
    for (int i = 0; i < fa::kNumTimedKernels; ++i) { fa::g_ms[i] = 0.0; fa::g_count[i] = 0; }
  }
  fa::g_on = enable != 0;
}

// Total device milliseconds and launch count of kernel `id` since the last enable
// (0 fwd, 1 bwd_pre, 2 bwd_dkdv, 3 bwd_dq, 4 the dK/dV + dQ window: both kernels, which overlap on
// two streams).  Synchronises on the recorded events.
void flash_attn_timing_read(int id, double* total_ms, long* count) {
  std::lock_guard<std::mutex> lk(fa::g_mu);
  fa::drain_locked();
  if (id < 0 || id >= fa::kNumTimedKernels) { *total_ms = 0.0; *count = 0; return; }
  *total_ms = fa::g_ms[id];
  *count = fa::g_count[id];
}

}  // extern "C"

// ---- launcher switches (fa_params.h Knob) ----
namespace fa {
namespace {
struct KnobDef { const char* env; int dflt; };
constexpr KnobDef kKnobs[kNumKnobs] = {{"FLASH_ATTN_MI355X_NO_SPLITKV", 0},
                                       {"FLASH_ATTN_MI355X_NO_XCD_GROUP", 0},
                                       {"FLASH_ATTN_MI355X_XCD_GROUP_MIN_MIB", 256},
                                       {"FLASH_ATTN_MI355X_BWD_ASM", 1},
                                       {"FLASH_ATTN_MI355X_DQ_ASM", 1},
                                       {"FLASH_ATTN_MI355X_FWD_PERSIST", 1},
                                       {"FLASH_ATTN_MI355X_BWD_PERSIST", 1},
                                       {"FLASH_ATTN_MI355X_ASM_XCD_GROUP_MIN_MIB", 0},
                                       {"FLASH_ATTN_MI355X_FUSE_PRE", 1},
                                       {"FLASH_ATTN_MI355X_VARLEN_ROUNDS", 2},
                                       {"FLASH_ATTN_MI355X_BWD_2W", 0},
                                       {"FLASH_ATTN_MI355X_FWD_VARLEN_ROUNDS", 1}};
std::atomic<int> g_knob[kNumKnobs] = {{INT_MIN}, {INT_MIN}, {INT_MIN}, {INT_MIN}, {INT_MIN},
                                      {INT_MIN}, {INT_MIN}, {INT_MIN}, {INT_MIN}, {INT_MIN}, {INT_MIN},
                                      {INT_MIN}};
}  // namespace

int knob(int id) {
  if (id < 0 || id >= kNumKnobs) return 0;
  int v = g_knob[id].load(std::memory_order_relaxed);
  if (v == INT_MIN) {
    const char* e = std::getenv(kKnobs[id].env);
    v = (e != nullptr && *e != 0) ? std::atoi(e) : kKnobs[id].dflt;
    int expect = INT_MIN;
    if (!g_knob[id].compare_exchange_strong(expect, v)) v = expect;
  }
  return v;
}

void set_knob(int id, int value) {
  if (id >= 0 && id < kNumKnobs) g_knob[id].store(value);
}
}  // namespace fa

extern "C" void flash_attn_set_knob(int id, int value) { fa::set_knob(id, value); }
extern "C" int flash_attn_get_knob(int id) { return fa::knob(id); }
