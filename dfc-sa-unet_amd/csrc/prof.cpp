// Per-kernel-class timing hook (HIP events on the launch stream) and library version.
// Used by bench.py to measure the dominant kernel's average launch duration inside the timed
// region without a separate profiler run.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <vector>

#include "dfcsa_internal.h"

namespace {
struct ClassState {
  bool enabled = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  std::vector<double> flops;
};
std::mutex g_mu;
ClassState g_cls[8];

hipEvent_t make_event() {
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

ProfScope::ProfScope(int c, hipStream_t s, double f) : cls(c), st(s), flops(f), on(false) {
  if (c <= 0 || c >= 8) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_cls[c].enabled) return;
  hipEvent_t a = make_event(), b = make_event();
  if (!a || !b) return;
  (void)hipEventRecord(a, st);
  g_cls[c].ev.push_back({a, b});
  g_cls[c].flops.push_back(f);
  on = true;
}

ProfScope::~ProfScope() {
  if (!on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  (void)hipEventRecord(g_cls[cls].ev.back().second, st);
}

extern "C" int dfcsa_prof_enable(int c, int enable) {
  if (c <= 0 || c >= 8) return DFCSA_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  g_cls[c].enabled = enable != 0;
  for (auto& p : g_cls[c].ev) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  g_cls[c].ev.clear();
  g_cls[c].flops.clear();
  return 0;
}

extern "C" int dfcsa_prof_read(int c, double* total_ms, int64_t* launches, double* flops) {
  if (c <= 0 || c >= 8) return DFCSA_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  double t = 0, f = 0;
  for (size_t i = 0; i < g_cls[c].ev.size(); ++i) {
    auto& p = g_cls[c].ev[i];
    (void)hipEventSynchronize(p.second);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.first, p.second);
    t += ms;
    f += g_cls[c].flops[i];
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = (int64_t)g_cls[c].ev.size();
  if (flops) *flops = f;
  return 0;
}

extern "C" const char* dfcsa_version(void) { return "libdfcsa 0.1 gfx950"; }

bool dfcsa_shapelog() {
  static const bool on = std::getenv("DFCSA_SHAPELOG") != nullptr;
  return on;
}
