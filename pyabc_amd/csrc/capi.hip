// Library-wide C-ABI plumbing: error reporting, version, tuning knobs.
#include <atomic>
#include <climits>
#include <cstdarg>
#include <cstdlib>
#include <mutex>

#include "common.hpp"

namespace abc {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {
constexpr const char* kKnobNames[kKnobCount] = {
    "ABC_KDE_MFMA_SPLIT", "ABC_KDE_MFMA_IB",   "ABC_KDE_MFMA_PIPE",
    "ABC_KDE_MFMA_LDS2",  "ABC_KDE_MFMA_SMAJOR", "ABC_KDE_TIER",
    "ABC_LZ_IB",          "ABC_LZ_TPB",          "ABC_KNN_ROWS",
    "ABC_KDE_PARENT_SHIFT", "ABC_KDE_PARENT_WIN", "ABC_PROPOSE_GROUP"};
std::atomic<int> g_knobs[kKnobCount];
std::once_flag g_knobs_once;

void load_knobs() {
  for (int k = 0; k < kKnobCount; ++k) {
    const char* e = getenv(kKnobNames[k]);
    g_knobs[k].store(e ? atoi(e) : INT_MIN, std::memory_order_relaxed);
  }
}
}  // namespace

int tuning_knob(Knob k, int dflt) {
  std::call_once(g_knobs_once, load_knobs);
  const int v = g_knobs[k].load(std::memory_order_relaxed);
  return v == INT_MIN ? dflt : v;
}
}  // namespace abc

extern "C" {
void abc_tuning_reload(void) {
  std::call_once(abc::g_knobs_once, [] {});
  abc::load_knobs();
}
const char* abc_last_error(void) { return abc::g_err; }
// Load every unit's code object on the current device up front; returns the
// number of units that failed to resolve (0 on a GPU).
int abc_preload(void) {
  return abc::preload_propose() + abc::preload_kde() + abc::preload_kde_mfma() +
         abc::preload_distance() + abc::preload_select() + abc::preload_stochastic() +
         abc::preload_local() + abc::preload_local_pdf32() + abc::preload_local_mfma() +
         abc::preload_sort();
}
int abc_version(void) { return 10000; }  // 0.1.0
}
