// Optional per-launch hipEvent timing (sesa_profile_*), used by bench.py to time the dominant
// kernel class live inside the timed region.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_internal.hpp"

namespace sesa {
namespace {
struct Rec {
  int kclass;
  double work;   // algorithmic FLOPs (MFMA / VALU classes) or bytes (streaming classes)
  double bytes;  // algorithmic HBM bytes of a compute-class launch (its operands read once, results written once)
  hipEvent_t e0, e1;
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
}  // namespace

bool profiling() { return g_on; }

// SESA_DEBUG_SYNC (diagnostic, tools/streams_bisect.py): "all" -- hipDeviceSynchronize after every libsesa launch,
// so no two launches ever run concurrently; "except:<k>" -- after every launch except those of kernel class k, so
// only class k's launches overlap work on other streams.  Unset: nothing.
namespace {
int debug_sync_mode() {   // -2 off, -1 all, k >= 0 all but class k
  static const int v = [] {
    const char* e = getenv("SESA_DEBUG_SYNC");
    if (!e) return -2;
    if (std::string(e) == "all") return -1;
    if (std::string(e).rfind("except:", 0) == 0) return atoi(e + 7);
    return -2;
  }();
  return v;
}
}  // namespace

void* profile_begin(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on) return nullptr;
  hipEvent_t e = get_event();
  (void)hipEventRecord(e, st);
  return e;
}

void profile_end(void* token, hipStream_t st, int kclass, double work, double bytes) {
  const int dbg = debug_sync_mode();
  if (dbg != -2 && dbg != kclass) (void)hipDeviceSynchronize();
  if (!token) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e1 = get_event();
  (void)hipEventRecord(e1, st);
  g_recs.push_back(Rec{kclass, work, bytes, (hipEvent_t)token, e1});
}

}  // namespace sesa

using namespace sesa;

extern "C" int sesa_profile_enable(int enable) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (enable) {
    for (auto& r : g_recs) {
      g_pool.push_back(r.e0);
      g_pool.push_back(r.e1);
    }
    g_recs.clear();
  }
  g_on = enable != 0;
  return SESA_OK;
}

extern "C" int sesa_profile_read(int kclass, double* total_ms, int64_t* launches, double* total_work) {
  return sesa_profile_read2(kclass, total_ms, launches, total_work, nullptr);
}

extern "C" int sesa_profile_read2(int kclass, double* total_ms, int64_t* launches, double* total_work,
                                  double* total_bytes) {
  clear_error();
  std::lock_guard<std::mutex> lk(g_mu);
  double ms = 0, work = 0, bytes = 0;
  int64_t n = 0;
  for (auto& r : g_recs) {
    if (r.kclass != kclass) continue;
    SESA_CHECK_HIP(hipEventSynchronize(r.e1));
    float t = 0;
    SESA_CHECK_HIP(hipEventElapsedTime(&t, r.e0, r.e1));
    ms += t;
    work += r.work;
    bytes += r.bytes;
    ++n;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = n;
  if (total_work) *total_work = work;
  if (total_bytes) *total_bytes = bytes;
  return SESA_OK;
}

// Sum over the class's launches of each launch's roofline floor, max(work / peak FLOP rate, bytes / peak HBM rate), in
// ms: the time the class would take if every launch ran at the bound of its own arithmetic intensity (a class mixes
// launches on both sides of the ridge, so this is tighter than the floor of the summed work and bytes).
extern "C" int sesa_profile_floor(int kclass, double peak_tflops, double peak_gbs, double* floor_ms) {
  clear_error();
  SESA_REQUIRE(floor_ms && peak_tflops > 0 && peak_gbs > 0, SESA_ERR_INVALID, "sesa_profile_floor: bad arguments");
  std::lock_guard<std::mutex> lk(g_mu);
  double f = 0;
  for (auto& r : g_recs) {
    if (r.kclass != kclass) continue;
    const double tc = r.work / (peak_tflops * 1e12), tm = r.bytes / (peak_gbs * 1e9);
    f += (tc > tm ? tc : tm) * 1e3;
  }
  *floor_ms = f;
  return SESA_OK;
}
