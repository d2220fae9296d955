// Optional per-launch hipEvent timing (sesa_profile_*), used by bench.py to time the dominant
// kernel class live inside the timed region.
#include <hip/hip_runtime.h>

#include <algorithm>
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

// SESA_DEBUG_ONLY=<k> (diagnostic, tools/fft_stress.py): the network forwards launch only the kernels of class k (the
// others are skipped, so the outputs are garbage) -- which class disturbs work on another stream.
bool debug_skip(int kclass) {
  static const int only = getenv("SESA_DEBUG_ONLY") ? atoi(getenv("SESA_DEBUG_ONLY")) : -1;
  return only >= 0 && kclass != only;
}

void* profile_begin(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on) return nullptr;
  hipEvent_t e = get_event();
  (void)hipEventRecord(e, st);
  return e;
}

void debug_trace_ws(hipStream_t st, int kclass);

void profile_end(void* token, hipStream_t st, int kclass, double work, double bytes) {
  const int dbg = debug_sync_mode();
  if (dbg != -2 && dbg != kclass) (void)hipDeviceSynchronize();
  debug_trace_ws(st, kclass);
  if (!token) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e1 = get_event();
  (void)hipEventRecord(e1, st);
  g_recs.push_back(Rec{kclass, work, bytes, (hipEvent_t)token, e1});
}

// Launch-output checksum trace (diagnostic, tools/streams_trace.py): while a trace buffer is set on this host thread
// (sesa_debug_trace_begin), every instrumented launch is followed, on its own stream, by a kernel adding an
// order-independent 64-bit checksum of the launch's output bytes (sum of word_i * (2 i + 1), wrapping) into the next
// slot of the buffer -- two runs of one forward can then be compared launch by launch.
namespace {
thread_local unsigned long long* t_trace = nullptr;
thread_local int t_trace_cap = 0;
thread_local std::vector<int> t_trace_cls;

__global__ void __launch_bounds__(256) cksum_kernel(const uint32_t* p, int64_t n, unsigned long long* out) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += (unsigned long long)p[i] * (unsigned long long)(2 * i + 1);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}
}  // namespace

thread_local const void* t_range = nullptr;
thread_local size_t t_range_bytes = 0;
void debug_trace_range(const void* p, size_t bytes) {
  t_range = p;
  t_range_bytes = bytes;
}
void debug_trace(hipStream_t st, int kclass, const void* p, size_t bytes);
// every profile_end: the forward's registered range (its workspace), so the first launch after which any byte of it
// differs between two runs is the launch that wrote the difference
void debug_trace_ws(hipStream_t st, int kclass) {
  if (t_trace && t_range) debug_trace(st, kclass, t_range, t_range_bytes);
}

void debug_trace(hipStream_t st, int kclass, const void* p, size_t bytes) {
  if (!t_trace || !p) return;
  const int i = (int)t_trace_cls.size();
  t_trace_cls.push_back(kclass);
  if (i >= t_trace_cap) return;
  const int64_t n = (int64_t)(bytes / 4);
  const unsigned blocks = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(cksum_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(p), n,
                     t_trace + i);
}

}  // namespace sesa

using namespace sesa;

extern "C" int sesa_debug_trace_begin(void* buf, int cap) {
  clear_error();
  SESA_REQUIRE(cap >= 0 && (buf || cap == 0), SESA_ERR_INVALID, "sesa_debug_trace_begin: bad arguments");
  t_trace = reinterpret_cast<unsigned long long*>(buf);
  t_trace_cap = cap;
  t_trace_cls.clear();
  return SESA_OK;
}

extern "C" int sesa_debug_trace_end(int* classes, int cap) {
  const int n = (int)t_trace_cls.size();
  if (classes)
    for (int i = 0; i < n && i < cap; ++i) classes[i] = t_trace_cls[i];
  t_trace = nullptr;
  t_trace_cap = 0;
  t_trace_cls.clear();
  t_range = nullptr;
  t_range_bytes = 0;
  return n;
}

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
