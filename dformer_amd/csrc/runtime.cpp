// Host-side runtime of libdformer_hip.so: error reporting, ABI version, and the launch tracer
// behind bench.py's per-kernel accounting (which kernels an entry point enqueued, and HIP-event
// durations of chosen kernels measured on the stream they were launched on).
#include <cxxabi.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dformer_hip.h"

static thread_local char g_err[512] = "";

void dfm_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* dfm_last_error(void) { return g_err; }
extern "C" int dfm_abi_version(void) { return 13; }  // 13: DfmGemmDesc.mul2 / out2; 12: dfm_build_tag; 11: dfm_block_fwd / _bwd; 10: dfm_convffn_fwd / _bwd; 9: dfm_nmf_fwd; 8: deferred reduction second stages; 7: DfmGemmDesc.workspace_bytes; 6: dfm_gemm_group
#ifndef DFM_BUILD_TAG
#define DFM_BUILD_TAG "default"
#endif
#ifndef DFM_RED_MIN_ROWS
#define DFM_RED_MIN_ROWS 256
#endif
#ifndef DFM_RED_BLOCKS
#define DFM_RED_BLOCKS 512
#endif
#define DFM_STR2(x) #x
#define DFM_STR(x) DFM_STR2(x)
// names the build a process loaded (variant builds set DFM_BUILD_TAG and the compile-time knobs on the
// make line), so an A/B or diagnostic run records which library it measured
extern "C" const char* dfm_build_tag(void) {
  return DFM_BUILD_TAG " red=" DFM_STR(DFM_RED_BLOCKS) "x" DFM_STR(DFM_RED_MIN_ROWS);
}

// ---------------------------------------------------------------- launch tracer
// dfm_trace_flags is read by DFM_LAUNCH (common.h) before every kernel launch; 0 = tracer off and
// the launch path is one load + branch.
int dfm_trace_flags = 0;

namespace {
struct Timed {
  const void* func;
  hipEvent_t e0, e1;
};
std::mutex g_mu;
std::vector<const void*> g_launched;          // DFM_TRACE_RECORD: kernels since the last take
std::vector<Timed> g_timed;                   // DFM_TRACE_TIME: event pairs awaiting read
std::vector<hipEvent_t> g_pool;               // recycled events
std::unordered_map<const void*, std::string> g_names;
std::vector<std::string> g_probe;             // demangled names to time (empty = every kernel)
hipEvent_t g_open = nullptr;                  // start event of the launch in flight

const std::string& name_of(const void* f) {
  auto it = g_names.find(f);
  if (it != g_names.end()) return it->second;
  const char* mangled = hipKernelNameRefByPtr(f, nullptr);
  std::string out = mangled ? mangled : "?";
  if (mangled) {
    int st = 0;
    char* dm = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
    if (st == 0 && dm) out = dm;
    free(dm);
  }
  return g_names.emplace(f, out).first->second;
}

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

bool timed(const void* f) {
  if (g_probe.empty()) return true;
  const std::string& n = name_of(f);
  for (const std::string& p : g_probe)
    if (n == p) return true;
  return false;
}
}  // namespace

void dfm_trace_pre(const void* func, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (dfm_trace_flags & DFM_TRACE_RECORD) g_launched.push_back(func);
  if ((dfm_trace_flags & DFM_TRACE_TIME) && timed(func)) {
    g_open = take_event();
    (void)hipEventRecord(g_open, s);
  }
}

void dfm_trace_post(const void* func, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_open != nullptr) {
    hipEvent_t e1 = take_event();
    (void)hipEventRecord(e1, s);
    g_timed.push_back({func, g_open, e1});
    g_open = nullptr;
  }
}

extern "C" int dfm_trace_set(int flags, const char* probe_name) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_probe.clear();  // one name, or several separated by '\n'
  for (const char* c = probe_name ? probe_name : ""; *c;) {
    const char* e = strchr(c, '\n');
    const size_t len = e ? (size_t)(e - c) : strlen(c);
    if (len) g_probe.emplace_back(c, len);
    c += len + (e ? 1 : 0);
  }
  g_launched.clear();
  dfm_trace_flags = flags;
  return DFM_OK;
}

extern "C" int dfm_trace_take(const void** funcs, int max) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = (int)g_launched.size();
  for (int i = 0; i < n && i < max; ++i) funcs[i] = g_launched[i];
  g_launched.clear();
  return n;
}

extern "C" int dfm_trace_read(const void** funcs, float* ms, int max) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = (int)g_timed.size();
  if (n > 0) (void)hipEventSynchronize(g_timed.back().e1);
  for (int i = 0; i < n; ++i) {
    if (i < max) {
      float t = 0.f;
      (void)hipEventElapsedTime(&t, g_timed[i].e0, g_timed[i].e1);
      funcs[i] = g_timed[i].func;
      ms[i] = t;
    }
    g_pool.push_back(g_timed[i].e0);
    g_pool.push_back(g_timed[i].e1);
  }
  g_timed.clear();
  return n;
}

extern "C" const char* dfm_kernel_name(const void* func) {
  std::lock_guard<std::mutex> lk(g_mu);
  return name_of(func).c_str();
}
