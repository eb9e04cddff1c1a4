// Kernel timer state (see ktimer.h). Host-only; events are recycled across enable() calls.
#include "ktimer.h"

#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "internal.h"

namespace argus {

thread_local double g_launch_work = 0.0, g_launch_bytes = 0.0;

namespace {
struct Rec {
  std::string name;
  double work, bytes;
  hipEvent_t start, stop;
};
struct Agg {
  int64_t launches = 0;
  double ms = 0.0, work = 0.0, bytes = 0.0;
};
std::mutex g_mu;
std::atomic<bool> g_on{false};
std::string g_filter;
hipStream_t g_stream = nullptr;  // only launches on this stream (nullptr: any)
bool g_any_stream = true;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;  // free events
std::vector<std::pair<std::string, Agg>> g_aggs;

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
void recycle_all() {
  for (auto& r : g_recs) {
    g_pool.push_back(r.start);
    g_pool.push_back(r.stop);
  }
  g_recs.clear();
}
}  // namespace

bool ktimer_wants(const char* name, hipStream_t st) {
  if (!g_on.load(std::memory_order_relaxed)) return false;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_any_stream && st != g_stream) return false;
  return g_filter.empty() || std::strncmp(name, g_filter.c_str(), g_filter.size()) == 0;
}

void ktimer_slot(const char* name, double work, double bytes, hipEvent_t* start, hipEvent_t* stop) {
  std::lock_guard<std::mutex> lk(g_mu);
  Rec r{name, work, bytes, take_event(), take_event()};
  *start = r.start;
  *stop = r.stop;
  g_recs.push_back(r);
}

}  // namespace argus

using namespace argus;

extern "C" {

int argus_ktimer_enable(const char* filter) {
  std::lock_guard<std::mutex> lk(g_mu);
  recycle_all();
  g_aggs.clear();
  g_filter = filter ? filter : "";
  g_any_stream = true;
  g_on = true;
  return ARGUS_OK;
}

int argus_ktimer_enable_on(const char* filter, argus_stream_t stream) {
  const int rc = argus_ktimer_enable(filter);
  std::lock_guard<std::mutex> lk(g_mu);
  g_stream = (hipStream_t)stream;
  g_any_stream = false;
  return rc;
}

int argus_ktimer_disable(void) {
  g_on = false;
  return ARGUS_OK;
}

int argus_ktimer_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::map<std::string, Agg> m;
  for (auto& a : g_aggs) m[a.first] = a.second;
  for (auto& r : g_recs) {
    if (hipEventSynchronize(r.stop) != hipSuccess) {
      set_error("ktimer: event synchronize failed");
      return -1;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.start, r.stop) != hipSuccess) {
      set_error("ktimer: elapsed time unavailable");
      return -1;
    }
    Agg& a = m[r.name];
    a.launches += 1;
    a.ms += ms;
    a.work += r.work;
    a.bytes += r.bytes;
  }
  recycle_all();
  g_aggs.assign(m.begin(), m.end());
  return (int)g_aggs.size();
}

int argus_ktimer_get(int i, char* name, int name_len, int64_t* launches, double* total_ms, double* work,
                     double* bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (i < 0 || i >= (int)g_aggs.size()) {
    set_error("ktimer_get: index out of range (call argus_ktimer_count first)");
    return ARGUS_ERR_ARG;
  }
  const auto& a = g_aggs[i];
  if (name && name_len > 0) {
    std::strncpy(name, a.first.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (launches) *launches = a.second.launches;
  if (total_ms) *total_ms = a.second.ms;
  if (work) *work = a.second.work;
  if (bytes) *bytes = a.second.bytes;
  return ARGUS_OK;
}

}  // extern "C"
