// Host-side dispatch trace: which kernel variant each op launched (names like "tn.c11", "wgrad.c10", "attn.fwd3"),
// counted while enabled. Tests use it to assert that the SHIPPED default paths run (tests/test_default_path_gpu.py);
// it costs one relaxed atomic load per launch when off.
#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>

#include "cu_budget.h"

namespace sftamd {

static std::atomic<bool> g_trace_on{false};
static std::mutex g_trace_mu;
static std::map<std::string, long> g_trace_counts;

bool trace_on() { return g_trace_on.load(std::memory_order_relaxed); }

void trace_hit(const std::string& name) {
  std::lock_guard<std::mutex> lock(g_trace_mu);
  ++g_trace_counts[name];
}

void dispatch_trace(bool on) {
  std::lock_guard<std::mutex> lock(g_trace_mu);
  if (on) g_trace_counts.clear();
  g_trace_on.store(on, std::memory_order_relaxed);
}

// "name=count;name=count;..." in name order
std::string dispatch_trace_read() {
  std::lock_guard<std::mutex> lock(g_trace_mu);
  std::ostringstream os;
  for (const auto& kv : g_trace_counts) os << kv.first << '=' << kv.second << ';';
  return os.str();
}

// set_cu_budget(n): the CU count the split / hybrid GEMM grids assume (0 = all); returns the effective budget.
int64_t set_cu_budget(int64_t n) {
  if (n < 0 || n > kNumCUs) throw std::invalid_argument("sftamd: set_cu_budget: 0..256");
  cu_budget_slot() = (int)n;
  return cu_budget();
}

}  // namespace sftamd
