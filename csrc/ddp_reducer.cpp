// Native bucket planner and ready tracker of the DDP engine (the c10d Reducer's C++ role —
// bucket assignment, per-bucket pending counts, in-order launch — next to parallel/ddp.py, which owns the flat
// buffers and issues the RCCL collectives).
//
// Plan (ddp_plan): parameters arrive in backward-ready order, grouped by optimizer region (decay, then no-decay).
// Every parameter is a contiguous slice of ONE flat buffer (offset rounded up to `align` elements); buckets are
// contiguous slices whose boundaries are multiples of `pad_unit` (= world_size x one 4 KiB page of elements), so
// every ZeRO-1 shard is an equal, page-aligned 1/world_size of its bucket. The first bucket closes at
// `first_cap` elements (communication starts early in backward), the others at `cap`; a parameter larger than
// `split_at` is cut at pad-unit-aligned points into ~cap-sized buckets, each of which counts it; the tied weight
// (sparse tied-embedding mode) gets buckets of its own, flagged replicated.
//
// Tracker (ddp_tracker_*): per-bucket pending counts reset before every backward; marking a parameter ready
// decrements every bucket that holds a slice of it and returns the buckets that can launch NOW — strictly in
// index order (a ready bucket waits for its predecessors), so every rank issues the same collective sequence.
// A parameter signalled twice in one backward is an error (it would launch a bucket before its gradients are
// complete).
#include "ddp_reducer_core.h"

#include <c10/util/Exception.h>

#include <memory>
#include <mutex>
#include <vector>

namespace sftamd {

namespace {

std::mutex& mu() {
  static std::mutex m;
  return m;
}
std::vector<std::unique_ptr<reducer::Tracker>>& trackers() {
  static std::vector<std::unique_ptr<reducer::Tracker>> v;
  return v;
}
reducer::Tracker& tracker(int64_t id) {
  TORCH_CHECK(id >= 0 && id < (int64_t)trackers().size() && trackers()[id], "ddp_tracker: bad id ", id);
  return *trackers()[id];
}

template <typename F>
auto guarded(F&& f) -> decltype(f()) {
  try {
    return f();
  } catch (const std::runtime_error& e) {
    TORCH_CHECK(false, e.what());
  }
}

}  // namespace

std::vector<int64_t> ddp_plan(std::vector<int64_t> sizes, std::vector<int64_t> region, int64_t tied, int64_t align,
                              int64_t pad_unit, int64_t cap, int64_t first_cap, int64_t split_at) {
  return guarded([&] { return reducer::plan(sizes, region, tied, align, pad_unit, cap, first_cap, split_at); });
}

int64_t ddp_tracker_create(std::vector<int64_t> owner_ptr, std::vector<int64_t> owners, int64_t n_buckets) {
  auto t = guarded([&] {
    return std::make_unique<reducer::Tracker>(std::move(owner_ptr), std::move(owners), n_buckets);
  });
  std::lock_guard<std::mutex> g(mu());
  trackers().push_back(std::move(t));
  return (int64_t)trackers().size() - 1;
}

void ddp_tracker_reset(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  tracker(id).reset();
}

std::vector<int64_t> ddp_tracker_mark(int64_t id, int64_t param) {
  std::lock_guard<std::mutex> g(mu());
  reducer::Tracker& t = tracker(id);
  return guarded([&] { return t.mark(param); });
}

std::vector<int64_t> ddp_tracker_drain(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  return tracker(id).drain();
}

std::vector<int64_t> ddp_tracker_pending(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  return tracker(id).pending;
}

void ddp_tracker_destroy(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  tracker(id);
  trackers()[id].reset();
}

}  // namespace sftamd
