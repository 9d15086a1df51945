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
#include <c10/util/Exception.h>

#include <cstdint>
#include <mutex>
#include <vector>

namespace sftamd {

namespace {

int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct Tracker {
  std::vector<int64_t> owner_ptr, owners;  // CSR: parameter -> bucket indices
  std::vector<int64_t> init, pending;      // per bucket
  std::vector<uint8_t> ready;
  std::vector<uint8_t> marked;             // per parameter, this backward
  int64_t next = 0;
  bool live = false;
};

std::mutex& mu() {
  static std::mutex m;
  return m;
}
std::vector<Tracker>& trackers() {
  static std::vector<Tracker> v;
  return v;
}
Tracker& tracker(int64_t id) {
  TORCH_CHECK(id >= 0 && id < (int64_t)trackers().size() && trackers()[id].live, "ddp_tracker: bad id ", id);
  return trackers()[id];
}

}  // namespace

// Returns one packed int list:
//   [numel, n_buckets, n_params, n_regions,
//    offset[n_params], bucket_start[n_buckets], bucket_end[n_buckets], bucket_replicated[n_buckets],
//    owner_ptr[n_params + 1], owners[owner_ptr[n_params]], (region_start, region_end, region_decay)[n_regions],
//    n_split_params]
std::vector<int64_t> ddp_plan(std::vector<int64_t> sizes, std::vector<int64_t> region, int64_t tied, int64_t align,
                              int64_t pad_unit, int64_t cap, int64_t first_cap, int64_t split_at) {
  const int64_t np = (int64_t)sizes.size();
  TORCH_CHECK((int64_t)region.size() == np, "ddp_plan: one region flag per parameter");
  TORCH_CHECK(align > 0 && pad_unit > 0 && cap > 0 && first_cap > 0, "ddp_plan: positive sizes");
  TORCH_CHECK(tied >= -1 && tied < np, "ddp_plan: tied index");
  for (int64_t i = 1; i < np; ++i) TORCH_CHECK(region[i] >= region[i - 1], "ddp_plan: parameters grouped by region");
  std::vector<int64_t> offset(np, 0), bstart, bend, brepl, owner_ptr(np + 1, 0), owners, regions;
  std::vector<std::vector<int64_t>> own(np);
  int64_t off = 0, n_split = 0;
  int64_t i = 0;
  while (i < np) {
    const int64_t reg = region[i];
    int64_t j = i;
    while (j < np && region[j] == reg) ++j;
    off = rup(off, pad_unit);
    const int64_t rs = off;
    // open bucket: index cur, start bstart[cur]; params counted in `cur_params`
    auto open = [&](int64_t at) {
      bstart.push_back(at);
      bend.push_back(at);
      brepl.push_back(0);
      return (int64_t)bstart.size() - 1;
    };
    int64_t cur = open(off);
    int64_t cur_params = 0;
    for (int64_t k = i; k < j; ++k) {
      const int64_t sz = rup(sizes[k], align);
      const int64_t limit = cur == 0 ? first_cap : cap;
      if (cur_params > 0 && off + sz - bstart[cur] > limit) {
        off = rup(off, pad_unit);
        bend[cur] = off;
        cur = open(off);
        cur_params = 0;
      }
      offset[k] = off;
      own[k].push_back(cur);
      ++cur_params;
      const int64_t end = off + sz;
      if (split_at > 0 && sz > split_at) {
        ++n_split;
        while (end - bstart[cur] > split_at) {
          const int64_t cut = (bstart[cur] + cap) / pad_unit * pad_unit;
          bend[cur] = cut;
          cur = open(cut);
          own[k].push_back(cur);
          cur_params = 1;
        }
      }
      off = end;
      if (k == tied) {  // buckets of its own: all-reduced early, updated on every rank
        for (int64_t b : own[k]) brepl[b] = 1;
        off = rup(off, pad_unit);
        bend[cur] = off;
        cur = open(off);
        cur_params = 0;
      }
    }
    off = rup(off, pad_unit);
    bend[cur] = off;
    if (cur_params == 0) {  // the bucket opened after a tied weight that ended its region
      bstart.pop_back();
      bend.pop_back();
      brepl.pop_back();
    }
    regions.push_back(rs);
    regions.push_back(off);
    regions.push_back(reg == 0 ? 1 : 0);
    i = j;
  }
  for (int64_t k = 0; k < np; ++k) {
    owner_ptr[k + 1] = owner_ptr[k] + (int64_t)own[k].size();
    owners.insert(owners.end(), own[k].begin(), own[k].end());
  }
  const int64_t nb = (int64_t)bstart.size();
  std::vector<int64_t> out = {off, nb, np, (int64_t)regions.size() / 3};
  out.insert(out.end(), offset.begin(), offset.end());
  out.insert(out.end(), bstart.begin(), bstart.end());
  out.insert(out.end(), bend.begin(), bend.end());
  out.insert(out.end(), brepl.begin(), brepl.end());
  out.insert(out.end(), owner_ptr.begin(), owner_ptr.end());
  out.insert(out.end(), owners.begin(), owners.end());
  out.insert(out.end(), regions.begin(), regions.end());
  out.push_back(n_split);
  return out;
}

int64_t ddp_tracker_create(std::vector<int64_t> owner_ptr, std::vector<int64_t> owners, int64_t n_buckets) {
  TORCH_CHECK(!owner_ptr.empty() && owner_ptr.front() == 0 && owner_ptr.back() == (int64_t)owners.size(),
              "ddp_tracker_create: CSR owner lists");
  Tracker t;
  t.owner_ptr = std::move(owner_ptr);
  t.owners = std::move(owners);
  t.init.assign(n_buckets, 0);
  for (int64_t b : t.owners) {
    TORCH_CHECK(b >= 0 && b < n_buckets, "ddp_tracker_create: bucket index out of range");
    ++t.init[b];
  }
  t.pending = t.init;
  t.ready.assign(n_buckets, 0);
  t.marked.assign(t.owner_ptr.size() - 1, 0);
  t.live = true;
  std::lock_guard<std::mutex> g(mu());
  trackers().push_back(std::move(t));
  return (int64_t)trackers().size() - 1;
}

void ddp_tracker_reset(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  Tracker& t = tracker(id);
  t.pending = t.init;
  std::fill(t.ready.begin(), t.ready.end(), 0);
  std::fill(t.marked.begin(), t.marked.end(), 0);
  t.next = 0;
}

// buckets that launch now (in index order); the launch pointer advances past them
std::vector<int64_t> ddp_tracker_mark(int64_t id, int64_t param) {
  std::lock_guard<std::mutex> g(mu());
  Tracker& t = tracker(id);
  TORCH_CHECK(param >= 0 && param + 1 < (int64_t)t.owner_ptr.size(), "ddp_tracker_mark: parameter index");
  TORCH_CHECK(!t.marked[param], "DDP parameter ", param, " signalled ready twice in one backward");
  t.marked[param] = 1;
  for (int64_t k = t.owner_ptr[param]; k < t.owner_ptr[param + 1]; ++k) {
    const int64_t b = t.owners[k];
    TORCH_CHECK(t.pending[b] > 0, "DDP bucket ", b, ": more ready signals than parameters");
    if (--t.pending[b] == 0) t.ready[b] = 1;
  }
  std::vector<int64_t> launch;
  while (t.next < (int64_t)t.ready.size() && t.ready[t.next]) launch.push_back(t.next++);
  return launch;
}

// the not-yet-launched buckets (after backward: launched regardless of readiness); the pointer moves to the end
std::vector<int64_t> ddp_tracker_drain(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  Tracker& t = tracker(id);
  std::vector<int64_t> rest;
  for (; t.next < (int64_t)t.ready.size(); ++t.next) rest.push_back(t.next);
  return rest;
}

std::vector<int64_t> ddp_tracker_pending(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  return tracker(id).pending;
}

void ddp_tracker_destroy(int64_t id) {
  std::lock_guard<std::mutex> g(mu());
  Tracker& t = tracker(id);
  t = Tracker{};
}

}  // namespace sftamd
