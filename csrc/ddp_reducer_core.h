// Core of the DDP bucket planner and ready tracker (see csrc/ddp_reducer.cpp): plain C++17, no torch, so the host
// sanitizer driver (tools/debug/reducer_sanitize.cpp) builds it with -fsanitize=address,undefined. Errors throw
// std::runtime_error; the op wrappers turn them into c10::Error (Python RuntimeError).
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace sftamd {
namespace reducer {

inline void require(bool ok, const std::string& msg) {
  if (!ok) throw std::runtime_error(msg);
}

inline int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Packed result:
//   [numel, n_buckets, n_params, n_regions,
//    offset[n_params], bucket_start[n_buckets], bucket_end[n_buckets], bucket_replicated[n_buckets],
//    owner_ptr[n_params + 1], owners[owner_ptr[n_params]], (region_start, region_end, region_decay)[n_regions],
//    n_split_params]
inline std::vector<int64_t> plan(const std::vector<int64_t>& sizes, const std::vector<int64_t>& region, int64_t tied,
                                 int64_t align, int64_t pad_unit, int64_t cap, int64_t first_cap, int64_t split_at) {
  const int64_t np = (int64_t)sizes.size();
  require((int64_t)region.size() == np, "ddp_plan: one region flag per parameter");
  require(align > 0 && pad_unit > 0 && cap > 0 && first_cap > 0, "ddp_plan: positive sizes");
  require(tied >= -1 && tied < np, "ddp_plan: tied index");
  for (int64_t i = 0; i < np; ++i) require(sizes[i] >= 0, "ddp_plan: negative parameter size");
  for (int64_t i = 1; i < np; ++i) require(region[i] >= region[i - 1], "ddp_plan: parameters grouped by region");
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

struct Tracker {
  std::vector<int64_t> owner_ptr, owners;  // CSR: parameter -> bucket indices
  std::vector<int64_t> init, pending;      // per bucket
  std::vector<uint8_t> ready;
  std::vector<uint8_t> marked;             // per parameter, this backward
  int64_t next = 0;

  Tracker(std::vector<int64_t> ptr, std::vector<int64_t> own, int64_t n_buckets)
      : owner_ptr(std::move(ptr)), owners(std::move(own)) {
    require(n_buckets >= 0, "ddp_tracker_create: bucket count");
    require(!owner_ptr.empty() && owner_ptr.front() == 0 && owner_ptr.back() == (int64_t)owners.size(),
            "ddp_tracker_create: CSR owner lists");
    for (size_t k = 1; k < owner_ptr.size(); ++k)
      require(owner_ptr[k] >= owner_ptr[k - 1], "ddp_tracker_create: CSR pointers non-decreasing");
    init.assign(n_buckets, 0);
    for (int64_t b : owners) {
      require(b >= 0 && b < n_buckets, "ddp_tracker_create: bucket index out of range");
      ++init[b];
    }
    marked.assign(owner_ptr.size() - 1, 0);
    reset();
  }

  void reset() {
    pending = init;
    ready.assign(init.size(), 0);
    std::fill(marked.begin(), marked.end(), 0);
    next = 0;
  }

  // buckets that launch now (in index order); the launch pointer advances past them
  std::vector<int64_t> mark(int64_t param) {
    require(param >= 0 && param + 1 < (int64_t)owner_ptr.size(), "ddp_tracker_mark: parameter index");
    require(!marked[param], "DDP parameter " + std::to_string(param) + " signalled ready twice in one backward");
    marked[param] = 1;
    for (int64_t k = owner_ptr[param]; k < owner_ptr[param + 1]; ++k) {
      const int64_t b = owners[k];
      require(pending[b] > 0, "DDP bucket " + std::to_string(b) + ": more ready signals than parameters");
      if (--pending[b] == 0) ready[b] = 1;
    }
    std::vector<int64_t> launch;
    while (next < (int64_t)ready.size() && ready[next]) launch.push_back(next++);
    return launch;
  }

  // the not-yet-launched buckets (after backward: launched regardless of readiness); the pointer moves to the end
  std::vector<int64_t> drain() {
    std::vector<int64_t> rest;
    for (; next < (int64_t)ready.size(); ++next) rest.push_back(next);
    return rest;
  }
};

}  // namespace reducer
}  // namespace sftamd
