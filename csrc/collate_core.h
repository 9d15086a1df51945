// Torch-free core of the native collator (csrc/data_pipeline.cpp): plain pointer loops over the CSR token
// store, shared by the torch ops and by the host sanitizer test (tools/debug/collate_sanitize.cpp, built with
// -fsanitize=address,undefined by tests/test_sanitizers_cpu.py — GPU ASan is not available on this pool).
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace sftamd {
namespace collate {

inline int64_t round_up(int64_t x, int64_t m) { return m > 1 ? (x + m - 1) / m * m : x; }

// lengths (truncated at max_length > 0) of the samples in `order`; returns the padded width T >= 1
inline int64_t pad_width(const int64_t* off, const int64_t* order, int64_t B, int64_t max_length,
                         int64_t pad_multiple, std::vector<int64_t>& lens) {
  lens.assign(B, 0);
  int64_t T = 1;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t i = order[b];
    int64_t l = off[i + 1] - off[i];
    if (max_length > 0) l = std::min(l, max_length);
    lens[b] = l;
    T = std::max(T, l);
  }
  return round_up(T, pad_multiple);
}

// ids / labels: [B, T], pre-filled with pad_id / -100 by the caller
inline void pad_fill(const int32_t* tok, const int64_t* off, const int64_t* order, const std::vector<int64_t>& lens,
                     int64_t T, int64_t* ids, int64_t* labels, int32_t* lengths) {
  const int64_t B = (int64_t)lens.size();
  for (int64_t b = 0; b < B; ++b) {
    const int32_t* src = tok + off[order[b]];
    for (int64_t t = 0; t < lens[b]; ++t) {
      ids[b * T + t] = src[t];
      labels[b * T + t] = src[t];
    }
    lengths[b] = (int32_t)lens[b];
  }
}

// packing plan: sequence boundaries cu (size n+1) of the samples that fit max_tokens (>= 1 sample); returns used
inline int64_t pack_plan(const int64_t* off, const int64_t* order, int64_t N, int64_t max_tokens,
                         std::vector<int64_t>& cu) {
  cu.assign(1, 0);
  int64_t used = 0, M = 0;
  for (; used < N; ++used) {
    const int64_t i = order[used];
    int64_t l = off[i + 1] - off[i];
    if (max_tokens > 0) l = std::min(l, max_tokens);
    if (max_tokens > 0 && M + l > max_tokens && used > 0) break;
    M += l;
    cu.push_back(M);
  }
  return used;
}

// ids / labels / pos: [Mp], pre-filled with pad_id / -100 / 0; cus: [nseq + 1] where nseq counts a tail-padding
// pseudo-sequence when Mp > M
inline void pack_fill(const int32_t* tok, const int64_t* off, const int64_t* order, const std::vector<int64_t>& cu,
                      int64_t Mp, int64_t* ids, int64_t* labels, int64_t* pos, int32_t* cus) {
  const int64_t M = cu.back();
  for (int64_t s = 0; s + 1 < (int64_t)cu.size(); ++s) {
    const int32_t* src = tok + off[order[s]];
    const int64_t b = cu[s], l = cu[s + 1] - cu[s];
    for (int64_t t = 0; t < l; ++t) {
      ids[b + t] = src[t];
      pos[b + t] = t;
      labels[b + t] = (t + 1 < l) ? src[t + 1] : -100;
    }
    cus[s] = (int32_t)cu[s];
  }
  const int64_t nreal = (int64_t)cu.size() - 1;
  cus[nreal] = (int32_t)M;
  if (Mp > M) {  // tail padding is its own (fully ignored) sequence
    for (int64_t t = M; t < Mp; ++t) pos[t] = t - M;
    cus[nreal + 1] = (int32_t)Mp;
  }
}

}  // namespace collate
}  // namespace sftamd
