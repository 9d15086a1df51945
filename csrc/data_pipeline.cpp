// Native (CPU) collation for the SFT data pipeline: right-padding to the
// longest sample (optionally to a multiple of 64 for MFMA-friendly M), HF label semantics
// (pads -> -100), and padding-free packing into varlen streams with cu_seqlens/position_ids.
// Token storage is one flat int32 array + int64 offsets (CSR), so a micro-batch is assembled
// with memcpy-speed loops instead of per-sample Python tensors.
#include <torch/library.h>
#include <ATen/ATen.h>

#include <algorithm>
#include <vector>

namespace sftamd {

static inline int64_t round_up(int64_t x, int64_t m) { return m > 1 ? (x + m - 1) / m * m : x; }

std::tuple<at::Tensor, at::Tensor, at::Tensor> pad_batch(const at::Tensor& tokens, const at::Tensor& offsets,
                                                         const at::Tensor& order, int64_t pad_id, int64_t pad_multiple,
                                                         int64_t max_length) {
  TORCH_CHECK(tokens.scalar_type() == at::kInt && offsets.scalar_type() == at::kLong && order.scalar_type() == at::kLong,
              "pad_batch: tokens int32, offsets/order int64");
  auto tok = tokens.contiguous();
  auto off = offsets.contiguous();
  auto ord = order.contiguous();
  const int32_t* tp = tok.data_ptr<int32_t>();
  const int64_t* op = off.data_ptr<int64_t>();
  const int64_t* orp = ord.data_ptr<int64_t>();
  const int64_t B = ord.numel();
  std::vector<int64_t> lens(B);
  int64_t T = 1;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t i = orp[b];
    int64_t l = op[i + 1] - op[i];
    if (max_length > 0) l = std::min(l, max_length);
    lens[b] = l;
    T = std::max(T, l);
  }
  T = round_up(T, pad_multiple);
  auto ids = at::full({B, T}, pad_id, at::kLong);
  auto labels = at::full({B, T}, -100, at::kLong);
  auto lengths = at::empty({B}, at::kInt);
  int64_t* ip = ids.data_ptr<int64_t>();
  int64_t* lp = labels.data_ptr<int64_t>();
  int32_t* lenp = lengths.data_ptr<int32_t>();
  for (int64_t b = 0; b < B; ++b) {
    const int32_t* src = tp + op[orp[b]];
    for (int64_t t = 0; t < lens[b]; ++t) {
      ip[b * T + t] = src[t];
      lp[b * T + t] = src[t];
    }
    lenp[b] = (int32_t)lens[b];
  }
  return {ids, labels, lengths};
}

// Packs samples (in `order`) into one stream of at most max_tokens tokens. Labels are shifted
// within each sequence (last token of a sequence -> -100). Returns
// (input_ids[M], shifted_labels[M], cu_seqlens[n+1] int32, position_ids[M], n_used[1]).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> pack_sequences(
    const at::Tensor& tokens, const at::Tensor& offsets, const at::Tensor& order, int64_t max_tokens, int64_t pad_id,
    int64_t pad_multiple) {
  TORCH_CHECK(tokens.scalar_type() == at::kInt && offsets.scalar_type() == at::kLong && order.scalar_type() == at::kLong,
              "pack_sequences: tokens int32, offsets/order int64");
  auto tok = tokens.contiguous();
  auto off = offsets.contiguous();
  auto ord = order.contiguous();
  const int32_t* tp = tok.data_ptr<int32_t>();
  const int64_t* op = off.data_ptr<int64_t>();
  const int64_t* orp = ord.data_ptr<int64_t>();
  const int64_t N = ord.numel();
  std::vector<int64_t> cu{0};
  int64_t used = 0, M = 0;
  for (; used < N; ++used) {
    const int64_t i = orp[used];
    int64_t l = op[i + 1] - op[i];
    if (max_tokens > 0) l = std::min(l, max_tokens);
    if (max_tokens > 0 && M + l > max_tokens && used > 0) break;
    M += l;
    cu.push_back(M);
  }
  const int64_t Mp = round_up(std::max<int64_t>(M, 1), pad_multiple);
  auto ids = at::full({Mp}, pad_id, at::kLong);
  auto labels = at::full({Mp}, -100, at::kLong);
  auto pos = at::zeros({Mp}, at::kLong);
  const int64_t nseq = (int64_t)cu.size() - 1 + (Mp > M ? 1 : 0);
  auto cus = at::empty({nseq + 1}, at::kInt);
  int64_t* ip = ids.data_ptr<int64_t>();
  int64_t* lp = labels.data_ptr<int64_t>();
  int64_t* pp = pos.data_ptr<int64_t>();
  int32_t* cp = cus.data_ptr<int32_t>();
  for (int64_t s = 0; s + 1 < (int64_t)cu.size(); ++s) {
    const int32_t* src = tp + op[orp[s]];
    const int64_t b = cu[s], l = cu[s + 1] - cu[s];
    for (int64_t t = 0; t < l; ++t) {
      ip[b + t] = src[t];
      pp[b + t] = t;
      lp[b + t] = (t + 1 < l) ? src[t + 1] : -100;
    }
    cp[s] = (int32_t)cu[s];
  }
  cp[cu.size() - 1] = (int32_t)M;
  if (Mp > M) {  // tail padding is its own (fully ignored) sequence
    for (int64_t t = M; t < Mp; ++t) pp[t] = t - M;
    cp[nseq] = (int32_t)Mp;
  }
  auto n_used = at::full({1}, used, at::kLong);
  return {ids, labels, cus, pos, n_used};
}

TORCH_LIBRARY_IMPL(sftamd, CPU, m) {
  m.impl("pad_batch", &pad_batch);
  m.impl("pack_sequences", &pack_sequences);
}

}  // namespace sftamd
