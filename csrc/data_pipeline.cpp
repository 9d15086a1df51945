// Native (CPU) collation for the SFT data pipeline: right-padding to the
// longest sample (optionally to a multiple of 64 for MFMA-friendly M), HF label semantics
// (pads -> -100), and padding-free packing into varlen streams with cu_seqlens/position_ids.
// Token storage is one flat int32 array + int64 offsets (CSR), so a micro-batch is assembled
// with memcpy-speed loops instead of per-sample Python tensors. The loops live in collate_core.h
// (torch-free, also built under host ASan/UBSan by tests/test_sanitizers_cpu.py).
#include <torch/library.h>
#include <ATen/ATen.h>

#include "collate_core.h"

namespace sftamd {

std::tuple<at::Tensor, at::Tensor, at::Tensor> pad_batch(const at::Tensor& tokens, const at::Tensor& offsets,
                                                         const at::Tensor& order, int64_t pad_id, int64_t pad_multiple,
                                                         int64_t max_length) {
  TORCH_CHECK(tokens.scalar_type() == at::kInt && offsets.scalar_type() == at::kLong && order.scalar_type() == at::kLong,
              "pad_batch: tokens int32, offsets/order int64");
  auto tok = tokens.contiguous();
  auto off = offsets.contiguous();
  auto ord = order.contiguous();
  const int64_t B = ord.numel();
  std::vector<int64_t> lens;
  const int64_t T = collate::pad_width(off.data_ptr<int64_t>(), ord.data_ptr<int64_t>(), B, max_length, pad_multiple,
                                       lens);
  auto ids = at::full({B, T}, pad_id, at::kLong);
  auto labels = at::full({B, T}, -100, at::kLong);
  auto lengths = at::empty({B}, at::kInt);
  collate::pad_fill(tok.data_ptr<int32_t>(), off.data_ptr<int64_t>(), ord.data_ptr<int64_t>(), lens, T,
                    ids.data_ptr<int64_t>(), labels.data_ptr<int64_t>(), lengths.data_ptr<int32_t>());
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
  std::vector<int64_t> cu;
  const int64_t used = collate::pack_plan(off.data_ptr<int64_t>(), ord.data_ptr<int64_t>(), ord.numel(), max_tokens, cu);
  const int64_t M = cu.back();
  const int64_t Mp = collate::round_up(std::max<int64_t>(M, 1), pad_multiple);
  auto ids = at::full({Mp}, pad_id, at::kLong);
  auto labels = at::full({Mp}, -100, at::kLong);
  auto pos = at::zeros({Mp}, at::kLong);
  const int64_t nseq = (int64_t)cu.size() - 1 + (Mp > M ? 1 : 0);
  auto cus = at::empty({nseq + 1}, at::kInt);
  collate::pack_fill(tok.data_ptr<int32_t>(), off.data_ptr<int64_t>(), ord.data_ptr<int64_t>(), cu, Mp,
                     ids.data_ptr<int64_t>(), labels.data_ptr<int64_t>(), pos.data_ptr<int64_t>(),
                     cus.data_ptr<int32_t>());
  auto n_used = at::full({1}, used, at::kLong);
  return {ids, labels, cus, pos, n_used};
}

TORCH_LIBRARY_IMPL(sftamd, CPU, m) {
  m.impl("pad_batch", &pad_batch);
  m.impl("pack_sequences", &pack_sequences);
}

}  // namespace sftamd
