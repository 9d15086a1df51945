// Fused decode-time sampler for gfx950: repetition penalty -> temperature -> top-k ->
// top-p -> multinomial draw, for one sequence over the full vocabulary, with no host round trip.
//
// The reference's generate() (ask_tuned_model.py:55-65 via HF) runs this as a chain of ~15 eager
// kernels plus a host sync per token (multinomial + .item()). Here it is two launches that can live
// inside the hipGraph of the decode step:
//   partial: grid of 2048-logit tiles, one 256-thread block each; logits read once (bf16 or fp32),
//            penalty from a device presence bitmask (the generated history as a set), scaled by
//            1/temperature, block radix sort (rocPRIM, 8 keys/thread), top K candidates written out;
//   final:   one block merges the <= 4096 candidates (radix sort, 16 keys/thread), then one wave-lane
//            applies softmax over the top K, the top-p cut (a token is dropped once the probability
//            mass ranked above it exceeds top_p — the same rule as inference/generation.py
//            sample_next) and draws with a counter-based uniform (hash of seed and the device step
//            counter, so every graph replay draws fresh). It writes the token to the next step's
//            embedding input, to a device token log, sets the token's presence bit and advances the
//            counters (position, KV length, step) — the decode loop runs replay after replay.
#include "common.h"

#include <rocprim/block/block_radix_sort.hpp>

namespace sftamd {
namespace samp {

constexpr int NT = 256;
constexpr int IPT = 8;                  // keys per thread, partial pass
constexpr int TILE = NT * IPT;          // 2048 logits per block
constexpr int IPT2 = 16;                // keys per thread, final pass (4096 candidates)
constexpr int KMAX = 64;                // top-k supported on the device path

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<u16>(u16 v) { return bf2f(v); }

template <typename T>
__global__ __launch_bounds__(NT) void partial_kernel(const T* __restrict__ logits, int V,
                                                     const unsigned* __restrict__ presence, float inv_temp,
                                                     float penalty, int K, float* __restrict__ cand_v,
                                                     int* __restrict__ cand_i) {
  using Sort = rocprim::block_radix_sort<float, NT, IPT, int>;
  __shared__ typename Sort::storage_type storage;
  float key[IPT];
  int idx[IPT];
  const int base = blockIdx.x * TILE;
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int i = base + j * NT + threadIdx.x;  // striped loads: coalesced
    float x = -INFINITY;
    if (i < V) {
      x = to_f<T>(logits[i]);
      if (penalty != 1.f && ((presence[i >> 5] >> (i & 31)) & 1u)) x = x < 0.f ? x * penalty : x / penalty;
      x *= inv_temp;
    }
    key[j] = x;
    idx[j] = i < V ? i : 0x7fffffff;
  }
  Sort().sort_desc(key, idx, storage);  // blocked result: thread t holds ranks IPT t .. IPT t + IPT - 1
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int r = threadIdx.x * IPT + j;
    if (r < K) {
      cand_v[blockIdx.x * K + r] = key[j];
      cand_i[blockIdx.x * K + r] = idx[j];
    }
  }
}

// state (int64): [0] step counter (RNG), [1] last token, [2] position, [3] KV length (int64 mirror)
__global__ __launch_bounds__(NT) void final_kernel(const float* __restrict__ cand_v, const int* __restrict__ cand_i,
                                                   int ncand, int K, float top_p, int do_sample, unsigned seed,
                                                   long long* __restrict__ state, long long* __restrict__ tok_out,
                                                   long long* __restrict__ pos_out, int* __restrict__ len_out,
                                                   long long* __restrict__ log, int log_cap,
                                                   unsigned* __restrict__ presence) {
  using Sort = rocprim::block_radix_sort<float, NT, IPT2, int>;
  __shared__ typename Sort::storage_type storage;
  __shared__ float top_v[KMAX];
  __shared__ int top_i[KMAX];
  float key[IPT2];
  int idx[IPT2];
#pragma unroll
  for (int j = 0; j < IPT2; ++j) {
    const int c = j * NT + threadIdx.x;
    key[j] = c < ncand ? cand_v[c] : -INFINITY;
    idx[j] = c < ncand ? cand_i[c] : 0x7fffffff;
  }
  Sort().sort_desc(key, idx, storage);
#pragma unroll
  for (int j = 0; j < IPT2; ++j) {
    const int r = threadIdx.x * IPT2 + j;
    if (r < K) {
      top_v[r] = key[j];
      top_i[r] = idx[j];
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const long long step = state[0];
  int tok = top_i[0];
  if (do_sample) {
    const float m = top_v[0];
    float z = 0.f;
    for (int r = 0; r < K; ++r) z += __expf(top_v[r] - m);
    // top-p: keep rank r while the mass ranked above it is <= top_p (rank 0 always kept)
    float above = 0.f, kept = 0.f;
    int n = 0;
    for (; n < K; ++n) {
      if (n > 0 && above > top_p) break;
      const float p = __expf(top_v[n] - m) / z;
      above += p;
      kept += p;
    }
    const unsigned h = hash_u32((unsigned long long)step, seed);
    const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f) * kept;  // uniform in (0, kept)
    float c = 0.f;
    tok = top_i[n - 1];
    for (int r = 0; r < n; ++r) {
      c += __expf(top_v[r] - m) / z;
      if (u <= c) {
        tok = top_i[r];
        break;
      }
    }
  }
  state[0] = step + 1;
  state[1] = tok;
  if (tok_out) tok_out[0] = tok;
  if (log && step < log_cap) log[step] = tok;
  if (pos_out) {  // advance the decode step's position / KV length for the next replay
    const long long p = state[2] + 1;
    state[2] = p;
    pos_out[0] = p;
    state[3] = p + 1;
    len_out[0] = (int)(p + 1);
  }
  atomicOr(presence + (tok >> 5), 1u << (tok & 31));
}

}  // namespace samp

// logits [V] (bf16 or fp32). presence int32 bitmask [ceil(V/32)]. state int64 [4]. tok_out / pos_out int64 [1]
// and len_out int32 [1] are optional (the decode graph's inputs). log int64 [cap] optional.
void sample_token(const at::Tensor& logits, at::Tensor presence, at::Tensor state, const c10::optional<at::Tensor>& tok_out,
                  const c10::optional<at::Tensor>& pos_out, const c10::optional<at::Tensor>& len_out,
                  const c10::optional<at::Tensor>& log, double temperature, int64_t top_k, double top_p,
                  double repetition_penalty, bool do_sample, int64_t seed) {
  SFT_CHECK_CUDA(logits);
  SFT_CHECK(logits.is_contiguous() && (logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16),
            "sample_token: contiguous fp32/bf16 logits");
  const int V = logits.numel();
  SFT_CHECK(presence.scalar_type() == at::kInt && presence.numel() >= (V + 31) / 32 && presence.is_contiguous(),
            "sample_token: presence int32 bitmask");
  SFT_CHECK(state.scalar_type() == at::kLong && state.numel() >= 4, "sample_token: state int64[4]");
  const int K = do_sample ? (int)top_k : 1;
  SFT_CHECK(K >= 1 && K <= samp::KMAX, "sample_token: top_k must be in [1, 64] on the device path");
  const int nblk = (V + samp::TILE - 1) / samp::TILE;
  SFT_CHECK(nblk * K <= samp::NT * samp::IPT2, "sample_token: vocabulary too large for one merge block");
  SFT_CHECK(!pos_out.has_value() || (len_out.has_value() && pos_out->scalar_type() == at::kLong &&
                                     len_out->scalar_type() == at::kInt), "sample_token: pos int64 / len int32");
  auto cv = at::empty({nblk * K}, logits.options().dtype(at::kFloat));
  auto ci = at::empty({nblk * K}, logits.options().dtype(at::kInt));
  const float inv_t = do_sample ? (float)(1.0 / std::max(temperature, 1e-5)) : 1.f;
  if (logits.scalar_type() == at::kFloat)
    samp::partial_kernel<float><<<nblk, samp::NT, 0, cur_stream()>>>(
        logits.data_ptr<float>(), V, (const unsigned*)presence.data_ptr<int>(), inv_t, (float)repetition_penalty, K,
        cv.data_ptr<float>(), ci.data_ptr<int>());
  else
    samp::partial_kernel<u16><<<nblk, samp::NT, 0, cur_stream()>>>(
        (const u16*)logits.data_ptr(), V, (const unsigned*)presence.data_ptr<int>(), inv_t, (float)repetition_penalty,
        K, cv.data_ptr<float>(), ci.data_ptr<int>());
  SFT_LAUNCH_CHECK();
  samp::final_kernel<<<1, samp::NT, 0, cur_stream()>>>(
      cv.data_ptr<float>(), ci.data_ptr<int>(), nblk * K, K, (float)top_p, do_sample ? 1 : 0, (unsigned)seed,
      (long long*)state.data_ptr<int64_t>(), tok_out.has_value() ? (long long*)tok_out->data_ptr<int64_t>() : nullptr,
      pos_out.has_value() ? (long long*)pos_out->data_ptr<int64_t>() : nullptr,
      len_out.has_value() ? len_out->data_ptr<int>() : nullptr,
      log.has_value() ? (long long*)log->data_ptr<int64_t>() : nullptr, log.has_value() ? (int)log->numel() : 0,
      (unsigned*)presence.data_ptr<int>());
  SFT_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) { m.impl("sample_token", &sample_token); }

}  // namespace sftamd
