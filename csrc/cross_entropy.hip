// Fused cross-entropy over a 128k vocabulary for gfx950.
//
// One 256-thread block per token row. Pass 1 streams the bf16 logits row once with 16-byte
// loads and keeps an online (max, sum e^(x-max), sum e^(x-max)*x, argmax) per thread; the
// block combines them to get logsumexp, the per-token loss, the entropy and the argmax
// accuracy bit (the TRL training metrics, at no extra pass). Pass 2 re-reads the row (L2 /
// Infinity-Cache resident: the launch caps the rows in flight, see ce_fwd) and overwrites it IN PLACE with the bf16 gradient
// (softmax - onehot) * (1/num_items_in_batch): fp32 logits are never materialised.
#include "common.h"

#include <climits>
#include <cstdlib>

namespace sftamd {

struct CEAcc {
  float m, s, t;  // running max, sum exp(x-m), sum exp(x-m)*x
  float bv;       // best value
  int bi;         // best index (first occurrence)
};

__device__ __forceinline__ void ce_merge(CEAcc& a, const CEAcc& b) {
  const float M = fmaxf(a.m, b.m);
  const float ea = (a.m == -INFINITY) ? 0.f : __expf(a.m - M);
  const float eb = (b.m == -INFINITY) ? 0.f : __expf(b.m - M);
  a.s = a.s * ea + b.s * eb;
  a.t = a.t * ea + b.t * eb;
  a.m = M;
  if (b.bv > a.bv || (b.bv == a.bv && b.bi < a.bi)) {
    a.bv = b.bv;
    a.bi = b.bi;
  }
}

template <int CE_U>  // row loads in flight per thread
__global__ __launch_bounds__(256) void ce_fwd_kernel(u16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                     const float* __restrict__ inv_count, float* __restrict__ stats,
                                                     int M, int V, int write_grad) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  u16* lr = logits + (long)row * V;
  const long label = labels[row];
  SFT_DASSERT(label == -100 || (label >= 0 && label < V));
  const bool valid = label >= 0 && label < V;
  const int nvec = V / 8;

  CEAcc acc{-INFINITY, 0.f, 0.f, -INFINITY, INT_MAX};
  auto accum = [&](const uint4& raw, int v) {
    float x[8];
    unpack8(raw, x);
    float mx = x[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) mx = fmaxf(mx, x[i]);
    CEAcc b{mx, 0.f, 0.f, -INFINITY, INT_MAX};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float e = __expf(x[i] - mx);
      b.s += e;
      b.t += e * x[i];
      if (x[i] > b.bv) {
        b.bv = x[i];
        b.bi = v * 8 + i;
      }
    }
    ce_merge(acc, b);
  };
  // U independent 16-byte loads in flight per thread before any of them is consumed: one load per iteration
  // leaves the row stream latency-bound (~3.5 TB/s); ties in the argmax resolve by index in ce_merge, so the
  // visiting order does not change the result
  int v = tid;
  for (; v + 256 * (CE_U - 1) < nvec; v += 256 * CE_U) {
    uint4 r[CE_U];
#pragma unroll
    for (int u = 0; u < CE_U; ++u) r[u] = *(const uint4*)(lr + (long)(v + 256 * u) * 8);
#pragma unroll
    for (int u = 0; u < CE_U; ++u) accum(r[u], v + 256 * u);
  }
  for (; v < nvec; v += 256) accum(*(const uint4*)(lr + (long)v * 8), v);
  // wave reduce
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    CEAcc b;
    b.m = __shfl_xor(acc.m, o, 64);
    b.s = __shfl_xor(acc.s, o, 64);
    b.t = __shfl_xor(acc.t, o, 64);
    b.bv = __shfl_xor(acc.bv, o, 64);
    b.bi = __shfl_xor(acc.bi, o, 64);
    ce_merge(acc, b);
  }
  __shared__ CEAcc red[4];
  __shared__ float sh_lse;
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    CEAcc a = red[0];
    for (int w = 1; w < 4; ++w) ce_merge(a, red[w]);
    const float lse = a.m + __logf(a.s);
    const float xl = valid ? bf2f(lr[label]) : 0.f;
    stats[row] = valid ? (lse - xl) : 0.f;
    stats[M + row] = lse;
    stats[2 * M + row] = lse - a.t / a.s;
    stats[3 * M + row] = (valid && a.bi == label) ? 1.f : 0.f;
    sh_lse = lse;
  }
  __syncthreads();
  if (!write_grad) return;
  const float lse = sh_lse;
  const float scale = valid ? inv_count[0] : 0.f;
  auto grad = [&](const uint4& raw, int v) {
    float x[8];
    unpack8(raw, x);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float p = __expf(x[i] - lse);
      x[i] = (p - ((v * 8 + i) == label ? 1.f : 0.f)) * scale;
    }
    *(uint4*)(lr + (long)v * 8) = pack8(x);
  };
  v = tid;
  for (; v + 256 * (CE_U - 1) < nvec; v += 256 * CE_U) {
    uint4 r[CE_U];
#pragma unroll
    for (int u = 0; u < CE_U; ++u) r[u] = *(const uint4*)(lr + (long)(v + 256 * u) * 8);
#pragma unroll
    for (int u = 0; u < CE_U; ++u) grad(r[u], v + 256 * u);
  }
  for (; v < nvec; v += 256) grad(*(const uint4*)(lr + (long)v * 8), v);
}

at::Tensor ce_fwd(at::Tensor logits, const at::Tensor& labels, const at::Tensor& inv_count, bool write_grad) {
  SFT_CHECK_BF16(logits);
  SFT_CHECK_CONTIG(logits);
  SFT_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  SFT_CHECK(inv_count.scalar_type() == at::kFloat && inv_count.is_cuda(), "inv_count must be a fp32 GPU tensor");
  const int V = logits.size(-1);
  const int M = logits.numel() / V;
  SFT_CHECK(V % 8 == 0, "vocab must be a multiple of 8");
  SFT_CHECK(labels.numel() == M, "labels size");
  auto lab = labels.contiguous();
  auto stats = at::empty({4, M}, logits.options().dtype(at::kFloat));
  if (M == 0) return stats;
  auto* lg = (u16*)logits.data_ptr();
  // Pass 2 re-reads the row from the Infinity Cache only while the rows in flight fit it: with 8 blocks per CU the
  // SmolLM3 bench's 2048 rows x 256 KB = 512 MB of rows in flight overflow the 256 MB cache and pass 2 goes back to HBM.
  // With the gradient written, cap the blocks per CU so the rows in flight stay near 200 MB by reserving dynamic LDS
  // (nothing is stored in it): 3 blocks per CU at V = 128,256 — 1.037 vs 1.227 ms per call at 8192 rows
  // (tools/bench_ce.py, profiles/r6_memory_kernels.md); the stats-only pass (eval) keeps full occupancy.
  int pad = 0;
  if (write_grad) {
    const long row_bytes = (long)V * 2;
    const long bpc = std::max(1L, std::min(8L, (200L << 20) / ((long)num_cus() * row_bytes)));
    if (bpc < 8) pad = (int)((160L * 1024) / bpc - 1024);
  }
    ce_fwd_kernel<4><<<M, 256, pad, cur_stream()>>>(lg, lab.data_ptr<int64_t>(), inv_count.data_ptr<float>(),
                                                  stats.data_ptr<float>(), M, V, write_grad ? 1 : 0);
  SFT_LAUNCH_CHECK();
  return stats;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) { m.impl("ce_fwd", &ce_fwd); }

}  // namespace sftamd
