// Single-token GQA decode attention over a preallocated KV cache (inference).
//
// Split-K ("flash-decoding"): grid (splits, kv_heads); each 256-thread workgroup scores one
// 256-key chunk for ALL query heads of its GQA group (K/V rows are read once per group, 16-byte
// loads), keeps the chunk's (max, sum, unnormalised P.V) in fp32, and a combine kernel merges
// the splits. The live cache length is read from DEVICE memory, so the whole decode step has
// static shapes and is captured once into a hipGraph and replayed per token (no host sync,
// no per-layer launch overhead).
#include "common.h"

namespace sftamd {
namespace decode {

constexpr int D = 128;
constexpr int CHUNK = 256;
constexpr int MAXREP = 8;
constexpr float LOG2E = 1.4426950408889634f;

// q: [nq*D] bf16; kc/vc: [S_max, nkv, D] bf16; part_o: [nkv, splits, rep, D] f32; part_ml: [nkv, splits, rep, 2]
__global__ __launch_bounds__(256) void split_kernel(const u16* __restrict__ q, const u16* __restrict__ kc,
                                                    const u16* __restrict__ vc, const int* __restrict__ len_p,
                                                    float* __restrict__ part_o, float* __restrict__ part_ml, int nq,
                                                    int nkv, float sl2) {
  __shared__ float qs[MAXREP][D];
  __shared__ float ps[MAXREP][CHUNK];
  __shared__ float red[MAXREP][8];
  __shared__ float acc2[2][MAXREP][D];
  const int split = blockIdx.x, kvh = blockIdx.y, splits = gridDim.x;
  const int rep = nq / nkv;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int len = *len_p;
  const int k0 = split * CHUNK;
  float* po = part_o + ((long)(kvh * splits + split) * rep) * D;
  float* pml = part_ml + ((long)(kvh * splits + split) * rep) * 2;
  if (k0 >= len) {  // empty chunk: neutral element for the combine
    if (tid < rep) {
      pml[tid * 2] = -INFINITY;
      pml[tid * 2 + 1] = 0.f;
    }
    return;
  }
  for (int i = tid; i < rep * D; i += 256) qs[i / D][i % D] = bf2f(q[(long)(kvh * rep + i / D) * D + i % D]);
  __syncthreads();
  const int key = k0 + tid;
  float s[MAXREP];
#pragma unroll
  for (int h = 0; h < MAXREP; ++h) s[h] = -INFINITY;
  if (key < len) {
    const u16* kr = kc + ((long)key * nkv + kvh) * D;
#pragma unroll
    for (int h = 0; h < MAXREP; ++h) s[h] = 0.f;
#pragma unroll 4
    for (int c = 0; c < D / 8; ++c) {
      float kf[8];
      unpack8(*(const uint4*)(kr + c * 8), kf);
#pragma unroll
      for (int h = 0; h < MAXREP; ++h)
        if (h < rep) {
#pragma unroll
          for (int e = 0; e < 8; ++e) s[h] += kf[e] * qs[h][c * 8 + e];
        }
    }
#pragma unroll
    for (int h = 0; h < MAXREP; ++h) s[h] *= sl2;
  }
  // chunk max / sum per head
  float m[MAXREP], l[MAXREP];
#pragma unroll
  for (int h = 0; h < MAXREP; ++h) {
    float v = wave_max(s[h]);
    if (lane == 0) red[h][wave] = v;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < MAXREP; ++h) m[h] = fmaxf(fmaxf(red[h][0], red[h][1]), fmaxf(red[h][2], red[h][3]));
  __syncthreads();
#pragma unroll
  for (int h = 0; h < MAXREP; ++h) {
    const float p = (h < rep && key < len) ? exp2f(s[h] - m[h]) : 0.f;
    if (h < rep) ps[h][tid] = p;
    const float v = wave_sum(p);
    if (lane == 0) red[h][4 + wave] = v;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < MAXREP; ++h) l[h] = (red[h][4] + red[h][5]) + (red[h][6] + red[h][7]);
  // P.V: thread -> (dim d, key parity kh)
  const int d = tid & (D - 1), kh = tid >> 7;
  float a[MAXREP];
#pragma unroll
  for (int h = 0; h < MAXREP; ++h) a[h] = 0.f;
  const int nk = min(CHUNK, len - k0);
  for (int t = kh; t < nk; t += 2) {
    const float v = bf2f(vc[((long)(k0 + t) * nkv + kvh) * D + d]);
#pragma unroll
    for (int h = 0; h < MAXREP; ++h)
      if (h < rep) a[h] += ps[h][t] * v;
  }
#pragma unroll
  for (int h = 0; h < MAXREP; ++h)
    if (h < rep) acc2[kh][h][d] = a[h];
  __syncthreads();
  if (kh == 0) {
    for (int h = 0; h < rep; ++h) po[h * D + d] = acc2[0][h][d] + acc2[1][h][d];
  }
  if (tid < rep) {
    pml[tid * 2] = m[tid];
    pml[tid * 2 + 1] = l[tid];
  }
}

__global__ __launch_bounds__(128) void combine_kernel(const float* __restrict__ part_o,
                                                      const float* __restrict__ part_ml, u16* __restrict__ out,
                                                      int nq, int nkv, int splits) {
  const int hq = blockIdx.x, d = threadIdx.x;
  const int rep = nq / nkv, kvh = hq / rep, h = hq - kvh * rep;
  float M = -INFINITY;
  for (int s = 0; s < splits; ++s) M = fmaxf(M, part_ml[((long)(kvh * splits + s) * rep + h) * 2]);
  float L = 0.f, O = 0.f;
  for (int s = 0; s < splits; ++s) {
    const long b = (long)(kvh * splits + s) * rep + h;
    const float ms = part_ml[b * 2];
    if (ms == -INFINITY) continue;
    const float w = exp2f(ms - M);
    L += w * part_ml[b * 2 + 1];
    O += w * part_o[b * D + d];
  }
  out[(long)hq * D + d] = f2bf(O / L);
}

}  // namespace decode

at::Tensor decode_attention(const at::Tensor& q, const at::Tensor& kcache, const at::Tensor& vcache,
                            const at::Tensor& cache_len, int64_t nq, int64_t nkv, double scale) {
  SFT_CHECK_BF16(q);
  SFT_CHECK_BF16(kcache);
  SFT_CHECK(q.is_contiguous() && kcache.is_contiguous() && vcache.is_contiguous(), "contiguous");
  SFT_CHECK(kcache.dim() == 3 && kcache.size(1) == nkv && kcache.size(2) == decode::D, "kcache [S, nkv, 128]");
  SFT_CHECK(q.numel() == nq * decode::D, "q must be [nq*128]");
  SFT_CHECK(nq % nkv == 0 && nq / nkv <= decode::MAXREP, "GQA ratio <= 8");
  SFT_CHECK(cache_len.scalar_type() == at::kInt && cache_len.is_cuda(), "cache_len int32 on device");
  const int smax = kcache.size(0);
  const int splits = (smax + decode::CHUNK - 1) / decode::CHUNK;
  const int rep = nq / nkv;
  auto po = at::empty({nkv * splits * rep * decode::D}, q.options().dtype(at::kFloat));
  auto pml = at::empty({nkv * splits * rep * 2}, q.options().dtype(at::kFloat));
  auto out = at::empty({nq * decode::D}, q.options());
  decode::split_kernel<<<dim3(splits, nkv), 256, 0, cur_stream()>>>(
      (const u16*)q.data_ptr(), (const u16*)kcache.data_ptr(), (const u16*)vcache.data_ptr(), cache_len.data_ptr<int>(),
      po.data_ptr<float>(), pml.data_ptr<float>(), nq, nkv, (float)scale * decode::LOG2E);
  SFT_LAUNCH_CHECK();
  decode::combine_kernel<<<nq, 128, 0, cur_stream()>>>(po.data_ptr<float>(), pml.data_ptr<float>(),
                                                       (u16*)out.data_ptr(), nq, nkv, splits);
  SFT_LAUNCH_CHECK();
  return out;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) { m.impl("decode_attention", &decode_attention); }

}  // namespace sftamd
