// Memory-bound elementwise kernels for gfx950: SwiGLU (K6), in-place RoPE on the packed
// qkv GEMM output (K4), embedding gather (K1) and deterministic embedding backward (K1b).
// All accesses are 16-byte vectors (8 x bf16); grids are capped at ~8 blocks/CU and
// grid-stride the rest (CDNA guide G11).
#include "common.h"

namespace sftamd {

static inline int ew_grid(long nvec) {
  long g = (nvec + 255) / 256;
  return (int)std::max<long>(1, std::min<long>(g, 256L * 8));
}

// ------------------------------------------------------------------------------ SwiGLU
// Streaming at HBM rate needs many 16-byte loads in flight per wave: each thread handles UNR vectors per
// grid-stride step and issues all their loads before any math or store. Index math stays 32-bit (host
// checks M * I / 8 < 2^31): a 64-bit division per vector is a long software sequence on the VALU.
constexpr int SW_UNR = 4;  // max unroll (grid sizing / index bound)

template <int SW_UNR>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const u16* __restrict__ gu, u16* __restrict__ out, int n,
                                                         int vpr) {
  const int I = vpr * 8;
  const int stride = gridDim.x * 256 * SW_UNR;
  for (int v0 = blockIdx.x * 256 * SW_UNR + threadIdx.x; v0 < n; v0 += stride) {
    uint4 ga[SW_UNR], ua[SW_UNR];
    long orow[SW_UNR];
#pragma unroll
    for (int k = 0; k < SW_UNR; ++k) {
      const int v = v0 + k * 256;
      const int m = v / vpr, c = (v - m * vpr) * 8;
      orow[k] = (long)m * I + c;
      if (v < n) {
        const u16* src = gu + (long)m * 2 * I + c;
        ga[k] = *(const uint4*)src;
        ua[k] = *(const uint4*)(src + I);
      }
    }
#pragma unroll
    for (int k = 0; k < SW_UNR; ++k) {
      if (v0 + k * 256 < n) {
        float g[8], u[8], o[8];
        unpack8(ga[k], g);
        unpack8(ua[k], u);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = g[i] / (1.f + __expf(-g[i])) * u[i];
        *(uint4*)(out + orow[k]) = pack8(o);
      }
    }
  }
}

template <int SW_UNR>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ gu,
                                                         u16* __restrict__ dgu, int n, int vpr) {
  const int I = vpr * 8;
  const int stride = gridDim.x * 256 * SW_UNR;
  for (int v0 = blockIdx.x * 256 * SW_UNR + threadIdx.x; v0 < n; v0 += stride) {
    uint4 ga[SW_UNR], ua[SW_UNR], da[SW_UNR];
    long grow[SW_UNR];
#pragma unroll
    for (int k = 0; k < SW_UNR; ++k) {
      const int v = v0 + k * 256;
      const int m = v / vpr, c = (v - m * vpr) * 8;
      grow[k] = (long)m * 2 * I + c;
      if (v < n) {
        ga[k] = *(const uint4*)(gu + grow[k]);
        ua[k] = *(const uint4*)(gu + grow[k] + I);
        da[k] = *(const uint4*)(dy + (long)m * I + c);
      }
    }
#pragma unroll
    for (int k = 0; k < SW_UNR; ++k) {
      if (v0 + k * 256 < n) {
        float g[8], u[8], d[8], dg[8], du[8];
        unpack8(ga[k], g);
        unpack8(ua[k], u);
        unpack8(da[k], d);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          swiglu_grad(d[i], g[i], u[i], dg[i], du[i]);
        }
        *(uint4*)(dgu + grow[k]) = pack8(dg);
        *(uint4*)(dgu + grow[k] + I) = pack8(du);
      }
    }
  }
}

static inline int sw_grid(long nvec, int unr) {
  long g = (nvec + 256L * unr - 1) / (256L * unr);
  return (int)std::max<long>(1, std::min<long>(g, 256L * 8));
}

at::Tensor swiglu_fwd(const at::Tensor& gu) {
  SFT_CHECK_BF16(gu);
  SFT_CHECK_CONTIG(gu);
  const int I = gu.size(-1) / 2;
  SFT_CHECK(I % 8 == 0, "intermediate size must be a multiple of 8");
  const long M = gu.numel() / (2 * I);
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  auto out = at::empty(sizes, gu.options());
  if (M == 0) return out;
  const long nvec = M * I / 8;
  SFT_CHECK(nvec < (1L << 31) - 256L * 8 * 256 * SW_UNR, "swiglu: tensor too large for 32-bit indexing");
  swiglu_fwd_kernel<4><<<sw_grid(nvec, 4), 256, 0, cur_stream()>>>((const u16*)gu.data_ptr(), (u16*)out.data_ptr(),
                                                                   (int)nvec, I / 8);
  SFT_LAUNCH_CHECK();
  return out;
}

at::Tensor swiglu_bwd(const at::Tensor& dy, const at::Tensor& gu) {
  SFT_CHECK_CONTIG(dy);
  SFT_CHECK_CONTIG(gu);
  const int I = gu.size(-1) / 2;
  const long M = gu.numel() / (2 * I);
  SFT_CHECK(I % 8 == 0 && dy.numel() == M * I, "swiglu_bwd: shapes");
  auto dgu = at::empty_like(gu);
  if (M == 0) return dgu;
  const long nvec = M * I / 8;
  SFT_CHECK(nvec < (1L << 31) - 256L * 8 * 256 * SW_UNR, "swiglu: tensor too large for 32-bit indexing");
  const u16 *dp = (const u16*)dy.data_ptr(), *gp = (const u16*)gu.data_ptr();
  u16* op = (u16*)dgu.data_ptr();
  swiglu_bwd_kernel<4><<<sw_grid(nvec, 4), 256, 0, cur_stream()>>>(dp, gp, op, (int)nvec, I / 8);
  SFT_LAUNCH_CHECK();
  return dgu;
}

// ------------------------------------------------------------------------------ RoPE
// qkv: [M, ld] with heads [0, nh) rotated (q heads then k heads), rotate_half convention:
// (x1, x2) = (x[i], x[i + D/2]) -> (x1 c - x2 s, x2 c + x1 s); inverse uses -s.
__global__ __launch_bounds__(256) void rope_kernel(u16* __restrict__ qkv, const float* __restrict__ cosb,
                                                   const float* __restrict__ sinb, long M, int ld, int nh, int D,
                                                   float sign) {
  const int half = D / 2;
  const int np = half / 8;  // 8-pair chunks per head
  const long n = M * nh * np;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < n; t += (long)gridDim.x * 256) {
    const long m = t / (nh * np);
    const int rem = (int)(t - m * nh * np);
    const int hh = rem / np, p = (rem - hh * np) * 8;
    u16* base = qkv + m * ld + hh * D;
    float a[8], b[8], c[8], s[8], o1[8], o2[8];
    unpack8(*(const uint4*)(base + p), a);
    unpack8(*(const uint4*)(base + half + p), b);
    const float4* cp = (const float4*)(cosb + m * half + p);
    const float4* sp = (const float4*)(sinb + m * half + p);
    *(float4*)&c[0] = cp[0];
    *(float4*)&c[4] = cp[1];
    *(float4*)&s[0] = sp[0];
    *(float4*)&s[4] = sp[1];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float si = sign * s[i];
      o1[i] = a[i] * c[i] - b[i] * si;
      o2[i] = b[i] * c[i] + a[i] * si;
    }
    *(uint4*)(base + p) = pack8(o1);
    *(uint4*)(base + half + p) = pack8(o2);
  }
}

void rope_(at::Tensor qkv, const at::Tensor& cos, const at::Tensor& sin, int64_t n_q, int64_t n_kv, int64_t head_dim,
           bool inverse) {
  SFT_CHECK_BF16(qkv);
  SFT_CHECK_CONTIG(qkv);
  SFT_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat, "cos/sin must be fp32");
  SFT_CHECK(cos.is_contiguous() && sin.is_contiguous(), "cos/sin contiguous");
  SFT_CHECK(head_dim % 16 == 0, "head_dim must be a multiple of 16");
  const int ld = qkv.size(-1);
  const long M = qkv.numel() / ld;
  SFT_CHECK(cos.numel() == M * head_dim / 2, "cos table shape");
  const int nh = n_q + n_kv;
  if (M == 0) return;
  const long n = M * nh * (head_dim / 16);
  rope_kernel<<<ew_grid(n), 256, 0, cur_stream()>>>((u16*)qkv.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), M,
                                                    ld, nh, (int)head_dim, inverse ? -1.f : 1.f);
  SFT_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------ embedding
__global__ __launch_bounds__(256) void embedding_fwd_kernel(const int64_t* __restrict__ ids, const u16* __restrict__ w,
                                                            u16* __restrict__ out, long M, int H, long V) {
  const int vpr = H / 8;
  const long n = M * vpr;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < n; t += (long)gridDim.x * 256) {
    const long m = t / vpr;
    const int c = (int)(t - m * vpr) * 8;
    long id = ids[m];
    SFT_DASSERT(id >= 0 && id < V);
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);
    *(uint4*)(out + m * H + c) = *(const uint4*)(w + id * H + c);
  }
}

// One wave per sorted position; the first position of each run of equal ids sums all rows of
// the run in fp32 (fixed order) and adds the result into the bf16 gradient row: one writer per
// row, no atomics, bitwise reproducible.
template <int NV>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const u16* __restrict__ dy, const int* __restrict__ sorted,
                                                            const int* __restrict__ perm, u16* __restrict__ gw, int M,
                                                            int H) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= M) return;
  const int id = sorted[i];
  SFT_DASSERT(i == 0 || sorted[i - 1] <= id);
  if (i > 0 && sorted[i - 1] == id) return;
  float acc[NV][8];
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
  // Runs of a frequent id are long on real chat data (the system prompt repeats in every sample: hundreds of
  // rows for one id), so rows are fetched EU at a time — all loads in flight before any add — and then summed
  // in the same sequential order as before (bitwise identical result, EU x fewer dependent round trips).
  constexpr int EU = 8;
  for (int k = i; k < M && sorted[k] == id; k += EU) {
    uint4 v[EU][NV];
    bool ok[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      ok[u] = (k + u < M) && sorted[k + u] == id;  // runs are contiguous: valid for a prefix of u
      const long row = ok[u] ? perm[k + u] : 0;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c = (lane + 64 * j) * 8;
        v[u][j] = (ok[u] && c < H) ? *(const uint4*)(dy + row * H + c) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      if (!ok[u]) break;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        float f[8];
        unpack8(v[u][j], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] += f[e];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < H) {
      float f[8];
      u16* p = gw + (long)id * H + c;
      unpack8(*(const uint4*)p, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += acc[j][e];
      *(uint4*)p = pack8(f);
    }
  }
}

at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& w) {
  SFT_CHECK_BF16(w);
  SFT_CHECK_CONTIG(w);
  SFT_CHECK(ids.scalar_type() == at::kLong, "ids must be int64");
  auto idc = ids.contiguous();
  const int H = w.size(1);
  SFT_CHECK(H % 8 == 0, "hidden % 8");
  const long M = idc.numel();
  auto sizes = idc.sizes().vec();
  sizes.push_back(H);
  auto out = at::empty(sizes, w.options());
  if (M == 0) return out;
  embedding_fwd_kernel<<<ew_grid(M * H / 8), 256, 0, cur_stream()>>>(idc.data_ptr<int64_t>(), (const u16*)w.data_ptr(),
                                                                      (u16*)out.data_ptr(), M, H, w.size(0));
  SFT_LAUNCH_CHECK();
  return out;
}

void embedding_bwd(const at::Tensor& dy, const at::Tensor& sorted_ids, const at::Tensor& perm, at::Tensor gw) {
  SFT_CHECK_CONTIG(dy);
  SFT_CHECK_BF16(gw);
  SFT_CHECK_CONTIG(gw);
  SFT_CHECK(sorted_ids.scalar_type() == at::kInt && perm.scalar_type() == at::kInt, "int32 index tensors");
  const int H = gw.size(1);
  const int M = sorted_ids.numel();
  SFT_CHECK(H % 8 == 0 && H <= 4096, "hidden");
  if (M == 0) return;
  dim3 grid((M + 3) / 4);
  auto launch = [&](auto nv) {
    constexpr int NV = decltype(nv)::value;
    embedding_bwd_kernel<NV><<<grid, 256, 0, cur_stream()>>>((const u16*)dy.data_ptr(), sorted_ids.data_ptr<int>(),
                                                             perm.data_ptr<int>(), (u16*)gw.data_ptr(), M, H);
  };
  if (H <= 512) launch(std::integral_constant<int, 1>());
  else if (H <= 1024) launch(std::integral_constant<int, 2>());
  else if (H <= 2048) launch(std::integral_constant<int, 4>());
  else launch(std::integral_constant<int, 8>());
  SFT_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// LoRA dropout: out[t,k] = a[t,k] + keep(t*K+k) * b[t,k] / (1-p), keep = drop_keep(index, seed) (common.h).
// The mask is a pure function of (seed, element index), so backward regenerates it instead of
// storing it; a and b may be column slices of wider buffers (row strides lda, ldb).
// grid: (column blocks of 256 x 8 elements, rows); no integer division in the index math
__global__ __launch_bounds__(256) void dropout_add_kernel(const u16* __restrict__ a, long lda, const u16* __restrict__ b,
                                                          long ldb, u16* __restrict__ out, long ldo, long T, int K,
                                                          unsigned thresh, float scale, unsigned seed) {
  const int k = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (k >= K) return;
  for (long t = blockIdx.y; t < T; t += gridDim.y) {
  float bv[8], o[8];
  unpack8(*(const uint4*)(b + t * ldb + k), bv);
  if (a) {
    unpack8(*(const uint4*)(a + t * lda + k), o);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = 0.f;
  }
  const unsigned long long idx = (unsigned long long)t * K + k;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] += drop_keep(idx + i, seed, thresh) ? bv[i] * scale : 0.f;
  *(uint4*)(out + t * ldo + k) = pack8(o);
  }
}

// LoRA input widening: X[:, :K] = x and (p > 0) xd = dropout(x), one read of x.
__global__ __launch_bounds__(256) void lora_widen_kernel(const u16* __restrict__ x, u16* __restrict__ X, long ldX,
                                                         u16* __restrict__ xd, long T, int K, unsigned thresh,
                                                         float scale, unsigned seed) {
  const int k = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (k >= K) return;
  for (long t = blockIdx.y; t < T; t += gridDim.y) {
  const uint4 v = *(const uint4*)(x + t * K + k);
  *(uint4*)(X + t * ldX + k) = v;
  if (xd) {
    float f[8];
    unpack8(v, f);
    const unsigned long long idx = (unsigned long long)t * K + k;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = drop_keep(idx + i, seed, thresh) ? f[i] * scale : 0.f;
    *(uint4*)(xd + t * (long)K + k) = pack8(f);
  }
  }
}


at::Tensor dropout_add(const c10::optional<at::Tensor>& a, const at::Tensor& b, double p, int64_t seed) {
  SFT_CHECK_CUDA(b);
  SFT_CHECK_BF16(b);
  SFT_CHECK(b.dim() == 2 && b.stride(1) == 1 && b.stride(0) % 8 == 0 && b.size(1) % 8 == 0, "dropout_add: b layout");
  const long T = b.size(0);
  const int K = b.size(1);
  const u16* ap = nullptr;
  long lda = 0;
  if (a.has_value() && a->defined()) {
    SFT_CHECK(a->sizes() == b.sizes() && a->stride(1) == 1 && a->stride(0) % 8 == 0 && a->scalar_type() == at::kBFloat16,
              "dropout_add: a layout");
    ap = (const u16*)a->data_ptr();
    lda = a->stride(0);
  }
  auto out = at::empty({T, K}, b.options());
  if (T == 0) return out;
  float scale;
  const unsigned thresh = drop_thresh16(p, &scale);
  dim3 grid((K / 8 + 255) / 256, (unsigned)std::min<long>(T, 65535));
  dropout_add_kernel<<<grid, 256, 0, cur_stream()>>>(ap, lda, (const u16*)b.data_ptr(), b.stride(0), (u16*)out.data_ptr(),
                                                     K, T, K, thresh, scale, (unsigned)seed);
  SFT_LAUNCH_CHECK();
  return out;
}

// Returns (X [T, K+R] with X[:, :K] = x (X[:, K:] uninitialised), xd = dropout(x) or an empty tensor if p == 0).
std::tuple<at::Tensor, at::Tensor> lora_widen(const at::Tensor& x, int64_t R, double p, int64_t seed) {
  SFT_CHECK_CUDA(x);
  SFT_CHECK_BF16(x);
  SFT_CHECK_CONTIG(x);
  SFT_CHECK(x.dim() == 2 && x.size(1) % 8 == 0 && R % 8 == 0, "lora_widen: x [T, K], K and R multiples of 8");
  const long T = x.size(0);
  const int K = x.size(1);
  auto X = at::empty({T, K + R}, x.options());
  at::Tensor xd = p > 0 ? at::empty_like(x) : at::empty({0}, x.options());
  if (T == 0) return {X, xd};
  float scale;
  const unsigned thresh = drop_thresh16(p, &scale);
  dim3 grid((K / 8 + 255) / 256, (unsigned)std::min<long>(T, 65535));
  lora_widen_kernel<<<grid, 256, 0, cur_stream()>>>((const u16*)x.data_ptr(), (u16*)X.data_ptr(), K + R,
                                                    p > 0 ? (u16*)xd.data_ptr() : nullptr, T, K, thresh, scale,
                                                    (unsigned)seed);
  SFT_LAUNCH_CHECK();
  return {X, xd};
}

// ------------------------------------------------------------------------------ CU occupancy probe (tools only)
// cu_hog(sink, blocks, usec): `blocks` workgroups that each hold one CU (81 KB of LDS: one per CU) and sleep until `usec`
// of wall time (s_memrealtime, 100 MHz) have passed — a stand-in for the RCCL channel blocks that sit on CUs while a
// collective overlaps the backward (tools/bench_cu_contention.py measures what the GEMM grids lose to them). Every wave
// exits at the deadline (usec is capped at 2 s).
__global__ __launch_bounds__(256) void cu_hog_kernel(unsigned long long ticks, int* __restrict__ sink) {
  extern __shared__ int hog_lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int n = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(16);
    ++n;
  }
  hog_lds[threadIdx.x] = n;
  __syncthreads();
  if (n < 0) sink[threadIdx.x] = hog_lds[255 - threadIdx.x];  // never taken: keeps the LDS allocation live
}

void cu_hog(at::Tensor sink, int64_t blocks, double usec) {
  SFT_CHECK(blocks > 0 && blocks <= 4096 && usec > 0, "cu_hog: 1..4096 blocks, usec > 0");
  SFT_CHECK(sink.is_cuda() && sink.scalar_type() == at::kInt && sink.numel() >= 256, "cu_hog: int32 sink of 256");
  constexpr int LDS = 81 * 1024;
  static bool attr = [] {
    return hipFuncSetAttribute((const void*)cu_hog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS) ==
           hipSuccess;
  }();
  SFT_CHECK(attr, "cu_hog: could not raise the dynamic LDS limit");
  const double us = std::min(usec, 2.0e6);
  cu_hog_kernel<<<(unsigned)blocks, 256, LDS, cur_stream()>>>((unsigned long long)(us * 100.0), sink.data_ptr<int>());
  SFT_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("cu_hog", &cu_hog);
  m.impl("dropout_add", &dropout_add);
  m.impl("lora_widen", &lora_widen);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("rope_", &rope_);
  m.impl("embedding_fwd", &embedding_fwd);
  m.impl("embedding_bwd", &embedding_bwd);
}

}  // namespace sftamd
