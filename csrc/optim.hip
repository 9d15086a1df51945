// Flat-buffer optimizer kernels for gfx950: global sum-of-squares for
// grad clipping and a fused AdamW that reads the clip coefficient from device memory (no host
// sync), updates the fp32 master + fp32 moments and writes the bf16 working copy, 8 elements
// per thread per iteration with 16/32-byte vector accesses.
#include <vector>

#include "common.h"

namespace sftamd {

__global__ __launch_bounds__(256) void sumsq_kernel(const u16* __restrict__ x, long n, float* __restrict__ part) {
  float s = 0.f;
  const long nv = n / 8;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nv; v += (long)gridDim.x * 256) {
    float f[8];
    unpack8(*(const uint4*)(x + v * 8), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += f[i] * f[i];
  }
  for (long i = nv * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float f = bf2f(x[i]);
    s += f * f;
  }
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

at::Tensor sumsq(const at::Tensor& x) {
  SFT_CHECK_BF16(x);
  SFT_CHECK_CONTIG(x);
  const long n = x.numel();
  int grid = (int)std::min<long>(std::max<long>(1, (n / 8 + 255) / 256), 1024);
  auto part = at::empty({grid}, x.options().dtype(at::kFloat));
  sumsq_kernel<<<grid, 256, 0, cur_stream()>>>((const u16*)x.data_ptr(), n, part.data_ptr<float>());
  SFT_LAUNCH_CHECK();
  return part;
}

// Sum of squares over a list of ranges of one flat bf16 buffer in ONE launch: block b covers chunk b =
// (start, length) of ``chunks`` (int64 [C, 2] on the device; the caller splits long ranges into <= 256K-element
// chunks so ~C blocks fill the chip). The gradient norm's leftovers after the wgrad epilogues took theirs
// (tied embedding, norm weights, adapters).
__global__ __launch_bounds__(256) void sumsq_chunks_kernel(const u16* __restrict__ x, const long* __restrict__ chunks,
                                                           float* __restrict__ part) {
  const long st = chunks[2 * blockIdx.x], n = chunks[2 * blockIdx.x + 1];
  const u16* p = x + st;
  float s = 0.f;
  if ((st & 7) == 0) {
    const long nv = n / 8;
    for (long v = threadIdx.x; v < nv; v += 256) {
      float f[8];
      unpack8(*(const uint4*)(p + v * 8), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += f[i] * f[i];
    }
    for (long i = nv * 8 + threadIdx.x; i < n; i += 256) {
      const float f = bf2f(p[i]);
      s += f * f;
    }
  } else {
    for (long i = threadIdx.x; i < n; i += 256) {
      const float f = bf2f(p[i]);
      s += f * f;
    }
  }
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

at::Tensor sumsq_chunks(const at::Tensor& x, const at::Tensor& chunks) {
  SFT_CHECK_BF16(x);
  SFT_CHECK_CONTIG(x);
  SFT_CHECK(chunks.scalar_type() == at::kLong && chunks.is_contiguous() && chunks.dim() == 2 && chunks.size(1) == 2 &&
                chunks.device() == x.device(),
            "sumsq_chunks: int64 [C, 2] (start, length) on the buffer's device");
  const long C = chunks.size(0);
  auto part = at::zeros({std::max<long>(C, 1)}, x.options().dtype(at::kFloat));
  if (C > 0) {
    sumsq_chunks_kernel<<<(unsigned)C, 256, 0, cur_stream()>>>((const u16*)x.data_ptr(), chunks.data_ptr<long>(),
                                                               part.data_ptr<float>());
    SFT_LAUNCH_CHECK();
  }
  return part;
}

// omb1 = 1 - beta1, omb2 = 1 - beta2 computed in double on the host (torch AdamW's constants:
// 1.f - 0.999f would be 1.0000467e-3, not fp32(1e-3)).
__device__ __forceinline__ void adam_elem(float& w, float g, float& m, float& v, float lr, float b1, float b2, float eps,
                                          float wd, float rbc1, float rsbc2, float omb1, float omb2) {
  m = b1 * m + omb1 * g;
  v = b2 * v + omb2 * g * g;
  const float denom = sqrtf(v) * rsbc2 + eps;
  w = w * (1.f - lr * wd) - lr * rbc1 * m / denom;
}

// Stochastic-rounding noise of element i: 16 bits of the stateless hash of its PAIR (elements 2q, 2q + 1 share
// hash(q, seed): low / high half), half the hashing of one hash per element — the bf16-moment update was VALU-bound on
// its three roundings per element (nt streams: 734 us with one hash per element vs 660 us round-to-nearest per 256 M
// elements, profiles/r6_memory_kernels.md). Twin: ops/reference.py bf16_stochastic_round.
__device__ __forceinline__ unsigned sr_hash(unsigned long long i, unsigned seed) {
  return hash_u32(i >> 1, seed) >> (16 * (unsigned)(i & 1));
}

// fp32 -> bf16 with stochastic rounding: add uniform noise below the bf16 ulp, then truncate.
// E[bf16(w)] = w, so pure-bf16 weights do not lose small Adam updates to round-to-nearest.
__device__ __forceinline__ u16 f2bf_sr(float f, unsigned r) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return f2bf(f);  // inf / nan
  u += (r & 0xffffu);
  return (u16)(u >> 16);
}

// 8 consecutive elements idx .. idx + 7: 4 pair hashes (5 when idx is odd: the pairs straddle the vector)
__device__ __forceinline__ uint4 pack8_sr(const float* f, unsigned long long idx, unsigned seed) {
  const unsigned long long q = idx >> 1;
  const bool odd = idx & 1;
  unsigned h[5];
#pragma unroll
  for (int k = 0; k < 4; ++k) h[k] = hash_u32(q + k, seed);
  h[4] = odd ? hash_u32(q + 4, seed) : 0u;
  u16 b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const unsigned r0 = (i & 1) ? (h[i >> 1] >> 16) : h[i >> 1];              // element idx + i, idx even
    const unsigned r1 = (i & 1) ? h[(i + 1) >> 1] : (h[(i + 1) >> 1] >> 16);  // idx odd: pair of idx + i shifted
    b[i] = f2bf_sr(f[i], odd ? r1 : r0);
  }
  return make_uint4(b[0] | (b[1] << 16), b[2] | (b[3] << 16), b[4] | (b[5] << 16), b[6] | (b[7] << 16));
}

// Moment storage: fp32 (default) or bf16 (BF16M: the reference's own state dtype — torch AdamW keeps
// exp_avg/exp_avg_sq in the bf16 parameter dtype — 14 instead of 22 HBM bytes per parameter). bf16
// moments are written with stochastic rounding on streams independent of the parameter's when SR is
// on, round-to-nearest otherwise.
template <bool BF16M>
struct Moments {
  static __device__ __forceinline__ void load(const void* base, long o, float* f) {
    if constexpr (BF16M) {
      unpack8(*(const uint4*)((const u16*)base + o), f);
    } else {
      *(float4*)&f[0] = *(const float4*)((const float*)base + o);
      *(float4*)&f[4] = *(const float4*)((const float*)base + o + 4);
    }
  }
  static __device__ __forceinline__ void store(void* base, long o, const float* f, bool sr, unsigned long long idx,
                                               unsigned seed) {
    if constexpr (BF16M) {
      *(uint4*)((u16*)base + o) = sr ? pack8_sr(f, idx, seed) : pack8(f);
    } else {
      *(float4*)((float*)base + o) = *(const float4*)&f[0];
      *(float4*)((float*)base + o + 4) = *(const float4*)&f[4];
    }
  }
  static __device__ __forceinline__ float load1(const void* base, long i) {
    if constexpr (BF16M) return bf2f(((const u16*)base)[i]);
    else return ((const float*)base)[i];
  }
  static __device__ __forceinline__ void store1(void* base, long i, float f, bool sr, unsigned long long idx,
                                                unsigned seed) {
    if constexpr (BF16M) ((u16*)base)[i] = sr ? f2bf_sr(f, sr_hash(idx, seed)) : f2bf(f);
    else ((float*)base)[i] = f;
  }
};

constexpr unsigned SEED_M = 0x68E31DA4u, SEED_V = 0xB5297A4Du;

// UNR vectors of 8 elements per thread per grid-stride step, all loads issued before any math: the update
// streams 22 (fp32 moments) or 14 (bf16) bytes per parameter, so bytes in flight per wave set its speed.
// Streams touched once per update: nontemporal loads / stores (720 vs 760 us per 256 M elements with bf16 moments +
// SR, 1127 vs 1154 with fp32 moments; profiles/r6_memory_kernels.md)
typedef unsigned __attribute__((ext_vector_type(4))) u32v4;
template <bool NT>
__device__ __forceinline__ uint4 ld16(const void* p) {
  if constexpr (NT) {
    const u32v4 v = __builtin_nontemporal_load((const u32v4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *(const uint4*)p;
  }
}
template <bool NT>
__device__ __forceinline__ void st16(void* p, const uint4& x) {
  if constexpr (NT) {
    const u32v4 v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, (u32v4*)p);
  } else {
    *(uint4*)p = x;
  }
}

template <bool MASTER, bool SR, bool BF16M, int UNR, bool NT = false>
__global__ __launch_bounds__(256) void adamw_kernel(u16* __restrict__ p, const u16* __restrict__ g,
                                                    float* __restrict__ master, void* __restrict__ mom,
                                                    void* __restrict__ var, const float* __restrict__ coef, long n,
                                                    float lr, float b1, float b2, float eps, float wd, float rbc1,
                                                    float rsbc2, float omb1, float omb2, unsigned seed, long idx0) {
  using Mo = Moments<BF16M>;
  const float c = coef[0];
  const long nv = n / 8;
  const long step = (long)gridDim.x * 256 * UNR;
  for (long v0 = blockIdx.x * 256L * UNR + threadIdx.x; v0 < nv; v0 += step) {
    float gf[UNR][8], w[UNR][8], mm[UNR][8], vv[UNR][8];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const long v = v0 + k * 256;
      if (v < nv) {
        const long o = v * 8;
        unpack8(ld16<NT>(g + o), gf[k]);
        if (MASTER) {
          *(float4*)&w[k][0] = *(const float4*)(master + o);
          *(float4*)&w[k][4] = *(const float4*)(master + o + 4);
        } else {
          unpack8(ld16<NT>(p + o), w[k]);
        }
        if constexpr (BF16M && NT) {
          unpack8(ld16<NT>((const u16*)mom + o), mm[k]);
          unpack8(ld16<NT>((const u16*)var + o), vv[k]);
        } else {
          Mo::load(mom, o, mm[k]);
          Mo::load(var, o, vv[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const long v = v0 + k * 256;
      if (v < nv) {
        const long o = v * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          adam_elem(w[k][i], gf[k][i] * c, mm[k][i], vv[k][i], lr, b1, b2, eps, wd, rbc1, rsbc2, omb1, omb2);
        if (MASTER) {
          *(float4*)(master + o) = *(float4*)&w[k][0];
          *(float4*)(master + o + 4) = *(float4*)&w[k][4];
        }
        if constexpr (BF16M && NT) {
          st16<NT>((u16*)mom + o, SR ? pack8_sr(mm[k], idx0 + o, seed ^ SEED_M) : pack8(mm[k]));
          st16<NT>((u16*)var + o, SR ? pack8_sr(vv[k], idx0 + o, seed ^ SEED_V) : pack8(vv[k]));
        } else {
          Mo::store(mom, o, mm[k], SR, idx0 + o, seed ^ SEED_M);
          Mo::store(var, o, vv[k], SR, idx0 + o, seed ^ SEED_V);
        }
        st16<NT>(p + o, SR ? pack8_sr(w[k], idx0 + o, seed) : pack8(w[k]));
      }
    }
  }
  for (long i = nv * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float w = MASTER ? master[i] : bf2f(p[i]);
    float m = Mo::load1(mom, i), vr = Mo::load1(var, i);
    adam_elem(w, bf2f(g[i]) * c, m, vr, lr, b1, b2, eps, wd, rbc1, rsbc2, omb1, omb2);
    if (MASTER) master[i] = w;
    Mo::store1(mom, i, m, SR, idx0 + i, seed ^ SEED_M);
    Mo::store1(var, i, vr, SR, idx0 + i, seed ^ SEED_V);
    p[i] = SR ? f2bf_sr(w, sr_hash(idx0 + i, seed)) : f2bf(w);
  }
}

void adamw_flat(at::Tensor param, const at::Tensor& grad, const c10::optional<at::Tensor>& master, at::Tensor exp_avg,
                at::Tensor exp_avg_sq, const at::Tensor& clip_coef, double lr, double beta1, double beta2, double eps,
                double weight_decay, double bc1, double bc2, int64_t sr_seed, int64_t sr_offset) {
  SFT_CHECK_BF16(param);
  SFT_CHECK_BF16(grad);
  SFT_CHECK(param.is_contiguous() && grad.is_contiguous() && exp_avg.is_contiguous() && exp_avg_sq.is_contiguous(),
            "contiguous");
  SFT_CHECK(exp_avg.scalar_type() == exp_avg_sq.scalar_type() &&
                (exp_avg.scalar_type() == at::kFloat || exp_avg.scalar_type() == at::kBFloat16),
            "moments must both be fp32 or both bf16");
  const bool bf16m = exp_avg.scalar_type() == at::kBFloat16;
  const long n = param.numel();
  SFT_CHECK(grad.numel() == n && exp_avg.numel() == n && exp_avg_sq.numel() == n, "sizes");
  if (n == 0) return;
  // launch shape: 4 vectors of 8 per thread step, at most 2048 blocks. bf16 moments with SR: 759 vs 822 us for 2
  // vectors per step (256 M elements, tools/bench_adamw.py, r5_run14; fp32 moments unchanged), neutral inside the
  // overlapped training step (r5_run16). Fewer blocks measured slower under the overlapped forward (gpu_run49).
  constexpr int UNR = 4;
  int grid = (int)std::min<long>(std::max<long>(1, (n / 8 + 256L * UNR - 1) / (256L * UNR)), 2048L);
  const float rbc1 = (float)(1.0 / bc1), rsbc2 = (float)(1.0 / std::sqrt(bc2));
  const bool has_master = master.has_value() && master->defined();
  if (has_master)
    SFT_CHECK(master->scalar_type() == at::kFloat && master->numel() == n && master->is_contiguous(), "master");
  float* mp = has_master ? master->data_ptr<float>() : nullptr;
  const unsigned seed = (unsigned)sr_seed;
  SFT_CHECK(clip_coef.scalar_type() == at::kFloat && clip_coef.numel() >= 1 && clip_coef.is_cuda(), "clip_coef");
  auto go = [&](auto ms, auto sr, auto bm) {
    constexpr bool M = decltype(ms)::value, S = decltype(sr)::value, B = decltype(bm)::value;
    adamw_kernel<M, S, B, UNR, true><<<grid, 256, 0, cur_stream()>>>(
        (u16*)param.data_ptr(), (const u16*)grad.data_ptr(), mp, exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
        clip_coef.data_ptr<float>(), n, (float)lr, (float)beta1, (float)beta2, (float)eps, (float)weight_decay,
        rbc1, rsbc2, (float)(1.0 - beta1), (float)(1.0 - beta2), seed, (long)sr_offset);
  };
  auto go2 = [&](auto ms, auto sr) {
    if (bf16m) go(ms, sr, std::true_type());
    else go(ms, sr, std::false_type());
  };
  if (has_master) go2(std::true_type(), std::false_type());
  else if (sr_seed != 0) go2(std::false_type(), std::true_type());
  else go2(std::false_type(), std::false_type());
  SFT_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("sumsq", &sumsq);
  m.impl("sumsq_chunks", &sumsq_chunks);
  m.impl("adamw_flat", &adamw_flat);
}

}  // namespace sftamd
