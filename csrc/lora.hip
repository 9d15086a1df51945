// LoRA adapter kernels for the wide-GEMM formulation (ops/fused.py LoRAWideFn).
//
// The frozen base weight lives in the left columns of W' = [W | B_blockdiag] and the activation is
// widened to X' = [x | s * dropout(x) A^T], so the adapter forward rides inside the base GEMM. What
// is left are two thin, memory-bound passes per adapted projection, each fused into one kernel:
//
//   lora_fwd:    X'[:, :K] = x,  X'[:, K:] = s * (dropout(x) @ A^T),  xd = dropout(x) (saved for dA)
//                one read of x. v_mfma_f32_16x16x32_bf16 with BOTH operands loaded straight from global
//                memory in fragment layout (x rows are the A operand, rows of A_cat the B operand:
//                16 contiguous bytes per lane each); each of the block's 8 waves reduces an eighth of
//                K and the partial 16 x R tiles are summed through LDS.
//   lora_bwd_dx: dx = base + keep * (dxa @ A) / (1-p), base = the base-weight dgrad (possibly a
//                column slice of dX'), one read of base and one write of dx; the rank-R product is a
//                VALU outer-product loop over an LDS-resident A tile (R <= 64 FMAs per output).
//
// The dropout mask is hash_u32(t*K + k, seed) >= p * 2^32 (common.h), identical to dropout_add and to
// the PyTorch reference, so nothing but the seed is stored between forward and backward.
#include "common.h"

namespace sftamd {
namespace lora {

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// block = 8 waves, 16 rows; wave w reduces k in [w*KW, (w+1)*KW), KW = K/8 (multiple of 32), four
// 32-column steps in flight per iteration (the kernel is a stream over x: latency, not math, bound).
template <int RF>  // R = 16 * RF adapter columns
__global__ __launch_bounds__(512) void fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ A,
                                                  u16* __restrict__ X, u16* __restrict__ xd, long T, int K, long ldX,
                                                  float s, unsigned thresh, float dscale, unsigned seed) {
  constexpr int R = 16 * RF;
  constexpr int NW = 8, U = 4;
  __shared__ float red[NW][16][R + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const long t0 = (long)blockIdx.x * 16;
  const long t = t0 + r;
  const bool rowok = t < T;
  const int KW = K / NW;
  const int kb = w * KW;
  f32x4 acc[RF];
#pragma unroll
  for (int j = 0; j < RF; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = kb; k < kb + KW; k += 32 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k + 32 * u + 8 * g;
      v[u] = (rowok && kk < kb + KW) ? *(const uint4*)(x + t * K + kk) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k + 32 * u + 8 * g;
      if (kk >= kb + KW) break;
      if (rowok) *(uint4*)(X + t * ldX + kk) = v[u];
      if (xd) {
        float f[8];
        unpack8(v[u], f);
        const unsigned long long idx = (unsigned long long)t * K + kk;
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = hash_u32(idx + i, seed) >= thresh ? f[i] * dscale : 0.f;
        v[u] = pack8(f);
        if (rowok) *(uint4*)(xd + t * K + kk) = v[u];
      }
      const bf16x8 a = __builtin_bit_cast(bf16x8, v[u]);
#pragma unroll
      for (int j = 0; j < RF; ++j) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, *(const uint4*)(A + (long)(16 * j + r) * K + kk));
        acc[j] = mfma(a, b, acc[j]);
      }
    }
  }
  // C layout: lane (g, r) holds rows 4g+i, column 16j + r
#pragma unroll
  for (int j = 0; j < RF; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][4 * g + i][16 * j + r] = acc[j][i];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * R; e += NW * 64) {
    const int row = e / R, col = e - row * R;
    const long tt = t0 + row;
    if (tt < T) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) v += red[q][row][col];
      X[tt * ldX + K + col] = f2bf(s * v);
    }
  }
  const int pad = (int)(ldX - K - R);  // zero columns [K + R, ldX) of the padded wide activation
  for (int e = threadIdx.x; e < 16 * pad; e += NW * 64) {
    const int row = e / pad, col = e - row * pad;
    if (t0 + row < T) X[(t0 + row) * ldX + K + R + col] = 0;
  }
}

// tile: 64 rows x 512 columns per 512-thread block; thread = 8 rows x 8 columns (the A tile in LDS is
// reused by 64 rows).
template <int R>
__global__ __launch_bounds__(512) void bwd_dx_kernel(const u16* __restrict__ base, long ldb, const u16* __restrict__ dxa,
                                                     const u16* __restrict__ A, u16* __restrict__ dx, long T, int K,
                                                     unsigned thresh, float dscale, unsigned seed, int drop) {
  __shared__ float As[R][512];
  __shared__ float Ds[64][R];
  const int tid = threadIdx.x;
  const int k0 = blockIdx.x * 512;
  const long t0 = (long)blockIdx.y * 64;
  for (int e = tid; e < R * 64; e += 512) {  // A[:, k0:k0+512] as 8-wide vectors
    const int rr = e >> 6, c8 = e & 63, k = k0 + c8 * 8;
    float f[8];
    if (k < K) {
      unpack8(*(const uint4*)(A + (long)rr * K + k), f);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) As[rr][c8 * 8 + i] = f[i];
  }
  for (int e = tid; e < 64 * R; e += 512) {
    const int row = e / R, col = e - row * R;
    Ds[row][col] = (t0 + row < T) ? bf2f(dxa[(t0 + row) * R + col]) : 0.f;
  }
  __syncthreads();
  const int c8 = tid & 63, rg = tid >> 6;
  const int k = k0 + c8 * 8;
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
#pragma unroll 4
  for (int rr = 0; rr < R; ++rr) {
    float a[8];
    *(float4*)&a[0] = *(const float4*)&As[rr][c8 * 8];
    *(float4*)&a[4] = *(const float4*)&As[rr][c8 * 8 + 4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = Ds[rg * 8 + i][rr];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] += d * a[j];
    }
  }
  if (k >= K) return;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long t = t0 + rg * 8 + i;
    if (t >= T) break;
    float o[8];
    unpack8(*(const uint4*)(base + t * ldb + k), o);
    const unsigned long long idx = (unsigned long long)t * K + k;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool keep = !drop || hash_u32(idx + j, seed) >= thresh;
      o[j] += keep ? acc[i][j] * dscale : 0.f;
    }
    *(uint4*)(dx + t * (long)K + k) = pack8(o);
  }
}

static unsigned thresh_of(double p, float* dscale) {
  const double pc = p < 0 ? 0 : (p > 0.999 ? 0.999 : p);
  *dscale = (float)(1.0 / (1.0 - pc));
  return (unsigned)(pc * 4294967296.0);
}

}  // namespace lora

// x [T, K], A [R, K] (R = 16, 32, 48 or 64) -> (X' [T, ldX], xd [T, K] or empty when p == 0); ldX >= K + R (0 = K + R):
// columns [K + R, ldX) are zero (the wide weight's padding to a whole K-tile pair of the HIP GEMMs)
std::tuple<at::Tensor, at::Tensor> lora_fwd(const at::Tensor& x, const at::Tensor& A, double s, double p, int64_t seed,
                                            int64_t ldX) {
  SFT_CHECK_CUDA(x);
  SFT_CHECK_BF16(x);
  SFT_CHECK_BF16(A);
  SFT_CHECK_CONTIG(x);
  SFT_CHECK_CONTIG(A);
  const long T = x.size(0);
  const int K = x.size(1), R = A.size(0);
  SFT_CHECK(A.size(1) == K && K % 256 == 0 && R % 16 == 0 && R >= 16 && R <= 64, "lora_fwd: shapes");
  if (ldX <= 0) ldX = K + R;
  SFT_CHECK(ldX >= K + R && ldX % 8 == 0, "lora_fwd: ldX >= K + R, multiple of 8");
  auto X = at::empty({T, ldX}, x.options());
  at::Tensor xd = p > 0 ? at::empty_like(x) : at::empty({0}, x.options());
  if (T == 0) return {X, xd};
  float dscale;
  const unsigned thresh = lora::thresh_of(p, &dscale);
  const int grid = (int)((T + 15) / 16);
  u16* xdp = p > 0 ? (u16*)xd.data_ptr() : nullptr;
#define LORA_FWD(RF)                                                                                              \
  lora::fwd_kernel<RF><<<grid, 512, 0, cur_stream()>>>((const u16*)x.data_ptr(), (const u16*)A.data_ptr(),     \
                                                       (u16*)X.data_ptr(), xdp, T, K, ldX, (float)s, thresh, dscale, \
                                                       (unsigned)seed)
  switch (R / 16) {
    case 1: LORA_FWD(1); break;
    case 2: LORA_FWD(2); break;
    case 3: LORA_FWD(3); break;
    default: LORA_FWD(4); break;
  }
#undef LORA_FWD
  SFT_LAUNCH_CHECK();
  return {X, xd};
}

// dx = base + keep * (dxa @ A) / (1-p); base [T, K] with row stride ldb (a column slice is fine)
at::Tensor lora_bwd_dx(const at::Tensor& base, const at::Tensor& dxa, const at::Tensor& A, double p, int64_t seed) {
  SFT_CHECK_CUDA(base);
  SFT_CHECK_BF16(base);
  SFT_CHECK_BF16(dxa);
  SFT_CHECK_BF16(A);
  SFT_CHECK_CONTIG(dxa);
  SFT_CHECK_CONTIG(A);
  const long T = base.size(0);
  const int K = base.size(1), R = A.size(0);
  SFT_CHECK(base.stride(1) == 1 && base.stride(0) % 8 == 0 && K % 8 == 0, "lora_bwd_dx: base layout");
  SFT_CHECK(dxa.size(0) == T && dxa.size(1) == R && A.size(1) == K && R % 16 == 0 && R <= 64, "lora_bwd_dx: shapes");
  auto dx = at::empty({T, K}, base.options());
  if (T == 0) return dx;
  float dscale;
  const unsigned thresh = lora::thresh_of(p, &dscale);
  dim3 grid((K + 511) / 512, (unsigned)((T + 63) / 64));
  SFT_CHECK(grid.y <= 65535u, "lora_bwd_dx: T too large");
#define LORA_BWD(RR)                                                                                              \
  lora::bwd_dx_kernel<RR><<<grid, 512, 0, cur_stream()>>>((const u16*)base.data_ptr(), base.stride(0),            \
                                                          (const u16*)dxa.data_ptr(), (const u16*)A.data_ptr(),    \
                                                          (u16*)dx.data_ptr(), T, K, thresh, dscale, (unsigned)seed, \
                                                          p > 0 ? 1 : 0)
  switch (R / 16) {
    case 1: LORA_BWD(16); break;
    case 2: LORA_BWD(32); break;
    case 3: LORA_BWD(48); break;
    default: LORA_BWD(64); break;
  }
#undef LORA_BWD
  SFT_LAUNCH_CHECK();
  return dx;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("lora_fwd", &lora_fwd);
  m.impl("lora_bwd_dx", &lora_bwd_dx);
}

}  // namespace sftamd
