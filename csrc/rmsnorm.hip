// Fused residual-add + RMSNorm forward/backward for gfx950.
//
// One wave64 per row: each lane owns NV 16-byte vectors (8 bf16) of the row, the sum of
// squares is a pure in-wave shuffle reduction (no LDS, no block barrier), and the
// residual add is fused so the residual stream is read once and written once.
// Backward keeps the weight gradient in registers across a grid-stride loop over rows (two rows
// in flight per wave), reduces the 8 waves of a block in LDS, and a second kernel sums the
// per-block partials in a fixed order (deterministic dW, no float atomics in HBM).
#include "common.h"

namespace sftamd {

template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ res,
                                                          const u16* __restrict__ w, u16* __restrict__ y,
                                                          u16* __restrict__ res_out, float* __restrict__ rstd_out,
                                                          int M, int H, float eps, long ldy) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const long base = (long)row * H;
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < H) {
      uint4 a = *(const uint4*)(x + base + c);
      unpack8(a, v[j]);
      if (res) {
        float r[8];
        unpack8(*(const uint4*)(res + base + c), r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[j][i] = bf2f(f2bf(v[j][i] + r[i]));
        *(uint4*)(res_out + base + c) = pack8(v[j]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[j][i] * v[j][i];
    }
  }
  ss = wave_sum(ss);
  const float rstd = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < H) {
      float wf[8], o[8];
      unpack8(*(const uint4*)(w + c), wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = bf2f(f2bf(v[j][i] * rstd)) * wf[i];
      *(uint4*)(y + (long)row * ldy + c) = pack8(o);
    }
  }
  if (lane == 0) rstd_out[row] = rstd;
}

// Backward: 4-wave blocks, ONE row per wave per iteration with every load of the row
// (h, dy, dres, rstd) issued together — v1 issues dres only after the dot-product reduction, so
// each of its iterations pays two serialised HBM latencies. ~120 VGPRs -> 4 waves/SIMD, 16 rows
// (192 KB) in flight per CU. The weight stays packed bf16 in registers; dW accumulates in fp32
// registers across the wave's rows and the 4 waves' partials are summed in LDS in a FIXED order
// (v1's LDS float atomics made dW run-to-run nondeterministic).
template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_bwd2_kernel(const u16* __restrict__ dy, const u16* __restrict__ h,
                                                           const u16* __restrict__ w, const float* __restrict__ rstd,
                                                           const u16* __restrict__ dres, u16* __restrict__ dx,
                                                           float* __restrict__ dw_part, int M, int H) {
  __shared__ __attribute__((aligned(16))) float red[4][NV * 512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  float dw[NV][8];
  uint4 wp[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (lane + 64 * j) * 8;
    wp[j] = c < H ? *(const uint4*)(w + c) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) dw[j][i] = 0.f;
  }
  const float invH = 1.f / (float)H;
  for (int row = blockIdx.x * 4 + wave; row < M; row += nwaves) {
    const long base = (long)row * H;
    uint4 hv[NV], gv[NV], dv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (lane + 64 * j) * 8;
      const bool ok = c < H;
      hv[j] = ok ? *(const uint4*)(h + base + c) : make_uint4(0, 0, 0, 0);
      gv[j] = ok ? *(const uint4*)(dy + base + c) : make_uint4(0, 0, 0, 0);
      dv[j] = (ok && dres) ? *(const uint4*)(dres + base + c) : make_uint4(0, 0, 0, 0);
    }
    const float r = rstd[row];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      float n[8], g[8], wf[8];
      unpack8(hv[j], n);
      unpack8(gv[j], g);
      unpack8(wp[j], wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float nn = n[i] * r;
        dw[j][i] = fmaf(g[i], nn, dw[j][i]);
        dot = fmaf(g[i] * wf[i], nn, dot);
      }
    }
    dot = wave_sum(dot) * invH;
    const float rr = r * dot;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (lane + 64 * j) * 8;
      if (c < H) {
        float n[8], g[8], wf[8], d[8], o[8];
        unpack8(hv[j], n);
        unpack8(gv[j], g);
        unpack8(wp[j], wf);
        unpack8(dv[j], d);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = fmaf(r, fmaf(g[i], wf[i], -n[i] * rr), d[i]);
        *(uint4*)(dx + base + c) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < H) {
      *(float4*)&red[wave][c] = make_float4(dw[j][0], dw[j][1], dw[j][2], dw[j][3]);
      *(float4*)&red[wave][c + 4] = make_float4(dw[j][4], dw[j][5], dw[j][6], dw[j][7]);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256)
    dw_part[(long)blockIdx.x * H + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// out[c] = sum_p part[p][c], fixed order (deterministic). Block = 64 columns (16 float4 lanes) x
// 64 row groups; each thread sums its rows with two independent accumulators, then a fixed
// LDS tree over the row groups. All P rows of a 64-column slab are in flight at once.
// out_bf (optional): the bf16 weight-gradient buffer itself (the DDP engine's flat gradient slice),
// written (accumulate = 0: first contribution of the step) or accumulated (beta = 1) in place — the
// fp32 dW never goes back to PyTorch for a separate copy/add kernel.
__global__ __launch_bounds__(1024) void col_sum2_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                        u16* __restrict__ out_bf, int accumulate, int P, int H) {
  __shared__ float4 red[64][16];
  const int c4 = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + c4 * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  if (c < H) {
    int p = rg;
    for (; p + 64 < P; p += 128) {
      const float4 x = *(const float4*)(part + (long)p * H + c);
      const float4 y = *(const float4*)(part + (long)(p + 64) * H + c);
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
    }
    if (p < P) {
      const float4 x = *(const float4*)(part + (long)p * H + c);
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    }
  }
  red[rg][c4] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  __syncthreads();
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    if (rg < s) {
      const float4 u = red[rg + s][c4];
      float4& v = red[rg][c4];
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    __syncthreads();
  }
  if (rg == 0 && c < H) {
    float4 r = red[0][c4];
    if (out_bf) {
      if (accumulate) {
        const uint2 o = *(const uint2*)(out_bf + c);
        r.x += __uint_as_float(o.x << 16);
        r.y += __uint_as_float(o.x & 0xffff0000u);
        r.z += __uint_as_float(o.y << 16);
        r.w += __uint_as_float(o.y & 0xffff0000u);
      }
      *(uint2*)(out_bf + c) = make_uint2(pk2bf(r.x, r.y),
                                         pk2bf(r.z, r.w));
    } else {
      *(float4*)(out + c) = r;
    }
  }
}


#define NV_DISPATCH(H, ...)                      \
  if ((H) <= 512) {                              \
    constexpr int NV = 1;                        \
    __VA_ARGS__;                                 \
  } else if ((H) <= 1024) {                      \
    constexpr int NV = 2;                        \
    __VA_ARGS__;                                 \
  } else if ((H) <= 2048) {                      \
    constexpr int NV = 4;                        \
    __VA_ARGS__;                                 \
  } else {                                       \
    constexpr int NV = 8;                        \
    __VA_ARGS__;                                 \
  }

// y_ld > H: y is the left [.., H] block of a [M, y_ld] buffer (row stride y_ld; columns H.. left for the consumer: the
// LoRA widening fills them in place, ops/fused.py _lora_wide_prep)
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                                                           const at::Tensor& weight, double eps, int64_t y_ld) {
  SFT_CHECK_CUDA(x);
  SFT_CHECK_BF16(x);
  SFT_CHECK_CONTIG(x);
  SFT_CHECK_BF16(weight);
  const int H = x.size(-1);
  const int M = x.numel() / H;
  SFT_CHECK(H % 8 == 0 && H <= 4096, "hidden size must be a multiple of 8 and <= 4096");
  if (y_ld <= 0) y_ld = H;
  SFT_CHECK(y_ld >= H && y_ld % 8 == 0, "rmsnorm_fwd: y_ld >= H, multiple of 8");
  at::Tensor y;
  if (y_ld == H) {
    y = at::empty_like(x);
  } else {
    auto buf = at::empty({(long)M, y_ld}, x.options());
    std::vector<int64_t> st(x.dim(), 1);
    for (int d = x.dim() - 2; d >= 0; --d) st[d] = (d == x.dim() - 2 ? y_ld : st[d + 1] * x.size(d + 1));
    y = buf.as_strided(x.sizes(), st);
  }
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  at::Tensor res_out = x;
  const u16* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    SFT_CHECK(residual->sizes() == x.sizes() && residual->is_contiguous(), "residual shape");
    res_out = at::empty_like(x);
    rp = (const u16*)residual->data_ptr();
  }
  if (M == 0) return {y, res_out, rstd};
  dim3 grid((M + 3) / 4);
  NV_DISPATCH(H, rmsnorm_fwd_kernel<NV><<<grid, 256, 0, cur_stream()>>>(
                     (const u16*)x.data_ptr(), rp, (const u16*)weight.data_ptr(), (u16*)y.data_ptr(),
                     (u16*)res_out.data_ptr(), rstd.data_ptr<float>(), M, H, (float)eps, (long)y_ld));
  SFT_LAUNCH_CHECK();
  return {y, res_out, rstd};
}

// dw_out (optional, bf16 [H]): receive the weight gradient directly (overwritten, or accumulated when
// ``accumulate``); the returned dW is then an empty tensor.
std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& weight,
                                               const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                                               const c10::optional<at::Tensor>& dw_out, bool accumulate) {
  SFT_CHECK_BF16(dy);
  SFT_CHECK_CONTIG(dy);
  SFT_CHECK_CONTIG(h);
  const int H = h.size(-1);
  const int M = h.numel() / H;
  auto dx = at::empty_like(h);
  const u16* dr = nullptr;
  if (dres.has_value() && dres->defined()) {
    SFT_CHECK(dres->is_contiguous() && dres->scalar_type() == at::kBFloat16, "dres");
    dr = (const u16*)dres->data_ptr();
  }
  SFT_CHECK(rstd.numel() == M && weight.numel() == H && dy.numel() == h.numel(), "rmsnorm_bwd: shape mismatch");
  SFT_CHECK(H % 8 == 0 && H <= 4096, "rmsnorm_bwd: hidden size must be a multiple of 8 and <= 4096");
  auto dw = at::empty({H}, h.options().dtype(at::kFloat));
  if (M == 0) return {dx, dw.zero_()};
  {
    // 4 rows per wave at M = 8192 (512 blocks = 2 per CU): partials stay small (4 MB fp32)
    const int nblk = std::max(1, std::min((M + 15) / 16, 512));
    auto part = at::empty({nblk, H}, h.options().dtype(at::kFloat));
    NV_DISPATCH(H, rmsnorm_bwd2_kernel<NV><<<nblk, 256, 0, cur_stream()>>>(
                       (const u16*)dy.data_ptr(), (const u16*)h.data_ptr(), (const u16*)weight.data_ptr(),
                       rstd.data_ptr<float>(), dr, (u16*)dx.data_ptr(), part.data_ptr<float>(), M, H));
    SFT_LAUNCH_CHECK();
    u16* obf = nullptr;
    if (dw_out.has_value() && dw_out->defined()) {
      SFT_CHECK(dw_out->scalar_type() == at::kBFloat16 && dw_out->is_contiguous() && dw_out->numel() == H &&
                    (reinterpret_cast<uintptr_t>(dw_out->data_ptr()) % 8) == 0,
                "rmsnorm_bwd: dw_out must be a contiguous, 8-byte aligned bf16 [H]");
      obf = (u16*)dw_out->data_ptr();
    }
    col_sum2_kernel<<<(H + 63) / 64, 1024, 0, cur_stream()>>>(part.data_ptr<float>(), dw.data_ptr<float>(), obf,
                                                              accumulate ? 1 : 0, nblk, H);
    SFT_LAUNCH_CHECK();
    return {dx, obf ? at::empty({0}, dw.options()) : dw};
  }
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
}

}  // namespace sftamd
