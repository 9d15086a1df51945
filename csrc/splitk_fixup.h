// Deterministic split-K fixup shared by the weight-gradient kernels (gemm_wgrad.hip ring variants, gemm_4w.hip):
// fp32 tile-local slabs of a tile's split pieces are summed in a fixed order into the bf16 output.
#pragma once

#include "common.h"

namespace sftamd {

// Split tiles t = tile0 .. tile0 + ntiles - 1: C[tile] = bf16(sum_s P[t][s] (+ C when accumulating)),
// 8 elements per thread, slabs summed in order s = 0..S-1. Tile numbering: row-major over [nbm][nbk] tiles, or
// (group > 0) blocked by `group` row-tiles as the launching kernel walks them.
template <int BM, int BN>
__device__ __forceinline__ void splitk_fixup_body(const float* __restrict__ P, u16* __restrict__ C, int tile0,
                                                  int ntiles, int splits, int nbk, int K, int accumulate,
                                                  float* __restrict__ nrm, int nbm, int group, const int bid) {
  constexpr int E8 = BM * BN / 8;
  if (nrm != nullptr && bid == 0) {  // the whole tiles' partials, parked past the slabs by ring_kernel
    const float* src = P + (long)ntiles * splits * BM * BN;
    for (int i = threadIdx.x; i < tile0 * 8; i += 256) nrm[i] = src[i];
  }
  static_assert((BM * BN / 8) % 256 == 0, "fixup blocks cover whole tiles");
  const long idx = (long)bid * 256 + threadIdx.x;
  if (idx >= (long)ntiles * E8) return;  // never taken: the grid covers whole tiles
  const int t = (int)(idx / E8), e = (int)(idx - (long)t * E8) * 8;
  const int row = e / BN, col = e - row * BN;
  const float* q = P + (long)t * splits * BM * BN + e;
  float v[8];
  *(float4*)&v[0] = *(const float4*)q;
  *(float4*)&v[4] = *(const float4*)(q + 4);
  for (int s = 1; s < splits; ++s) {
    const float4 a = *(const float4*)(q + (long)s * BM * BN), b = *(const float4*)(q + (long)s * BM * BN + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
  const int tile = tile0 + t;
  int bn, bk;
  if (group > 0) {  // GROUP-blocked tile order of gemm_4w.hip (group M-tiles x all nbk N-tiles per group)
    const int per_group = group * nbk, grp = tile / per_group, first = grp * group;
    const int gsz = min(nbm - first, group), in = tile - grp * per_group;
    bn = first + in % gsz;
    bk = in / gsz;
  } else {
    bn = tile / nbk;
    bk = tile - bn * nbk;
  }
  u16* out = C + (long)(bn * BM + row) * K + bk * BN + col;
  if (accumulate) {
    float o[8];
    unpack8(*(const uint4*)out, o);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += o[i];
  }
  const uint4 pk = pack8(v);
  *(uint4*)out = pk;
  if (nrm != nullptr) {  // per-block slot (blocks never straddle a tile: E8 % 256 == 0)
    float r[8], ss = 0.f;
    unpack8(pk, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += r[i] * r[i];
    ss = wave_sum(ss);
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) nrm[(long)tile0 * 8 + bid] = red[0] + red[1] + red[2] + red[3];
  }
}

template <int BM, int BN>
__global__ void __launch_bounds__(256) splitk_fixup_kernel(const float* __restrict__ P, u16* __restrict__ C, int tile0,
                                                           int ntiles, int splits, int nbk, int K, int accumulate,
                                                           float* __restrict__ nrm, int nbm = 0, int group = 0) {
  splitk_fixup_body<BM, BN>(P, C, tile0, ntiles, splits, nbk, K, accumulate, nrm, nbm, group, blockIdx.x);
}

// The fixups of up to four problems of one multi-problem launch as ONE grid: problem i owns blocks [b_i, b_{i+1})
// (b_0 = 0, unused = INT_MAX); per problem the arguments of splitk_fixup_kernel.
struct FixArgs {
  const float* P;
  u16* C;
  float* nrm;
  int tile0, ntiles, nbk, K, accumulate, nbm, group;
};

template <int BM, int BN>
__global__ void __launch_bounds__(256) splitk_fixup_multi_kernel(FixArgs f0, FixArgs f1, FixArgs f2, FixArgs f3,
                                                                 int b1, int b2, int b3, int splits) {
  const int b = blockIdx.x;
  const int pi = (b >= b1) + (b >= b2) + (b >= b3);
#define FXSEL(x) (pi == 0 ? f0.x : pi == 1 ? f1.x : pi == 2 ? f2.x : f3.x)
  const int bid = b - (pi == 0 ? 0 : pi == 1 ? b1 : pi == 2 ? b2 : b3);
  splitk_fixup_body<BM, BN>(FXSEL(P), FXSEL(C), FXSEL(tile0), FXSEL(ntiles), splits, FXSEL(nbk), FXSEL(K),
                            FXSEL(accumulate), FXSEL(nrm), FXSEL(nbm), FXSEL(group), bid);
#undef FXSEL
}

}  // namespace sftamd
