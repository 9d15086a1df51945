// LoRA adapter kernels for the wide-GEMM formulation (ops/fused.py LoRAWideFn).
//
// The frozen base weight lives in the left columns of W' = [W | B_blockdiag] and the activation is
// widened to X' = [x | s * dropout(x) A^T], so the adapter forward rides inside the base GEMM. What
// is left are two thin, memory-bound passes per adapted projection, each fused into one kernel:
//
//   lora_fwd:    X'[:, :K] = x,  X'[:, K:] = s * (dropout(x) @ A^T)  (xd = dropout(x) only when asked)
//                one read of x, streamed row-contiguously through LDS into v_mfma_f32_16x16x32_bf16
//                fragments (rows of A_cat loaded from global memory in fragment layout); the partial
//                16 x R tiles of the block's 8 waves are summed through LDS.
//   lora_bwd_dx: dx = base + keep * (dxa @ A) / (1-p), base = the base-weight dgrad (possibly a
//                column slice of dX'), one read of base and one write of dx; the rank-R product on
//                16x16x16 MFMAs whose B columns are permuted so every lane holds 8 contiguous outputs.
//   lora_tsum:   the adapter gradients' token reductions (dA, dB^T), one pass over the wide operand.
//
// The dropout mask is drop_keep(t*K + k, seed, p * 65536) (common.h; keep8 below computes it per 8-element chunk),
// identical to dropout_add and to the PyTorch reference, so nothing but the seed is stored between forward and
// backward.
#include "common.h"

namespace sftamd {
namespace lora {

// keep bits of the 8 elements i0 .. i0 + 7 (bit j: drop_keep(i0 + j, seed, thresh16), common.h), bit-identical: the 8
// elements are 4 pairs, one hash each (low / high 16 bits for the even / odd element); with i0 % 8 == 0 the 4 pair
// indices share the high word (no carry out of the low one), so the first multiply of the hash becomes a constant add
// per pair and the high-word / seed terms are computed once per chunk.
__device__ __forceinline__ unsigned keep8(unsigned long long i0, unsigned seed, unsigned thresh) {
  const unsigned long long q0 = i0 >> 1;
  const unsigned lo = (unsigned)q0 * 0x9E3779B9u;
  const unsigned hi = (unsigned)(q0 >> 32) * 0x85EBCA6Bu ^ seed * 0xC2B2AE35u;
  unsigned bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned x = (lo + (unsigned)j * 0x9E3779B9u) ^ hi;
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    bits |= ((unsigned)((x & 0xFFFFu) >= thresh) << (2 * j)) | ((unsigned)((x >> 16) >= thresh) << (2 * j + 1));
  }
  return bits;
}

// zero the dropped bf16 elements of an 8-element chunk (bit j of `bits` = keep element j): pure bit selects, the
// 1 / (1 - p) scale is applied to the reduction's fp32 result instead of to every element
__device__ __forceinline__ uint4 mask8(uint4 v, unsigned bits) {
  auto m = [&](int j) {
    return ((0u - ((bits >> j) & 1u)) & 0xFFFFu) | ((0u - ((bits >> (j + 1)) & 1u)) & 0xFFFF0000u);
  };
  return make_uint4(v.x & m(0), v.y & m(2), v.z & m(4), v.w & m(6));
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// block = 8 waves, 16 rows, streamed in 512-column chunks; wave w loads and consumes columns 64 w .. 64 w + 63 of
// each chunk (each wave instruction reads or writes 8 rows x 128 contiguous bytes). The lane's pieces are copied to
// X', masked (dropout) into an LDS tile [16][512 + 8] (and to xd when asked), and the wave reads its 64 columns of the
// tile back as MFMA A fragments (ds_read_b128; the 16-byte row padding spreads the 16 rows over all banks) against
// rows of A_cat loaded straight from global memory in fragment layout. The next chunk's global loads are issued before
// this chunk's stores, LDS write and MFMAs; two LDS tiles alternate; the waves only meet at the final reduction. (The first version loaded x itself in fragment layout, every wave
// instruction touching 16 rows x 64 B: 153.9 vs 128.5 us for the SwiGLU-fused K = 11008 case, 115.8 vs 91.2 plain,
// tools/bench_lora_kernels.py, r4_run29.)
// SW: x is the SwiGLU input gu [T, 2K] (gate | up) and the widened activation is act = silu(gate) * up, rounded to bf16
// as the SwiGLU kernel does (the LoRA MLP's down projection: no separate SwiGLU pass, no act tensor).
template <int RF, bool SW = false, int NCH = 0>  // R = 16 * RF adapter columns; NCH > 0: K == 512 NCH
__global__ __launch_bounds__(512) void fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ A,
                                                  u16* __restrict__ X, u16* __restrict__ xd, long T, int K, long ldX,
                                                  float s, unsigned thresh, float dscale, unsigned seed, int drop,
                                                  long ldx, int copy) {
  constexpr int R = 16 * RF, NW = 8, CK = 512, XP = CK + 8, NV = SW ? 2 : 1, DEP = NCH > 0 ? NCH : 1;
  __shared__ __attribute__((aligned(16))) u16 xs[2][16][XP];
  __shared__ float red[NW][16][R + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const long t0 = (long)blockIdx.x * 16;
  // loader role: rows (lane >> 3) + 8 h of the block, columns lc .. lc + 7 of the chunk — wave w loads exactly the
  // 64 columns its MFMAs read (8 rows x 128 B per wave instruction), so the LDS tile regions are wave-private and the
  // chunk loop needs no workgroup barrier
  const int lc = 64 * w + 8 * (lane & 7);
  long lt[2];
  bool lok[2];
  const u16* xrow[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    lt[h] = t0 + (lane >> 3) + 8 * h;
    lok[h] = lt[h] < T;
    xrow[h] = x + (lok[h] ? lt[h] : T - 1) * ldx;
  }
  f32x4 acc[RF];
#pragma unroll
  for (int j = 0; j < RF; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 rw[DEP][2][NV];
  auto load = [&](uint4 (&dst)[2][NV], int k0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = k0 + lc, cc = c < K ? c : 0;
      dst[h][0] = *(const uint4*)(xrow[h] + cc);
      if constexpr (SW) dst[h][1] = *(const uint4*)(xrow[h] + K + cc);
    }
  };
  // the wave's A_cat fragments of a chunk (rows 16 j + r, columns 64 w + 32 ks + 8 g): loaded one chunk ahead for
  // R <= 32 or short rows (for R >= 48 the streamed variants went past 128 VGPRs: half the occupancy, or spills)
  constexpr bool PFA = RF <= 2 || (NCH > 0 && RF <= 3);
  uint4 an[2][RF];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kk = k0 + 64 * w + 32 * ks + 8 * g;
#pragma unroll
      for (int j = 0; j < RF; ++j)
        an[ks][j] = kk < K ? *(const uint4*)(A + (long)(16 * j + r) * K + kk) : make_uint4(0, 0, 0, 0);
    }
  };
  const int nch = NCH > 0 ? NCH : (K + CK - 1) / CK;
  if constexpr (NCH > 0) {  // short rows: every chunk's loads in flight at once
#pragma unroll
    for (int c = 0; c < NCH; ++c) load(rw[c], c * CK);
  } else {
    load(rw[0], 0);
  }
  if constexpr (PFA) load_a(0);
#pragma unroll
  for (int ch = 0; ch < nch; ++ch) {
    const int k0 = ch * CK;
    const int sl = NCH > 0 ? ch : 0;
    uint4 v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (SW) {
        float ga[8], up[8], o[8];
        unpack8(rw[sl][h][0], ga);
        unpack8(rw[sl][h][1], up);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = ga[i] / (1.f + __expf(-ga[i])) * up[i];
        v[h] = pack8(o);
      } else {
        v[h] = rw[sl][h][0];
      }
    }
    uint4 ac[2][RF];
    if constexpr (PFA) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < RF; ++j) ac[ks][j] = an[ks][j];
    }
    if (ch + 1 < nch) {  // the next chunk flies under this chunk's stores, LDS write and MFMAs (loading two or three
                         // ahead measured slower: 127.6 / 135.8 vs 126.1 us SwiGLU-fused, r5_run22)
      if constexpr (NCH == 0) load(rw[0], k0 + CK);
      if constexpr (PFA) load_a(k0 + CK);
    }
    u16(*tile)[XP] = xs[ch & 1];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = k0 + lc;
      if (c < K) {
        if (copy && lok[h]) *(uint4*)(X + lt[h] * ldX + c) = v[h];  // (!copy: x IS X[:, :K], written by its producer)
        if (drop) {
          const unsigned bits = keep8((unsigned long long)lt[h] * K + c, seed, thresh);
          if (xd && lok[h]) {  // dropout(x) itself, scaled (tests / save_xd only)
            float f[8];
            unpack8(v[h], f);
#pragma unroll
            for (int i = 0; i < 8; ++i) f[i] = ((bits >> i) & 1u) ? f[i] * dscale : 0.f;
            *(uint4*)(xd + lt[h] * K + c) = pack8(f);
          }
          v[h] = mask8(v[h], bits);  // the 1 / (1 - p) scale goes into s below
        }
        *(uint4*)&tile[(lane >> 3) + 8 * h][lc] = v[h];
      }
    }
    // the wave's own tile columns are complete (its reads of this tile two chunks ago came earlier in program order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kl = 64 * w + 32 * ks + 8 * g;
      if (k0 + 64 * w + 32 * ks < K) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, *(const uint4*)&tile[r][kl]);
#pragma unroll
        for (int j = 0; j < RF; ++j) {
          const uint4 b = PFA ? ac[ks][j] : *(const uint4*)(A + (long)(16 * j + r) * K + k0 + kl);
          acc[j] = mfma(a, __builtin_bit_cast(bf16x8, b), acc[j]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RF; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][4 * g + i][16 * j + r] = acc[j][i];
  __syncthreads();
  for (int e = tid; e < 16 * R; e += NW * 64) {
    const int row = e / R, col = e - row * R;
    const long tt = t0 + row;
    if (tt < T) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) v += red[q][row][col];
      X[tt * ldX + K + col] = f2bf((drop ? s * dscale : s) * v);  // kept elements entered the MFMAs unscaled
    }
  }
  const int pad = (int)(ldX - K - R);
  for (int e = tid; e < 16 * pad; e += NW * 64) {
    const int row = e / pad, col = e - row * pad;
    if (t0 + row < T) X[(t0 + row) * ldX + K + R + col] = 0;
  }
}

// lora_bwd_dx: dx = base + keep * (dxa @ A) / (1-p) in one pass over base (and gu, writing dgu = swiglu_bwd(dx, gu)
// for the down projection of a LoRA MLP: no dx round trip through HBM), the rank-R product on the matrix cores and no
// LDS: wave = 16 token rows x 128 columns, the
// product dxa [16, R] . A [R, 128] as eight v_mfma_f32_16x16x16_bf16 tiles whose B columns are PERMUTED — tile j,
// column c is output column 8 c + j — so lane (g = l >> 4, c = l & 15) ends up holding rows 4 g .. 4 g + 3 x the 8
// CONTIGUOUS columns 8 c .. 8 c + 7: exactly the 16-byte pieces of base / gu / dx it loads and stores (each wave
// instruction touches 4 rows x 256 contiguous bytes). The B fragments come from 16-byte loads of A rows (8 columns
// of one k) repacked by bit selects; dxa and A are loaded first, so the MFMAs wait only for them while base / gu fly.
// (Replaced a VALU outer product over an fp32 A tile staged in LDS, 32 rows x 512 columns per 512-thread block:
// 39.1 / 30.5 / 22.6 -> 17.5 / 16.7 / 14.8 us for the R = 48 / 32 / 16 adapters at K = 2048, 197.9 -> 159.5 us for the
// dgu-writing K = 11008 pass, T = 8192; LoRA 133.2 -> 135.8 samples/s, r5_run16.)
__device__ __forceinline__ f32x4 mfma16(const uint2& a, const uint2& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c, 0,
                                                   0, 0);
}

template <int R, bool SWIGLU>
__global__ __launch_bounds__(256) void bwd_dx_kernel(const u16* __restrict__ base, long ldb,
                                                          const u16* __restrict__ dxa, const u16* __restrict__ A,
                                                          u16* __restrict__ dx, long T, int K, unsigned thresh,
                                                          float dscale, unsigned seed, int drop,
                                                          const u16* __restrict__ gu) {
  constexpr int KS = R / 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int kw = blockIdx.x * 512 + 128 * w;
  if (kw >= K) return;  // whole wave past the last column (no barriers in this kernel)
  const long t0 = (long)blockIdx.y * 16;
  const int k = kw + 8 * c;
  const bool kok = k < K;
  const int kc = kok ? k : K - 8;
  uint2 da[KS];
  uint4 av[KS][4];
  const long ta = min(t0 + c, T - 1);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    da[s] = *(const uint2*)(dxa + ta * R + 16 * s + 4 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) av[s][i] = *(const uint4*)(A + (long)(16 * s + 4 * g + i) * K + kc);
  }
  uint4 vb[4], vg[4], vu[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long t = min(t0 + 4 * g + e, T - 1);
    vb[e] = *(const uint4*)(base + t * ldb + kc);
    if constexpr (SWIGLU) {
      vg[e] = *(const uint4*)(gu + t * 2L * K + kc);
      vu[e] = *(const uint4*)(gu + t * 2L * K + K + kc);
    }
  }
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const unsigned* p0 = (const unsigned*)&av[s][0];
    const unsigned* p1 = (const unsigned*)&av[s][1];
    const unsigned* p2 = (const unsigned*)&av[s][2];
    const unsigned* p3 = (const unsigned*)&av[s][3];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // B fragment of tile j: A[4 g .. 4 g + 3][column 8 c + j]
      const int h = j >> 1;
      uint2 b;
      if (j & 1) {
        b.x = (p0[h] >> 16) | (p1[h] & 0xFFFF0000u);
        b.y = (p2[h] >> 16) | (p3[h] & 0xFFFF0000u);
      } else {
        b.x = (p0[h] & 0xFFFFu) | (p1[h] << 16);
        b.y = (p2[h] & 0xFFFFu) | (p3[h] << 16);
      }
      acc[j] = mfma16(da[s], b, acc[j]);
    }
  }
  if (!kok) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long t = t0 + 4 * g + e;
    if (t >= T) break;
    float o[8];
    unpack8(vb[e], o);
    const unsigned bits = drop ? keep8((unsigned long long)t * K + k, seed, thresh) : 0xFFu;
#pragma unroll
    for (int j = 0; j < 8; ++j)  // an explicit fma: the SWIGLU and plain instantiations must round identically
      o[j] = ((bits >> j) & 1u) ? __builtin_fmaf(acc[j][e], dscale, o[j]) : o[j];
    if constexpr (SWIGLU) {  // o = dact (fp32); the same arithmetic as swiglu_bwd_kernel on the bf16-rounded dact
      float gt[8], up[8], dg[8], du[8];
      unpack8(vg[e], gt);
      unpack8(vu[e], up);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        swiglu_grad(bf2f(f2bf(o[j])), gt[j], up[j], dg[j], du[j]);
      }
      *(uint4*)(dx + t * 2L * K + k) = pack8(dg);
      *(uint4*)(dx + t * 2L * K + K + k) = pack8(du);
    } else {
      *(uint4*)(dx + t * (long)K + k) = pack8(o);
    }
  }
}

// Thin token reductions of the adapter backward, one pass over the wide operand:
//   out [splits, R, K] (fp32 partial sums, one slab per token chunk, plain stores) = sum_t S[t, r] * Xd[t, k]
// (lora_grad_out sums the slabs while it scatters them into the gradients: no zero fill and no atomics, which at
// ~3 M fp32 atomics per call for the qkv shapes had made these reductions 3-5x slower than their HBM traffic)
// with Xd = dropout(X) (the forward's mask regenerated from the seed) or X itself.
//   dA    = dxa^T dropout(x):  X = X'[:, :K] (the widened activation), S = dxa [T, R]
//   dB^T  = (s xa)^T dy:       X = dy [T, n],                          S = X'[:, K:K+R] (the adapter columns)
// Workgroup = 64 KT columns of k x a chunk of tc tokens, 64 tokens per stage: the X tile (dropped elements zeroed by
// bit selects; the 1 / (1 - p) scale is applied to the fp32 result) and the S tile go into LDS row-major with 16-byte
// stores, and both MFMA fragments are transposed reads (ds_read_b64_tr_b16: A = X^T rows k, B = S^T rows r, 8
// consecutive tokens per lane); the next stage's global loads are issued before this stage's MFMAs. Wave w owns k
// rows 16 KT w .. 16 KT (w + 1) - 1 of the tile.
__device__ __forceinline__ bf16x8 lds_tr8(const u16* p0, const u16* p1) {
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)p1);
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int RF, int KT>  // KT 16-row k tiles per wave: a workgroup covers 64 KT columns of k
__global__ __launch_bounds__(256) void tsum_kernel(const u16* __restrict__ X, long ldX, const u16* __restrict__ S,
                                                   long ldS, float* __restrict__ out, long T, int K, long tc,
                                                   unsigned thresh, float dscale, unsigned seed, int drop) {
  constexpr int R = 16 * RF, ST = 64, NK = 64 * KT;
  // row pitches padded so that a transposed read's 4 rows x 4 column groups hit distinct banks (pitch = 36 dwords
  // mod 64) and rows stay 16-byte aligned
  constexpr int XP = NK + (KT == 1 ? 8 : 72), SP = R + 8;
  constexpr int TPR = NK / 8, RPP = 256 / TPR, XH = ST / RPP;  // X chunk threads per row, rows per pass, passes
  constexpr int SCH = ST * R / 8, SPT = (SCH + 255) / 256;       // S chunks of 8 per stage, per thread
  __shared__ __attribute__((aligned(16))) u16 xs[ST][XP];
  __shared__ __attribute__((aligned(16))) u16 ss[ST][SP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int k0 = blockIdx.x * NK;
  const long t_begin = (long)blockIdx.y * tc, t_end = min(T, t_begin + tc);
  const int tr = tid / TPR, cx = 8 * (tid % TPR);  // X chunks: rows tr + RPP h of the stage, columns cx .. cx + 7
  const int k = k0 + cx;
  f32x4 acc[KT][RF];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int j = 0; j < RF; ++j) acc[kt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 xv[XH], sv[SPT];
  auto load = [&](uint4 (&xd)[XH], uint4 (&sd)[SPT], long t0) {
#pragma unroll
    for (int h = 0; h < XH; ++h) {
      const long t = t0 + tr + RPP * h;
      xd[h] = (t < t_end && k < K) ? *(const uint4*)(X + t * ldX + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int e = tid + 256 * u, row = e / (R / 8), cc = e - row * (R / 8);
      const long t = t0 + row;
      sd[u] = (e < SCH && t < t_end) ? *(const uint4*)(S + t * ldS + 8 * cc) : make_uint4(0, 0, 0, 0);
    }
  };
  // transposed-read lane addresses: group g reads tokens 8 (g & 1) + 16 (g >> 1)... of a 32-token k-step: rows
  // 8 gg + q (lo) and 8 gg + 4 + q (hi) with gg = g, columns c0 + 4 p
  const int q = r16 >> 2, p = r16 & 3;
  load(xv, sv, t_begin);
  for (long t0 = t_begin; t0 < t_end; t0 += ST) {
    __syncthreads();  // the previous stage's reads are done
#pragma unroll
    for (int h = 0; h < XH; ++h) {
      uint4 v = xv[h];
      if (drop) v = mask8(v, keep8((unsigned long long)(t0 + tr + RPP * h) * K + k, seed, thresh));
      *(uint4*)&xs[tr + RPP * h][cx] = v;
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int e = tid + 256 * u, row = e / (R / 8), cc = e - row * (R / 8);
      if (e < SCH) *(uint4*)&ss[row][8 * cc] = sv[u];
    }
    __syncthreads();
    // the next stage's loads fly under this stage's MFMAs (two / three stages ahead measured slower: r5_run22)
    if (t0 + ST < t_end) load(xv, sv, t0 + ST);
#pragma unroll
    for (int ks = 0; ks < ST / 32; ++ks) {
      const int rl = 32 * ks + 8 * g + q;
      bf16x8 b[RF];
#pragma unroll
      for (int j = 0; j < RF; ++j) b[j] = lds_tr8(&ss[rl][16 * j + 4 * p], &ss[rl + 4][16 * j + 4 * p]);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int c0 = 16 * (KT * w + kt) + 4 * p;
        const bf16x8 a = lds_tr8(&xs[rl][c0], &xs[rl + 4][c0]);
#pragma unroll
        for (int j = 0; j < RF; ++j) acc[kt][j] = mfma(a, b[j], acc[kt][j]);
      }
    }
  }
  // C layout: lane (g, r16) holds rows 4 g + i (k), column r16 (r) of each 16 x 16 block: 4 consecutive k per lane
  float* slab = out + (long)blockIdx.y * R * K;
  const float sc = drop ? dscale : 1.f;  // the dropout scale of the kept elements
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int kk = k0 + 16 * (KT * w + kt) + 4 * g;
    if (kk < K) {  // K % 8 == 0: the lane's 4 columns are all in range or all out
#pragma unroll
      for (int j = 0; j < RF; ++j) *(f32x4*)(slab + (long)(16 * j + r16) * K + kk) = acc[kt][j] * sc;
    }
  }
}

// Scatter blocks of an fp32 [R, K] sum into up to 4 parameter gradients (bf16 or fp32, written or accumulated), one
// launch for all adapters of a projection: output q is rows [r0, r0 + nr) x columns [c0, c0 + nc) of the sum,
// transposed when tr (dB = (dB^T)^T: out[i][j] = sum[r0 + j][c0 + i]).
// sum over the ns slabs (fixed order): eight independent loads in flight per step, not one dependent chain
__device__ __forceinline__ float slab_sum(const float* __restrict__ p, long o, long slab, int ns) {
  float v = 0.f;
  int z = 0;
  for (; z + 8 <= ns; z += 8) {
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = p[o + (z + i) * slab];
#pragma unroll
    for (int i = 0; i < 8; ++i) v += f[i];
  }
  for (; z < ns; ++z) v += p[o + z * slab];
  return v;
}

struct GradOuts {  // up to 8 outputs, each a block of one of two fp32 sums
  const float* sum[2];
  int K[2], ns[2];
  long slab[2];
  void* ptr[8];
  int src[8], tr[8], r0[8], c0[8], nr[8], nc[8];
  int f32[8], acc[8];
};

__global__ __launch_bounds__(256) void grad_out_kernel(GradOuts go) {
  const int q = blockIdx.y;
  const int n = go.nr[q] * go.nc[q];  // elements of output q ([nc, nr] when tr, else [nr, nc])
  const int sq = go.src[q], K = go.K[sq], ns = go.ns[sq];
  const float* __restrict__ sum = go.sum[sq];
  const long slab = go.slab[sq];
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    int i, j;
    float v;
    long oe = e;
    if (go.tr[q]) {  // out [nc][nr]: element (i, j) = sum[r0 + j][c0 + i]; consecutive threads read consecutive i
                     // (the slab reads dominate), the writes go nr elements apart
      j = e / go.nc[q];
      i = e - j * go.nc[q];
      v = slab_sum(sum, (long)(go.r0[q] + j) * K + go.c0[q] + i, slab, ns);
      oe = (long)i * go.nr[q] + j;
    } else {
      i = e / go.nc[q];
      j = e - i * go.nc[q];
      v = slab_sum(sum, (long)(go.r0[q] + i) * K + go.c0[q] + j, slab, ns);
    }
    if (go.f32[q]) {
      float* o = (float*)go.ptr[q] + oe;
      *o = go.acc[q] ? *o + v : v;
    } else {
      u16* o = (u16*)go.ptr[q] + oe;
      *o = f2bf(go.acc[q] ? bf2f(*o) + v : v);
    }
  }
}

// Batched strided 2-D copies of 16-bit elements, one launch for any number of them: row d of the int64 descriptor
// table is {src, dst, rows, cols, src row stride, dst row stride} (pointers as integers, strides in elements).
// ops/fused.py syncs every adapter's B into its wide weight W' and every A into its projection's A_cat with it, once
// per optimizer step for the whole model (it replaced ~7 copy kernels and 2 concatenations per layer and step).
__global__ __launch_bounds__(256) void copy2d_batch_kernel(const long long* __restrict__ desc) {
  const long long* d = desc + 6L * blockIdx.y;
  const u16* src = (const u16*)d[0];
  u16* dst = (u16*)d[1];
  const long rows = d[2], cols = d[3], lds = d[4], ldd = d[5];
  const long n = rows * cols;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += gridDim.x * 256L) {
    const long i = e / cols, j = e - i * cols;
    dst[i * ldd + j] = src[i * lds + j];
  }
}

static unsigned thresh_of(double p, float* dscale) { return drop_thresh16(p, dscale); }

}  // namespace lora

// x [T, K], A [R, K] (R = 16, 32, 48 or 64) -> (X' [T, ldX], xd): xd = dropout(x) [T, K] only with save_xd and
// p > 0, else empty (the backward regenerates the mask from the seed: lora_tsum, lora_bwd_dx). ldX >= K + R (0 = K + R): columns
// [K + R, ldX) are zero (the wide weight's padding to a whole K-tile pair of the HIP GEMMs)
// swiglu: x is gu [T, 2K] and the widened activation is act = silu(gate) * up (see fwd_kernel SW)
namespace lora {
// one widening launch: x rows of stride ldx (copy = 0: x IS X's left block, produced in place by its producer)
static void launch_fwd(const u16* x, long ldx, int copy, const at::Tensor& A, u16* X, u16* xdp, long T, int K, long ldX,
                       double s, double p, int64_t seed, bool swiglu) {
  const int R = A.size(0);
  float dscale;
  const unsigned thresh = thresh_of(p, &dscale);
  const int grid = (int)((T + 15) / 16);
  const u16* Ap = (const u16*)A.data_ptr();
#define LORA_FWD(RF)                                                                                              \
  if (!swiglu && K == 2048)                                                                                       \
    fwd_kernel<RF, false, 4><<<grid, 512, 0, cur_stream()>>>(x, Ap, X, xdp, T, K, ldX, (float)s, thresh, dscale,  \
                                                             (unsigned)seed, p > 0 ? 1 : 0, ldx, copy);           \
  else if (swiglu)                                                                                                \
    fwd_kernel<RF, true><<<grid, 512, 0, cur_stream()>>>(x, Ap, X, xdp, T, K, ldX, (float)s, thresh, dscale,      \
                                                         (unsigned)seed, p > 0 ? 1 : 0, ldx, copy);               \
  else                                                                                                            \
    fwd_kernel<RF, false><<<grid, 512, 0, cur_stream()>>>(x, Ap, X, xdp, T, K, ldX, (float)s, thresh, dscale,     \
                                                          (unsigned)seed, p > 0 ? 1 : 0, ldx, copy)
  switch (R / 16) {
    case 1: LORA_FWD(1); break;
    case 2: LORA_FWD(2); break;
    case 3: LORA_FWD(3); break;
    default: LORA_FWD(4); break;
  }
#undef LORA_FWD
  SFT_LAUNCH_CHECK();
}
}  // namespace lora

std::tuple<at::Tensor, at::Tensor> lora_fwd(const at::Tensor& x, const at::Tensor& A, double s, double p, int64_t seed,
                                            int64_t ldX, bool save_xd, bool swiglu) {
  SFT_CHECK_CUDA(x);
  SFT_CHECK_BF16(x);
  SFT_CHECK_BF16(A);
  SFT_CHECK_CONTIG(x);
  SFT_CHECK_CONTIG(A);
  const long T = x.size(0);
  SFT_CHECK(!swiglu || (x.size(1) % 2 == 0 && !save_xd), "lora_fwd swiglu: gu [T, 2K], no saved dropout(x)");
  const int K = swiglu ? x.size(1) / 2 : x.size(1), R = A.size(0);
  SFT_CHECK(A.size(1) == K && K % 256 == 0 && R % 16 == 0 && R >= 16 && R <= 64, "lora_fwd: shapes");
  if (ldX <= 0) ldX = K + R;
  SFT_CHECK(ldX >= K + R && ldX % 8 == 0, "lora_fwd: ldX >= K + R, multiple of 8");
  auto X = at::empty({T, ldX}, x.options());
  at::Tensor xd = (p > 0 && save_xd) ? at::empty({T, (long)K}, x.options()) : at::empty({0}, x.options());
  if (T == 0) return {X, xd};
  lora::launch_fwd((const u16*)x.data_ptr(), x.size(1), 1, A, (u16*)X.data_ptr(),
                   (p > 0 && save_xd) ? (u16*)xd.data_ptr() : nullptr, T, K, ldX, s, p, seed, swiglu);
  return {X, xd};
}

// The same widening when x already sits in X's left columns (X [T, ldX], x = X[:, :K], written there by its producer:
// the RMSNorm forward's strided output): fills only the adapter columns [K, K + R) and the zero padding.
void lora_fwd_inplace(at::Tensor X, int64_t K, const at::Tensor& A, double s, double p, int64_t seed) {
  SFT_CHECK_CUDA(X);
  SFT_CHECK_BF16(X);
  SFT_CHECK_BF16(A);
  SFT_CHECK_CONTIG(A);
  SFT_CHECK(X.dim() == 2 && X.stride(1) == 1 && X.stride(0) == X.size(1) && (uintptr_t)X.data_ptr() % 16 == 0,
            "lora_fwd_inplace: X [T, ldX] row-contiguous");
  const long T = X.size(0), ldX = X.size(1);
  const int R = A.size(0);
  SFT_CHECK(A.size(1) == K && K % 256 == 0 && R % 16 == 0 && R >= 16 && R <= 64 && ldX >= K + R && ldX % 8 == 0,
            "lora_fwd_inplace: shapes");
  if (T == 0) return;
  lora::launch_fwd((const u16*)X.data_ptr(), ldX, 0, A, (u16*)X.data_ptr(), nullptr, T, (int)K, ldX, s, p, seed,
                   false);
}

// dx = base + keep * (dxa @ A) / (1-p); base [T, K] with row stride ldb (a column slice is fine). With gu [T, 2K]
// (gate | up): returns dgu = swiglu_bwd(dx, gu) [T, 2K] instead.
at::Tensor lora_bwd_dx(const at::Tensor& base, const at::Tensor& dxa, const at::Tensor& A, double p, int64_t seed,
                       const c10::optional<at::Tensor>& gu) {
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
  const bool sw = gu.has_value() && gu->defined();
  if (sw) {
    SFT_CHECK_BF16(*gu);
    SFT_CHECK_CONTIG(*gu);
    SFT_CHECK(gu->size(0) == T && gu->size(1) == 2L * K, "lora_bwd_dx: gu [T, 2K]");
  }
  auto dx = at::empty({T, sw ? 2L * K : (long)K}, base.options());
  if (T == 0) return dx;
  float dscale;
  const unsigned thresh = lora::thresh_of(p, &dscale);
  dim3 grid((K + 511) / 512, (unsigned)((T + 15) / 16));
  SFT_CHECK(grid.y <= 65535u, "lora_bwd_dx: T too large");
#define LORA_BWD(RR)                                                                                              \
  if (sw)                                                                                                         \
    lora::bwd_dx_kernel<RR, true><<<grid, 256, 0, cur_stream()>>>(                                               \
        (const u16*)base.data_ptr(), base.stride(0), (const u16*)dxa.data_ptr(), (const u16*)A.data_ptr(),        \
        (u16*)dx.data_ptr(), T, K, thresh, dscale, (unsigned)seed, p > 0 ? 1 : 0, (const u16*)gu->data_ptr());    \
  else                                                                                                            \
    lora::bwd_dx_kernel<RR, false><<<grid, 256, 0, cur_stream()>>>(                                              \
        (const u16*)base.data_ptr(), base.stride(0), (const u16*)dxa.data_ptr(), (const u16*)A.data_ptr(),        \
        (u16*)dx.data_ptr(), T, K, thresh, dscale, (unsigned)seed, p > 0 ? 1 : 0, nullptr)
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

// dxa [T, R] = s * dy [T, n] . Bc [n, R]  (Bc = the adapters' B columns of the wide weight W', row stride ldb): the
// adapter-dx projection, a thin-N GEMM that is one streaming pass over dy. Workgroup = 32 token rows x all R columns,
// dy streamed in chunks of CH = 256 CW columns: every wave instruction loads 32 CW contiguous 16-byte pieces of one row
// into registers, the chunk goes to an LDS tile [32][CH + 8]; the chunk's Bc rows [CH][R] are loaded 4 n-rows x 8
// columns per thread and written TRANSPOSED into an LDS tile [R][CH + 8] (ds_write_b64 of 4 n-values), so both MFMA
// operands are plain row reads with k = n contiguous (ds_read_b128). Wave w owns columns CH/4 w .. of each chunk (every
// row and R fragment); the 4 waves' fp32 partials are summed through LDS (aliasing the tiles) at the end. The next
// chunk's global loads are issued before this chunk's MFMAs. Faster than hipBLASLt's addmm for the 2048 / 3072-column
// dy of the o / down / qkv adapters (13 / 13 / 24 vs 26 / 25 / 34 us at 8192 tokens); on gate_up's 22016 columns
// every workgroup re-reads all of Bc in 64-byte row pieces, as many bytes as its dy rows, and addmm stays ahead (CW = 1:
// 133 vs 107 us; CW = 2 was slower still, 150 us): ops/fused.py routes only narrow dy here (profiles/r5_lora.md).
namespace lora {
template <int RF, int CW>  // R = 16 RF, chunk = 256 CW columns
__global__ __launch_bounds__(256) void dxa_kernel(const u16* __restrict__ dy, long ldy, const u16* __restrict__ Bc,
                                                  long ldb, u16* __restrict__ out, long T, int n, float s) {
  constexpr int R = 16 * RF, CH = 256 * CW, LD = CH + 8;
  constexpr int XP = 4 * CW;              // dy pieces per thread per chunk
  constexpr int TPR = CH / 8, RPP = 256 / TPR;  // threads per row, rows per pass
  constexpr int BT = R * CH / 32;         // B tasks per chunk (4 n-rows x 8 columns each)
  constexpr int BPT = (BT + 255) / 256;   // per thread
  constexpr int TILES = (32 + R) * LD * 2, RED = 4 * 32 * (R + 4) * 4;
  __shared__ __attribute__((aligned(16))) char smem[TILES > RED ? TILES : RED];
  u16 (*xs)[LD] = reinterpret_cast<u16 (*)[LD]>(smem);
  u16 (*bs)[LD] = reinterpret_cast<u16 (*)[LD]>(smem + 32 * LD * 2);
  float (*red)[32][R + 4] = reinterpret_cast<float (*)[32][R + 4]>(smem);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, ii = lane & 15;
  const long t0 = (long)blockIdx.x * 32;
  const int xr = tid / TPR, xc = 8 * (tid % TPR);  // dy piece: rows xr + RPP q, columns xc .. xc + 7 of the chunk
  uint4 xv[XP], bv[BPT][4];
  auto load = [&](int c0) {
#pragma unroll
    for (int q = 0; q < XP; ++q) {
      const long t = t0 + xr + RPP * q;
      xv[q] = (t < T && c0 + xc < n) ? *(const uint4*)(dy + t * ldy + c0 + xc) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int task = tid + 256 * u, ng = task / (R / 8), rg = task - ng * (R / 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int nn = c0 + 4 * ng + e;
        bv[u][e] = (task < BT && nn < n) ? *(const uint4*)(Bc + (long)nn * ldb + 8 * rg) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  f32x4 acc[2][RF];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < RF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int c0 = 0; c0 < n; c0 += CH) {
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int q = 0; q < XP; ++q) *(uint4*)&xs[xr + RPP * q][xc] = xv[q];
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int task = tid + 256 * u, ng = task / (R / 8), rg = task - ng * (R / 8);
      if (task < BT) {
        const unsigned* b0 = (const unsigned*)&bv[u][0];
        const unsigned* b1 = (const unsigned*)&bv[u][1];
        const unsigned* b2 = (const unsigned*)&bv[u][2];
        const unsigned* b3 = (const unsigned*)&bv[u][3];
#pragma unroll
        for (int h = 0; h < 4; ++h) {  // columns 8 rg + 2 h (low halves) and + 1 (high halves) of the 4 n-rows
          const unsigned lo01 = (b0[h] & 0xFFFFu) | (b1[h] << 16), lo23 = (b2[h] & 0xFFFFu) | (b3[h] << 16);
          const unsigned hi01 = (b0[h] >> 16) | (b1[h] & 0xFFFF0000u), hi23 = (b2[h] >> 16) | (b3[h] & 0xFFFF0000u);
          *(uint2*)&bs[8 * rg + 2 * h][4 * ng] = make_uint2(lo01, lo23);
          *(uint2*)&bs[8 * rg + 2 * h + 1][4 * ng] = make_uint2(hi01, hi23);
        }
      }
    }
    __syncthreads();
    if (c0 + CH < n) load(c0 + CH);  // the next chunk's loads fly under this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < 2 * CW; ++ks) {
      const int kc = (CH / 4) * w + 32 * ks + 8 * g;
      bf16x8 a[2], b[RF];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *(const bf16x8*)&xs[16 * i + ii][kc];
#pragma unroll
      for (int j = 0; j < RF; ++j) b[j] = *(const bf16x8*)&bs[16 * j + ii][kc];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < RF; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
  }
  __syncthreads();  // the tiles are reused for the partial sums
  // C layout: lane (g, ii) holds rows 16 i + 4 g + e, column 16 j + ii
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < RF; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w][16 * i + 4 * g + e][16 * j + ii] = acc[i][j][e];
  __syncthreads();
  for (int o = tid; o < 32 * R / 2; o += 256) {  // two adjacent columns per thread, fixed summation order
    const int row = o / (R / 2), col = 2 * (o - row * (R / 2));
    const long t = t0 + row;
    if (t < T) {
      const float v0 = ((red[0][row][col] + red[1][row][col]) + red[2][row][col]) + red[3][row][col];
      const float v1 = ((red[0][row][col + 1] + red[1][row][col + 1]) + red[2][row][col + 1]) + red[3][row][col + 1];
      *(unsigned*)(out + t * R + col) = pk2bf(v0 * s, v1 * s);
    }
  }
}

// Wide dy (gate_up: n = 22016): Bc = B_blockdiag is zero outside its sub-projections' blocks (rows [o_b, o_b + rows_b)
// x columns [c_b, c_b + r)), so each block's r columns of dxa only need dy's columns [o_b, o_b + rows_b) — half of
// gate_up's dy per output column, and 16 instead of 32 MFMA columns. Work item = 64 token rows x one PIECE of a block's
// n-range (pieces cut so the grid is ~512 workgroups): every workgroup reads its dy rows once and only its piece of Bc
// (the dense kernel above re-read all of Bc per 32 token rows, as many bytes as dy itself). Wave w owns token rows
// 16 w .. 16 w + 15 of the block and the whole chunk (no cross-wave reduction); fp32 partials [piece][T][r] are summed
// per block and scaled by dxa_finish_kernel.
constexpr int DXA_MAXP = 16;
struct DxaPieces {
  int n0[DXA_MAXP], n1[DXA_MAXP], blk[DXA_MAXP];  // dy column range, block index
  int c[4], p0[4], np[4];                          // per block: first dxa column, first piece, pieces
};

template <int RF>  // r = 16 RF columns per block
__global__ __launch_bounds__(256) void dxa_piece_kernel(const u16* __restrict__ dy, long ldy,
                                                        const u16* __restrict__ Bc, long ldb,
                                                        float* __restrict__ part, long T, DxaPieces pc) {
  constexpr int r = 16 * RF, CH = 256, LD = CH + 8, XP = 8, TPR = CH / 8, RPP = 256 / TPR;
  constexpr int BT = r * CH / 32, BPT = (BT + 255) / 256;  // Bc tasks (4 n-rows x 8 columns) per chunk / thread
  __shared__ __attribute__((aligned(16))) u16 xs[64][LD];
  __shared__ __attribute__((aligned(16))) u16 bs[r][LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, ii = lane & 15;
  const long t0 = (long)blockIdx.x * 64;
  const int pi = blockIdx.y, n0 = pc.n0[pi], n1 = pc.n1[pi], cb = pc.c[pc.blk[pi]];
  const int xr = tid / TPR, xc = 8 * (tid % TPR);  // dy piece: rows xr + RPP q, columns xc .. xc + 7 of the chunk
  uint4 xv[XP], bv[BPT][4];
  auto load = [&](int c0) {
#pragma unroll
    for (int q = 0; q < XP; ++q) {
      const long t = t0 + xr + RPP * q;
      xv[q] = (t < T && c0 + xc < n1) ? *(const uint4*)(dy + t * ldy + c0 + xc) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int task = tid + 256 * u, ng = task / (r / 8), rg = task - ng * (r / 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int nn = c0 + 4 * ng + e;
        bv[u][e] = (task < BT && nn < n1) ? *(const uint4*)(Bc + (long)nn * ldb + cb + 8 * rg)
                                          : make_uint4(0, 0, 0, 0);
      }
    }
  };
  f32x4 acc[RF];
#pragma unroll
  for (int j = 0; j < RF; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(n0);
  for (int c0 = n0; c0 < n1; c0 += CH) {
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int q = 0; q < XP; ++q) *(uint4*)&xs[xr + RPP * q][xc] = xv[q];
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int task = tid + 256 * u, ng = task / (r / 8), rg = task - ng * (r / 8);
      if (task < BT) {
        const unsigned* b0 = (const unsigned*)&bv[u][0];
        const unsigned* b1 = (const unsigned*)&bv[u][1];
        const unsigned* b2 = (const unsigned*)&bv[u][2];
        const unsigned* b3 = (const unsigned*)&bv[u][3];
#pragma unroll
        for (int h = 0; h < 4; ++h) {  // columns 8 rg + 2 h (low halves) and + 1 (high halves) of the 4 n-rows
          const unsigned lo01 = (b0[h] & 0xFFFFu) | (b1[h] << 16), lo23 = (b2[h] & 0xFFFFu) | (b3[h] << 16);
          const unsigned hi01 = (b0[h] >> 16) | (b1[h] & 0xFFFF0000u), hi23 = (b2[h] >> 16) | (b3[h] & 0xFFFF0000u);
          *(uint2*)&bs[8 * rg + 2 * h][4 * ng] = make_uint2(lo01, lo23);
          *(uint2*)&bs[8 * rg + 2 * h + 1][4 * ng] = make_uint2(hi01, hi23);
        }
      }
    }
    __syncthreads();
    if (c0 + CH < n1) load(c0 + CH);  // the next chunk's loads fly under this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < CH / 32; ++ks) {
      const int kc = 32 * ks + 8 * g;
      const bf16x8 a = *(const bf16x8*)&xs[16 * w + ii][kc];
#pragma unroll
      for (int j = 0; j < RF; ++j) acc[j] = mfma(a, *(const bf16x8*)&bs[16 * j + ii][kc], acc[j]);
    }
  }
  // C layout: lane (g, ii) holds token rows 16 w + 4 g + e, column 16 j + ii
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long t = t0 + 16 * w + 4 * g + e;
    if (t < T) {
#pragma unroll
      for (int j = 0; j < RF; ++j) part[((long)pi * T + t) * r + 16 * j + ii] = acc[j][e];
    }
  }
}

// dxa[t][c_b + j] = s * (sum of block b's pieces, in piece order)[t][j]; columns outside every block are zero
template <int RF>
__global__ __launch_bounds__(256) void dxa_finish_kernel(const float* __restrict__ part, u16* __restrict__ out,
                                                         long T, int R, int nblk, DxaPieces pc, float s) {
  constexpr int r = 16 * RF;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= T * R) return;
  const long t = e / R;
  const int col = (int)(e - t * R);
  float v = 0.f;
  for (int b = 0; b < nblk; ++b) {
    const int j = col - pc.c[b];
    if (j >= 0 && j < r) {
      for (int q = 0; q < pc.np[b]; ++q) v += part[((long)(pc.p0[b] + q) * T + t) * r + j];
    }
  }
  out[e] = f2bf(v * s);
}
}  // namespace lora

// out [splits, R, K] fp32 partial sums (over token chunks; lora_grad_out or .sum(0) adds them) of S^T dropout(X[:, :K]) (the mask regenerated from seed when p > 0); X rows of stride >= K, S [T, R]
// (a column slice of a wider tensor is fine)
// dxa [T, R] = s dy [T, n] . Bc [n, R]; Bc may be a column slice of a wider weight (row stride Bc.stride(0))
at::Tensor lora_dxa(const at::Tensor& dy, const at::Tensor& Bc, double s) {
  SFT_CHECK_CUDA(dy);
  SFT_CHECK_BF16(dy);
  SFT_CHECK_BF16(Bc);
  const long T = dy.size(0);
  const int n = dy.size(1), R = Bc.size(1);
  SFT_CHECK(dy.stride(1) == 1 && dy.stride(0) % 8 == 0 && (uintptr_t)dy.data_ptr() % 16 == 0 && n % 8 == 0,
            "lora_dxa: dy rows 16-byte aligned");
  SFT_CHECK(Bc.size(0) == n && Bc.stride(1) == 1 && Bc.stride(0) % 8 == 0 && (uintptr_t)Bc.data_ptr() % 16 == 0,
            "lora_dxa: Bc [n, R] with 16-byte aligned rows");
  SFT_CHECK(R % 16 == 0 && R >= 16 && R <= 64, "lora_dxa: R in 16..64, multiple of 16");
  auto out = at::empty({T, R}, dy.options());
  if (T == 0) return out;
  const unsigned grid = (unsigned)((T + 31) / 32);
#define LORA_DXA(RF)                                                                                              \
  lora::dxa_kernel<RF, 1><<<grid, 256, 0, cur_stream()>>>((const u16*)dy.data_ptr(), dy.stride(0),                \
      (const u16*)Bc.data_ptr(), Bc.stride(0), (u16*)out.data_ptr(), T, n, (float)s)
  switch (R / 16) {
    case 1: LORA_DXA(1); break;
    case 2: LORA_DXA(2); break;
    case 3: LORA_DXA(3); break;
    default: LORA_DXA(4); break;
  }
#undef LORA_DXA
  SFT_LAUNCH_CHECK();
  return out;
}

// The same product when Bc is block-diagonal: block b = rows [o[b], o[b] + rows[b]) x columns [c[b], c[b] + r) of Bc,
// every other element zero (the wide weight's B_blockdiag; the caller guarantees it). Up to 4 blocks.
at::Tensor lora_dxa_blocks(const at::Tensor& dy, const at::Tensor& Bc, at::IntArrayRef o, at::IntArrayRef rows,
                           at::IntArrayRef c, int64_t r, double s) {
  SFT_CHECK_CUDA(dy);
  SFT_CHECK_BF16(dy);
  SFT_CHECK_BF16(Bc);
  const long T = dy.size(0);
  const int n = dy.size(1), R = Bc.size(1), nb = o.size();
  SFT_CHECK(dy.stride(1) == 1 && dy.stride(0) % 8 == 0 && (uintptr_t)dy.data_ptr() % 16 == 0 && n % 8 == 0,
            "lora_dxa_blocks: dy rows 16-byte aligned");
  SFT_CHECK(Bc.size(0) == n && Bc.stride(1) == 1 && Bc.stride(0) % 8 == 0 && (uintptr_t)Bc.data_ptr() % 16 == 0,
            "lora_dxa_blocks: Bc [n, R] with 16-byte aligned rows");
  SFT_CHECK(nb >= 1 && nb <= 4 && (int)rows.size() == nb && (int)c.size() == nb && (r == 16 || r == 32),
            "lora_dxa_blocks: 1..4 blocks of rank 16 or 32");
  long total = 0;
  for (int b = 0; b < nb; ++b) {
    SFT_CHECK(o[b] >= 0 && rows[b] > 0 && o[b] + rows[b] <= n && o[b] % 8 == 0 && c[b] >= 0 && c[b] + r <= R &&
                  c[b] % 8 == 0, "lora_dxa_blocks: block out of range / misaligned");
    total += rows[b];
  }
  auto out = at::empty({T, R}, dy.options());
  if (T == 0) return out;
  // pieces: ~512 workgroups over the token blocks, piece sizes a multiple of the 256-column chunk
  const long tb = (T + 63) / 64;
  lora::DxaPieces pc{};
  int np = 0;
  // piece sizes per block (a multiple of the chunk): the largest target that keeps every piece in the table
  for (long want = std::max<long>(nb, std::min<long>(lora::DXA_MAXP, (512 + tb - 1) / tb)); want >= 1; --want) {
    long sz[4], count = 0;
    for (int b = 0; b < nb; ++b) {
      const long pb = std::max<long>(1, (want * rows[b] + total - 1) / total);
      sz[b] = ((rows[b] + pb - 1) / pb + 255) / 256 * 256;
      count += (rows[b] + sz[b] - 1) / sz[b];
    }
    if (count > lora::DXA_MAXP) continue;
    for (int b = 0; b < nb; ++b) {
      pc.c[b] = (int)c[b];
      pc.p0[b] = np;
      for (long a = 0; a < rows[b]; a += sz[b]) {
        pc.n0[np] = (int)(o[b] + a);
        pc.n1[np] = (int)(o[b] + std::min(rows[b], a + sz[b]));
        pc.blk[np] = b;
        ++np;
      }
      pc.np[b] = np - pc.p0[b];
    }
    break;
  }
  SFT_CHECK(np >= nb, "lora_dxa_blocks: piece table");
  auto part = at::empty({(long)np, T, r}, dy.options().dtype(at::kFloat));
  dim3 grid((unsigned)tb, (unsigned)np);
  const unsigned fgrid = (unsigned)((T * R + 255) / 256);
  if (r == 16) {
    lora::dxa_piece_kernel<1><<<grid, 256, 0, cur_stream()>>>((const u16*)dy.data_ptr(), dy.stride(0),
        (const u16*)Bc.data_ptr(), Bc.stride(0), part.data_ptr<float>(), T, pc);
    SFT_LAUNCH_CHECK();
    lora::dxa_finish_kernel<1><<<fgrid, 256, 0, cur_stream()>>>(part.data_ptr<float>(), (u16*)out.data_ptr(), T, R,
                                                                nb, pc, (float)s);
  } else {
    lora::dxa_piece_kernel<2><<<grid, 256, 0, cur_stream()>>>((const u16*)dy.data_ptr(), dy.stride(0),
        (const u16*)Bc.data_ptr(), Bc.stride(0), part.data_ptr<float>(), T, pc);
    SFT_LAUNCH_CHECK();
    lora::dxa_finish_kernel<2><<<fgrid, 256, 0, cur_stream()>>>(part.data_ptr<float>(), (u16*)out.data_ptr(), T, R,
                                                                nb, pc, (float)s);
  }
  SFT_LAUNCH_CHECK();
  return out;
}

at::Tensor lora_tsum(const at::Tensor& X, int64_t K, const at::Tensor& S, double p, int64_t seed) {
  SFT_CHECK_CUDA(X);
  SFT_CHECK_BF16(X);
  SFT_CHECK_BF16(S);
  const long T = X.size(0);
  const int R = S.size(1);
  SFT_CHECK(X.stride(1) == 1 && X.stride(0) % 8 == 0 && X.size(1) >= K && K % 8 == 0, "lora_tsum: X layout");
  SFT_CHECK(S.stride(1) == 1 && S.stride(0) % 8 == 0 && (uintptr_t)S.data_ptr() % 16 == 0, "lora_tsum: S layout");
  SFT_CHECK(S.size(0) == T && R % 16 == 0 && R >= 16 && R <= 64, "lora_tsum: S [T, R], R in 16..64");
  if (T == 0) return at::zeros({1, R, K}, X.options().dtype(at::kFloat));
  float dscale;
  const unsigned thresh = lora::thresh_of(p, &dscale);
  // wide operands (K >= 8192: the down projection's dA, gate_up's dB) take 256-column workgroups, each wave
  // instruction reading 2 rows x 512 B (64-column ones read 8 rows x 128 B), on about 512 workgroups; the rest
  // 64-column ones on about 1024. The token range is split into chunks of whole 64-token stages.
  const bool wide = K >= 8192;
  const int nk = wide ? 256 : 64, nkb = (int)((K + nk - 1) / nk);
  // (768 / 1024 workgroups for the dropout-regenerating wide dA measured neutral in the LoRA step, r5_run16; wave-private
  // stages — each wave loading its own 64 columns and S copy, no barriers — 37.3 vs 38.0 us for dA but 74.1 vs 68.0
  // for gate_up's dB^T, r5_run20: not kept)
  long splits = std::max(1L, std::min((T + 63) / 64, (wide ? 512L : 1024L) / nkb));
  const long tc = ((T + splits - 1) / splits + 63) / 64 * 64;
  splits = (T + tc - 1) / tc;
  auto out = at::empty({splits, R, K}, X.options().dtype(at::kFloat));  // every element written by one workgroup
  dim3 grid(nkb, (unsigned)splits);
#define LORA_TSUM(RF)                                                                                             \
  if (wide)                                                                                                       \
    lora::tsum_kernel<RF, 4><<<grid, 256, 0, cur_stream()>>>((const u16*)X.data_ptr(), X.stride(0),              \
        (const u16*)S.data_ptr(), S.stride(0), out.data_ptr<float>(), T, (int)K, tc, thresh, dscale,             \
        (unsigned)seed, p > 0 ? 1 : 0);                                                                          \
  else                                                                                                            \
    lora::tsum_kernel<RF, 1><<<grid, 256, 0, cur_stream()>>>((const u16*)X.data_ptr(), X.stride(0),              \
        (const u16*)S.data_ptr(), S.stride(0), out.data_ptr<float>(), T, (int)K, tc, thresh, dscale,             \
        (unsigned)seed, p > 0 ? 1 : 0)
  switch (R / 16) {
    case 1: LORA_TSUM(1); break;
    case 2: LORA_TSUM(2); break;
    case 3: LORA_TSUM(3); break;
    default: LORA_TSUM(4); break;
  }
#undef LORA_TSUM
  SFT_LAUNCH_CHECK();
  return out;
}

// outs[q] (+)= block q of sum ([R, K] fp32, or [splits, R, K] slabs summed on the fly): rows [r0[q], +nr), columns
// [c0[q], +nc), transposed when tr. lora_grad_out2 does two such groups (a projection's dB^T and dA sums) in ONE
// launch.
namespace lora {
static void add_group(GradOuts& go, int& n, long& most, int g, const at::Tensor& sum, at::TensorList outs,
                      at::IntArrayRef r0, at::IntArrayRef c0, bool tr, at::IntArrayRef accumulate) {
  SFT_CHECK(sum.scalar_type() == at::kFloat && sum.is_contiguous() && (sum.dim() == 2 || sum.dim() == 3),
            "lora_grad_out: fp32 [R, K] or [splits, R, K]");
  const int m = outs.size();
  SFT_CHECK(m >= 1 && n + m <= 8 && (int)r0.size() == m && (int)c0.size() == m && (int)accumulate.size() == m,
            "lora_grad_out: 1..4 outputs per sum");
  const int R = sum.size(sum.dim() - 2), K = sum.size(sum.dim() - 1);
  go.sum[g] = sum.data_ptr<float>();
  go.K[g] = K;
  go.ns[g] = sum.dim() == 3 ? sum.size(0) : 1;
  go.slab[g] = (long)R * K;
  for (int i = 0; i < m; ++i, ++n) {
    const at::Tensor& o = outs[i];
    SFT_CHECK(o.is_contiguous() && o.dim() == 2 &&
                  (o.scalar_type() == at::kBFloat16 || o.scalar_type() == at::kFloat), "lora_grad_out: contiguous bf16 / fp32 2-D outputs");
    const int nr = tr ? o.size(1) : o.size(0), nc = tr ? o.size(0) : o.size(1);
    SFT_CHECK(r0[i] >= 0 && r0[i] + nr <= R && c0[i] >= 0 && c0[i] + nc <= K, "lora_grad_out: block out of range");
    go.ptr[n] = o.data_ptr();
    go.src[n] = g;
    go.tr[n] = tr ? 1 : 0;
    go.r0[n] = (int)r0[i];
    go.c0[n] = (int)c0[i];
    go.nr[n] = nr;
    go.nc[n] = nc;
    go.f32[n] = o.scalar_type() == at::kFloat;
    go.acc[n] = accumulate[i] != 0;
    most = std::max(most, (long)nr * nc);
  }
}

static void launch_grad_out(const GradOuts& go, int n, long most) {
  dim3 grid((unsigned)std::min(1024L, (most + 255) / 256), (unsigned)n);
  grad_out_kernel<<<grid, 256, 0, cur_stream()>>>(go);
  SFT_LAUNCH_CHECK();
}
}  // namespace lora

void lora_grad_out(const at::Tensor& sum, at::TensorList outs, at::IntArrayRef r0, at::IntArrayRef c0, bool tr,
                   at::IntArrayRef accumulate) {
  lora::GradOuts go{};
  int n = 0;
  long most = 0;
  lora::add_group(go, n, most, 0, sum, outs, r0, c0, tr, accumulate);
  lora::launch_grad_out(go, n, most);
}

void lora_grad_out2(const at::Tensor& sa, at::TensorList oa, at::IntArrayRef ra, at::IntArrayRef ca, bool ta,
                    at::IntArrayRef aa, const at::Tensor& sb, at::TensorList ob, at::IntArrayRef rb,
                    at::IntArrayRef cb, bool tb, at::IntArrayRef ab) {
  lora::GradOuts go{};
  int n = 0;
  long most = 0;
  lora::add_group(go, n, most, 0, sa, oa, ra, ca, ta, aa);
  lora::add_group(go, n, most, 1, sb, ob, rb, cb, tb, ab);
  lora::launch_grad_out(go, n, most);
}

// desc: int64 [n, 6] device table (see copy2d_batch_kernel); max_elems: the largest rows * cols in it
void copy2d_batch(const at::Tensor& desc, int64_t max_elems) {
  SFT_CHECK_CUDA(desc);
  SFT_CHECK(desc.scalar_type() == at::kLong && desc.is_contiguous() && desc.dim() == 2 && desc.size(1) == 6,
            "copy2d_batch: int64 [n, 6] descriptors");
  const long n = desc.size(0);
  SFT_CHECK(n <= 65535, "copy2d_batch: at most 65535 copies per launch");
  if (n == 0 || max_elems <= 0) return;
  dim3 grid((unsigned)std::min(64L, (long)((max_elems + 255) / 256)), (unsigned)n);
  lora::copy2d_batch_kernel<<<grid, 256, 0, cur_stream()>>>((const long long*)desc.data_ptr());
  SFT_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("lora_fwd", &lora_fwd);
  m.impl("copy2d_batch", &copy2d_batch);
  m.impl("lora_bwd_dx", &lora_bwd_dx);
  m.impl("lora_tsum", &lora_tsum);
  m.impl("lora_fwd_inplace", &lora_fwd_inplace);
  m.impl("lora_dxa", &lora_dxa);
  m.impl("lora_dxa_blocks", &lora_dxa_blocks);
  m.impl("lora_grad_out", &lora_grad_out);
  m.impl("lora_grad_out2", &lora_grad_out2);
}

}  // namespace sftamd
