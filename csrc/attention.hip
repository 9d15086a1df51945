// Varlen causal GQA flash-attention forward/backward for gfx950.
//
// Layout: the packed QKV GEMM output qkv[M, (nq + 2*nkv) * 128] (bf16, token-major, no
// transposes anywhere); sequences are [cu[b], cu[b+1]). Output o[M, nq*128], lse[nq, M] (fp32,
// natural log). Backward returns dqkv in the same packed layout, ready for the fused QKV
// linear's backward.
//
// CDNA4 mapping:
// * MFMA v_mfma_f32_16x16x32_bf16 throughout (wave64; lane maps below), fp32 accumulate;
// * "swapped" products (S^T = K Q^T, dP^T = V dO^T, ...) put the reduction index of the next
//   product in the accumulator registers, so P / dS feed the next MFMA straight from
//   registers (cvt to bf16, no LDS round trip, no cross-lane shuffles);
// * K/V/Q/dO tiles are staged in LDS as [rows][128] bf16 images with an XOR swizzle that is
//   conflict-free for both 16-byte row reads (MFMA operands along head_dim) and the gfx950
//   transposed read ds_read_b64_tr_b16 (MFMA operands along the key/query axis);
// * online softmax in the exp2 domain with fp32 running max/sum per query row; the four lanes
//   that share a query column combine with two xor-shuffles.
//
// mfma_f32_16x16x32_bf16 lane maps (g = lane >> 4, r = lane & 15, j = 0..7, i = 0..3):
//   A[row r][k 8g+j], B[k 8g+j][col r], C[row 4g+i][col r].
// Accumulator-as-operand: two 16-row C tiles (t0, t1) give lane (g, r) the k values
//   {4g+i} from t0 and {16+4g+i} from t1; we use that order as the k permutation
//   p(8g+j) = j<4 ? 4g+j : 16+4g+(j-4) on BOTH operands of the next MFMA.
#include "common.h"

#include <cstring>

namespace sftamd {

namespace attn {

constexpr int D = 128;       // head_dim (SmolLM3-3B, Llama-3-8B)
constexpr int ROWB = D * 2;  // bytes per LDS image row
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// 16-byte chunk swizzle of the [rows][128] bf16 images (256-B rows = one LDS bank row):
// ch ^ ((row & 3) << 2 | S((row >> 2) & 3)), S = {0, 2, 3, 1}. Checked exhaustively (tools/lds_swizzle_check.py)
// against the MI355X lane groups: conflict-free for the 16-B row reads (ds_read_b128 groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) AND for the transposed ds_read_b64_tr_b16 reads (2 x 32 lanes);
// the previous S(q) = q was 2-way on both.
__device__ __forceinline__ int swz(int row, int ch) {
  return ch ^ (((row & 3) << 2) | ((0x78 >> (2 * ((row >> 2) & 3))) & 3));
}
__device__ __forceinline__ int img_off(int row, int ch) { return row * ROWB + 16 * swz(row, ch); }

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Stage rows [0, R) of a row-major global matrix (row stride ld elements) into an LDS image.
// Rows >= nvalid are zero-filled (never read from HBM).
template <int R, int NT>
__device__ __forceinline__ void stage(char* lds, const u16* __restrict__ g, long ld, int nvalid, int tid) {
#pragma unroll
  for (int it = 0; it < (R * 16) / NT; ++it) {
    const int idx = tid + it * NT;
    const int r = idx >> 4, ch = idx & 15;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nvalid) v = *(const uint4*)(g + (long)r * ld + ch * 8);
    *(uint4*)(lds + img_off(r, ch)) = v;
  }
}

// Operand along head_dim: rows rbase + (lane & 15), k-step s covers d = 32s .. 32s+31.
__device__ __forceinline__ bf16x8 frag_row(const char* lds, int rbase, int s, int lane) {
  return *(const bf16x8*)(lds + img_off(rbase + (lane & 15), 4 * s + (lane >> 4)));
}

// Operand along the row axis (transposed): lane gets column 16*cb + (lane & 15) of rows
// rb + p(8g + j) (the accumulator permutation above). Two ds_read_b64_tr_b16.
template <bool TR>
__device__ __forceinline__ bf16x8 frag_tr(const char* lds, int rb, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (TR) {
    const int q = i >> 2, p = i & 3;
    const int ch = 2 * cb + (p >> 1);
    const int r0 = rb + 4 * g + q;
    const int o0 = img_off(r0, ch) + 8 * (p & 1);
    const int o1 = img_off(r0 + 16, ch) + 8 * (p & 1);
    typedef __attribute__((address_space(3))) s16x4 lds_s4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + o0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + o1));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  } else {
    const int col = 16 * cb + i;
    const int ch = col >> 3, e = col & 7;
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = rb + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
      v[j] = *(const short*)(lds + img_off(row, ch) + 2 * e);
    }
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ bf16x8 pack_acc(const f32x4& t0, const f32x4& t1) {
  bf16x8 r;
  r[0] = (__bf16)t0[0];
  r[1] = (__bf16)t0[1];
  r[2] = (__bf16)t0[2];
  r[3] = (__bf16)t0[3];
  r[4] = (__bf16)t1[0];
  r[5] = (__bf16)t1[1];
  r[6] = (__bf16)t1[2];
  r[7] = (__bf16)t1[3];
  return r;
}

__device__ __forceinline__ bf16x8 load_frag_global(const u16* p, bool ok) {
  if (!ok) return bf16x8{};
  return __builtin_bit_cast(bf16x8, *(const uint4*)p);
}

__device__ __forceinline__ void store4(u16* p, const f32x4& v, float s) {
  uint2 w;
  w.x = (unsigned)f2bf(v[0] * s) | ((unsigned)f2bf(v[1] * s) << 16);
  w.y = (unsigned)f2bf(v[2] * s) | ((unsigned)f2bf(v[3] * s) << 16);
  *(uint2*)p = w;
}

// Store a lane's 8 x 4 head-dim values (columns 16 dt + 4g + i, p = row + 4g) with the rotate_half RoPE inverted
// first — the backward of the forward rotation (x1, x2) -> (x1 c - x2 s, x2 c + x1 s) is
// (g1, g2) -> (g1 c + g2 s, g2 c - g1 s). Columns c and c + 64 of a pair sit in the same lane (dt and dt + 4), so
// the rotation is in-register, on the fp32 accumulators before the single bf16 rounding. cs / sn: this row's
// [64] fp32 cos / sin table + 4g.
__device__ __forceinline__ void store4_rope_bwd(u16* p, const f32x4 (&v)[8], float s, const float* cs, const float* sn) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const float4 c4 = *(const float4*)(cs + 16 * dt), s4 = *(const float4*)(sn + 16 * dt);
    const float c[4] = {c4.x, c4.y, c4.z, c4.w}, n[4] = {s4.x, s4.y, s4.z, s4.w};
    f32x4 lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = v[dt][i] * s, b = v[dt + 4][i] * s;
      lo[i] = a * c[i] + b * n[i];
      hi[i] = b * c[i] - a * n[i];
    }
    store4(p + 16 * dt, lo, 1.f);
    store4(p + 16 * dt + 64, hi, 1.f);
  }
}

// ------------------------------------------------------------------------------ forward
// grid (q-blocks of 64, nq, nseq); 4 waves x 16 query rows. Per 64-key tile: S^T (16 MFMA),
// online softmax in registers, O^T += V^T P^T (16 MFMA).
template <bool TR>
__global__ __launch_bounds__(256) void fwd_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                  float* __restrict__ lse, const int* __restrict__ cu, int nq, int nkv,
                                                  int total, float sl2, int causal) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * ROWB];
  char* Ks = smem;
  char* Vs = smem + 64 * ROWB;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int q0 = qb * 64;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int qrow = q0 + wave * 16 + (lane & 15);
  const bool qok = qrow < len;
  const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load_frag_global(qp + 32 * s, qok);

  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min(qb + 1, nkb) : nkb;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const int kvalid = min(64, len - k0);
    __syncthreads();
    stage<64, 256>(Ks, qkv + (long)(start + k0) * ld + (nq + kvh) * D, ld, kvalid, tid);
    stage<64, 256>(Vs, qkv + (long)(start + k0) * ld + (nq + nkv + kvh) * D, ld, kvalid, tid);
    __syncthreads();
    f32x4 sc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) sc[nt] = mfma(frag_row(Ks, 16 * nt, s, lane), qf[s], sc[nt]);
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * nt + 4 * g + i;
        float v = sc[nt][i] * sl2;
        if (key >= len || (causal && key > qrow)) v = -INFINITY;
        sc[nt][i] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);
    float rs = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(sc[nt][i] - mnew);
        sc[nt][i] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) o[dt] = mfma(frag_tr<TR>(Vs, 32 * ks, dt, lane), pb, o[dt]);
    }
  }
  if (qok) {
    const float inv = 1.f / l;
    u16* op = out + (long)(start + qrow) * nq * D + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(op + 16 * dt, o[dt], inv);
    if (g == 0) lse[(long)h * total + start + qrow] = (m + log2f(l)) * LN2;
  }
}

// ------------------------------------------------------------------------------ backward
// delta[h][m] = sum_d dO[m, h*D + d] * O[m, h*D + d]   (16 lanes per row)
__global__ __launch_bounds__(256) void delta_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                    float* __restrict__ delta, int total, int nq) {
  const long rowid = blockIdx.x * 16L + (threadIdx.x >> 4);  // (m, h) flattened as m*nq + h
  const int sub = threadIdx.x & 15;
  float s = 0.f;
  const bool ok = rowid < (long)total * nq;
  if (ok) {
    const long base = rowid * D + sub * 8;
    float a[8], c[8];
    unpack8(*(const uint4*)(dout + base), a);
    unpack8(*(const uint4*)(out + base), c);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] * c[i];
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
  if (ok && sub == 0) {
    const long m = rowid / nq;
    const int h = (int)(rowid - m * nq);
    delta[(long)h * total + m] = s;
  }
}

// dK/dV: grid (key blocks of 64, nkv, nseq); wave owns 16 keys (K, V fragments in registers,
// dK^T/dV^T accumulators in registers); loops over the GQA group's query heads and 64-row
// query tiles: S, dP (32 MFMA) -> P, dS -> dV^T += dO^T P, dK^T += Q^T dS (32 MFMA).
template <bool TR>
__global__ __launch_bounds__(256) void bwd_dkdv_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                       const float* __restrict__ lse, const float* __restrict__ delta,
                                                       const int* __restrict__ cu, u16* __restrict__ dqkv, int nq,
                                                       int nkv, int total, float sl2, float scale, int causal) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * ROWB + 2 * 64 * 4];
  char* Qs = smem;
  char* Os = smem + 64 * ROWB;
  float* Ls = (float*)(smem + 2 * 64 * ROWB);
  float* Dl = Ls + 64;
  const int kb = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int k0 = kb * 64;
  if (k0 >= len) return;
  const int rep = nq / nkv;
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int key = k0 + wave * 16 + (lane & 15);
  const bool kok = key < len;
  bf16x8 kf[4], vf[4];
  {
    const u16* kp = qkv + (long)(start + key) * ld + (nq + kvh) * D + 8 * g;
    const u16* vp = qkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = load_frag_global(kp + 32 * s, kok);
      vf[s] = load_frag_global(vp + 32 * s, kok);
    }
  }
  f32x4 dk[8], dv[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int qt0 = causal ? kb : 0;
  const int nqt = (len + 63) / 64;
  for (int r = 0; r < rep; ++r) {
    const int h = kvh * rep + r;
    for (int qt = qt0; qt < nqt; ++qt) {
      const int q0 = qt * 64;
      const int qvalid = min(64, len - q0);
      __syncthreads();
      stage<64, 256>(Qs, qkv + (long)(start + q0) * ld + h * D, ld, qvalid, tid);
      stage<64, 256>(Os, dout + (long)(start + q0) * ldo + h * D, ldo, qvalid, tid);
      if (tid < 64) {
        const bool ok = tid < qvalid;
        Ls[tid] = ok ? lse[(long)h * total + start + q0 + tid] * LOG2E : 0.f;
        Dl[tid] = ok ? delta[(long)h * total + start + q0 + tid] : 0.f;
      }
      __syncthreads();
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc[mt] = mfma(frag_row(Qs, 16 * mt, s, lane), kf[s], sc[mt]);
          dp[mt] = mfma(frag_row(Os, 16 * mt, s, lane), vf[s], dp[mt]);
        }
      }
      // lane: key column, query rows q0 + 16mt + 4g + i
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qi = 16 * mt + 4 * g + i;
          const int q = q0 + qi;
          float p = exp2f(sc[mt][i] * sl2 - Ls[qi]);
          if (q >= len || (causal && key > q)) p = 0.f;
          sc[mt][i] = p;
          dp[mt][i] = p * (dp[mt][i] - Dl[qi]);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
        const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          dv[dt] = mfma(frag_tr<TR>(Os, 32 * ks, dt, lane), pb, dv[dt]);
          dk[dt] = mfma(frag_tr<TR>(Qs, 32 * ks, dt, lane), db, dk[dt]);
        }
      }
    }
  }
  if (kok) {
    u16* kp = dqkv + (long)(start + key) * ld + (nq + kvh) * D + 4 * g;
    u16* vp = dqkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      store4(kp + 16 * dt, dk[dt], scale);
      store4(vp + 16 * dt, dv[dt], 1.f);
    }
  }
}

// dQ: grid (q blocks of 64, nq, nseq); wave owns 16 query rows (Q, dO fragments in registers);
// per 64-key tile: S^T, dP^T (32 MFMA) -> dS^T -> dQ^T += K^T dS^T (16 MFMA).
template <bool TR>
__global__ __launch_bounds__(256) void bwd_dq_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     const int* __restrict__ cu, u16* __restrict__ dqkv, int nq,
                                                     int nkv, int total, float sl2, float scale, int causal) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * ROWB];
  char* Ks = smem;
  char* Vs = smem + 64 * ROWB;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int q0 = qb * 64;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int qrow = q0 + wave * 16 + (lane & 15);
  const bool qok = qrow < len;
  bf16x8 qf[4], df[4];
  {
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
    const u16* dp = dout + (long)(start + qrow) * ldo + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = load_frag_global(qp + 32 * s, qok);
      df[s] = load_frag_global(dp + 32 * s, qok);
    }
  }
  const float lse2 = qok ? lse[(long)h * total + start + qrow] * LOG2E : 0.f;
  const float dl = qok ? delta[(long)h * total + start + qrow] : 0.f;
  f32x4 dq[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min(qb + 1, nkb) : nkb;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const int kvalid = min(64, len - k0);
    __syncthreads();
    stage<64, 256>(Ks, qkv + (long)(start + k0) * ld + (nq + kvh) * D, ld, kvalid, tid);
    stage<64, 256>(Vs, qkv + (long)(start + k0) * ld + (nq + nkv + kvh) * D, ld, kvalid, tid);
    __syncthreads();
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc[nt] = mfma(frag_row(Ks, 16 * nt, s, lane), qf[s], sc[nt]);
        dp[nt] = mfma(frag_row(Vs, 16 * nt, s, lane), df[s], dp[nt]);
      }
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * nt + 4 * g + i;
        float p = exp2f(sc[nt][i] * sl2 - lse2);
        if (key >= len || (causal && key > qrow) || !qok) p = 0.f;
        dp[nt][i] = p * (dp[nt][i] - dl);
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) dq[dt] = mfma(frag_tr<TR>(Ks, 32 * ks, dt, lane), db, dq[dt]);
    }
  }
  if (qok) {
    u16* qp = dqkv + (long)(start + qrow) * ld + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(qp + 16 * dt, dq[dt], scale);
  }
}


// ============================================================================== v2 kernels
// Same math and lane maps as v1, restructured for latency hiding on CDNA4:
// * K/V (fwd, dQ) and Q/dO (dK/dV) tiles are double-buffered in LDS; the next tile is issued
//   global->registers BEFORE the current tile's MFMAs and written to the other LDS buffer after
//   them (T14 async-STAGE split), so HBM/L2 latency hides under compute; one barrier per tile;
// * fwd/dQ use 8-wave (512-thread) workgroups over 128 query rows, halving K/V staging per row
//   and giving two waves per SIMD; waves whose 16 rows are entirely below a causal key tile skip
//   its MFMAs (wave-uniform branch);
// * dK/dV is split over the query heads of a GQA group (4x the workgroups, no causal tail of
//   32 sequential tiles): each workgroup writes an fp32 partial slab, and a vectorised reduce
//   kernel sums the rep partials in a fixed order (deterministic) straight into packed dqkv.

template <int R, int NT>
struct TileRegs {
  static constexpr int N = (R * 16) / NT;
  uint4 v[N];
  __device__ __forceinline__ void load(const u16* __restrict__ g, long ld, int nvalid, int tid) {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int idx = tid + it * NT;
      const int r = idx >> 4, ch = idx & 15;
      v[it] = make_uint4(0, 0, 0, 0);
      if (r < nvalid) v[it] = *(const uint4*)(g + (long)r * ld + ch * 8);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int idx = tid + it * NT;
      *(uint4*)(lds + img_off(idx >> 4, idx & 15)) = v[it];
    }
  }
};

template <bool TR, int NW, int NBUF>
__global__ __launch_bounds__(NW * 64) void fwd2_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                       float* __restrict__ lse, const int* __restrict__ cu, int nq,
                                                       int nkv, int total, float sl2, int causal) {
  constexpr int NT = NW * 64, BM = NW * 16, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * NBUF * TB];  // K0 V0 (K1 V1)
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * BM;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int qrow = q0 + wave * 16 + (lane & 15);
  const int wlast = q0 + wave * 16 + 15;  // last query row of this wave
  const bool qok = qrow < len;
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* vbase = qkv + (long)start * ld + (nq + nkv + kvh) * D;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  {
    TileRegs<64, NT> tk, tv;
    tk.load(kbase, ld, min(64, len), tid);
    tv.load(vbase, ld, min(64, len), tid);
    tk.store(smem, tid);
    tv.store(smem + TB, tid);
  }
  bf16x8 qf[4];
  {
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = load_frag_global(qp + 32 * s, qok);
  }
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    char* Ks = smem + (NBUF == 2 ? (kt & 1) : 0) * 2 * TB;
    char* Vs = Ks + TB;
    const bool pre = kt + 1 < nkt;
    TileRegs<64, NT> tk, tv;
    if (pre) {
      const int kv = min(64, len - k0 - 64);
      tk.load(kbase + (long)(k0 + 64) * ld, ld, kv, tid);
      tv.load(vbase + (long)(k0 + 64) * ld, ld, kv, tid);
    }
    if (!causal || k0 <= wlast) {
      f32x4 sc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) sc[nt] = mfma(frag_row(Ks, 16 * nt, s, lane), qf[s], sc[nt]);
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = k0 + 16 * nt + 4 * g + i;
          float v = sc[nt][i] * sl2;
          if (key >= len || (causal && key > qrow)) v = -INFINITY;
          sc[nt][i] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(m, tmax);
      const float alpha = exp2f(m - mnew);
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = exp2f(sc[nt][i] - mnew);
          sc[nt][i] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      m = mnew;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[dt] = mfma(frag_tr<TR>(Vs, 32 * ks, dt, lane), pb, o[dt]);
      }
    }
    if (pre) {
      if (NBUF == 1) __syncthreads();  // every wave is done reading the single buffer
      char* Kn = smem + (NBUF == 2 ? ((kt + 1) & 1) : 0) * 2 * TB;
      tk.store(Kn, tid);
      tv.store(Kn + TB, tid);
    }
    __syncthreads();
  }
  if (qok) {
    const float inv = 1.f / l;
    u16* op = out + (long)(start + qrow) * nq * D + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(op + 16 * dt, o[dt], inv);
    if (g == 0) lse[(long)h * total + start + qrow] = (m + log2f(l)) * LN2;
  }
}

template <bool TR, int NW, int NBUF>
__global__ __launch_bounds__(NW * 64) void bwd_dq2_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta, const int* __restrict__ cu,
                                                          u16* __restrict__ dqkv, int nq, int nkv, int total,
                                                          float sl2, float scale, int causal) {
  constexpr int NT = NW * 64, BM = NW * 16, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * NBUF * TB];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * BM;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int qrow = q0 + wave * 16 + (lane & 15);
  const int wlast = q0 + wave * 16 + 15;
  const bool qok = qrow < len;
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* vbase = qkv + (long)start * ld + (nq + nkv + kvh) * D;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  {
    TileRegs<64, NT> tk, tv;
    tk.load(kbase, ld, min(64, len), tid);
    tv.load(vbase, ld, min(64, len), tid);
    tk.store(smem, tid);
    tv.store(smem + TB, tid);
  }
  bf16x8 qf[4], df[4];
  {
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
    const u16* dp = dout + (long)(start + qrow) * ldo + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = load_frag_global(qp + 32 * s, qok);
      df[s] = load_frag_global(dp + 32 * s, qok);
    }
  }
  const float lse2 = qok ? lse[(long)h * total + start + qrow] * LOG2E : 0.f;
  const float dl = qok ? delta[(long)h * total + start + qrow] : 0.f;
  f32x4 dq[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    char* Ks = smem + (NBUF == 2 ? (kt & 1) : 0) * 2 * TB;
    char* Vs = Ks + TB;
    const bool pre = kt + 1 < nkt;
    TileRegs<64, NT> tk, tv;
    if (pre) {
      const int kv = min(64, len - k0 - 64);
      tk.load(kbase + (long)(k0 + 64) * ld, ld, kv, tid);
      tv.load(vbase + (long)(k0 + 64) * ld, ld, kv, tid);
    }
    if (!causal || k0 <= wlast) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc[nt] = mfma(frag_row(Ks, 16 * nt, s, lane), qf[s], sc[nt]);
          dp[nt] = mfma(frag_row(Vs, 16 * nt, s, lane), df[s], dp[nt]);
        }
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = k0 + 16 * nt + 4 * g + i;
          float p = exp2f(sc[nt][i] * sl2 - lse2);
          if (key >= len || (causal && key > qrow) || !qok) p = 0.f;
          dp[nt][i] = p * (dp[nt][i] - dl);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) dq[dt] = mfma(frag_tr<TR>(Ks, 32 * ks, dt, lane), db, dq[dt]);
      }
    }
    if (pre) {
      if (NBUF == 1) __syncthreads();  // every wave is done reading the single buffer
      char* Kn = smem + (NBUF == 2 ? ((kt + 1) & 1) : 0) * 2 * TB;
      tk.store(Kn, tid);
      tv.store(Kn + TB, tid);
    }
    __syncthreads();
  }
  if (qok) {
    u16* qp = dqkv + (long)(start + qrow) * ld + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(qp + 16 * dt, dq[dt], scale);
  }
}

// dK/dV partials for ONE query head h (grid (key blocks, nq, nseq)); writes fp32 slab
// part[r][token][2*nkv*D] (r = h % rep; dK at kvh*D, dV at (nkv+kvh)*D). When rep == 1 the
// result goes straight to dqkv (bf16, dK scaled).
template <bool TR, int NBUF>
__global__ __launch_bounds__(256, 2) void bwd_dkdv2_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           const int* __restrict__ cu, float* __restrict__ part,
                                                           u16* __restrict__ dqkv, int nq, int nkv, int total,
                                                           float sl2, float scale, int causal) {
  constexpr int NT = 256, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * NBUF * TB + NBUF * 2 * 64 * 4];
  float* LDs = (float*)(smem + 2 * NBUF * TB);  // [buf][lse2 64 | delta 64]
  const int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int k0 = kb * 64;
  if (k0 >= len) return;
  const int rep = nq / nkv;
  const int kvh = h / rep, r = h - kvh * rep;
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int key = k0 + wave * 16 + (lane & 15);
  const int wfirst = k0 + wave * 16;
  const bool kok = key < len;
  const u16* qbase = qkv + (long)start * ld + h * D;
  const u16* obase = dout + (long)start * ldo + h * D;
  const float* lbase = lse + (long)h * total + start;
  const float* dbase = delta + (long)h * total + start;
  const int qt0 = causal ? kb : 0;
  const int nqt = (len + 63) / 64;
  {
    const int q0 = qt0 * 64, qv = min(64, len - q0);
    TileRegs<64, NT> tq, to;
    tq.load(qbase + (long)q0 * ld, ld, qv, tid);
    to.load(obase + (long)q0 * ldo, ldo, qv, tid);
    tq.store(smem, tid);
    to.store(smem + TB, tid);
    if (tid < 64) {
      LDs[tid] = tid < qv ? lbase[q0 + tid] * LOG2E : 0.f;
      LDs[64 + tid] = tid < qv ? dbase[q0 + tid] : 0.f;
    }
  }
  bf16x8 kf[4], vf[4];
  {
    const u16* kp = qkv + (long)(start + key) * ld + (nq + kvh) * D + 8 * g;
    const u16* vp = qkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = load_frag_global(kp + 32 * s, kok);
      vf[s] = load_frag_global(vp + 32 * s, kok);
    }
  }
  f32x4 dk[8], dv[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  for (int qt = qt0; qt < nqt; ++qt) {
    const int q0 = qt * 64;
    const int buf = NBUF == 2 ? ((qt - qt0) & 1) : 0;
    char* Qs = smem + buf * 2 * TB;
    char* Os = Qs + TB;
    const float* Ls = LDs + buf * 128;
    const float* Dl = Ls + 64;
    const bool pre = qt + 1 < nqt;
    TileRegs<64, NT> tq, to;
    float pl = 0.f, pd = 0.f;
    if (pre) {
      const int qn = q0 + 64, qv = min(64, len - qn);
      tq.load(qbase + (long)qn * ld, ld, qv, tid);
      to.load(obase + (long)qn * ldo, ldo, qv, tid);
      if (tid < 64 && tid < qv) {
        pl = lbase[qn + tid] * LOG2E;
        pd = dbase[qn + tid];
      }
    }
    // a wave whose 16 keys are all later than every query of the tile contributes nothing
    if (!causal || wfirst <= q0 + 63) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc[mt] = mfma(frag_row(Qs, 16 * mt, s, lane), kf[s], sc[mt]);
          dp[mt] = mfma(frag_row(Os, 16 * mt, s, lane), vf[s], dp[mt]);
        }
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qi = 16 * mt + 4 * g + i;
          const int q = q0 + qi;
          float p = exp2f(sc[mt][i] * sl2 - Ls[qi]);
          if (q >= len || (causal && key > q)) p = 0.f;
          sc[mt][i] = p;
          dp[mt][i] = p * (dp[mt][i] - Dl[qi]);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
        const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          dv[dt] = mfma(frag_tr<TR>(Os, 32 * ks, dt, lane), pb, dv[dt]);
          dk[dt] = mfma(frag_tr<TR>(Qs, 32 * ks, dt, lane), db, dk[dt]);
        }
      }
    }
    if (pre) {
      if (NBUF == 1) __syncthreads();
      const int nb = NBUF == 2 ? (buf ^ 1) : 0;
      char* Qn = smem + nb * 2 * TB;
      tq.store(Qn, tid);
      to.store(Qn + TB, tid);
      if (tid < 64) {
        float* Ln = LDs + nb * 128;
        Ln[tid] = pl;
        Ln[64 + tid] = pd;
      }
    }
    __syncthreads();
  }
  if (!kok) return;
  if (rep == 1) {
    u16* kp = dqkv + (long)(start + key) * ld + (nq + kvh) * D + 4 * g;
    u16* vp = dqkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      store4(kp + 16 * dt, dk[dt], scale);
      store4(vp + 16 * dt, dv[dt], 1.f);
    }
    return;
  }
  const long pld = 2L * nkv * D;
  float* pk = part + ((long)r * total + start + key) * pld + kvh * D + 4 * g;
  float* pv = pk + (long)nkv * D;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    *(float4*)(pk + 16 * dt) = make_float4(dk[dt][0], dk[dt][1], dk[dt][2], dk[dt][3]);
    *(float4*)(pv + 16 * dt) = make_float4(dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
  }
}

// dqkv[m, nq*D + c] = bf16(sum_r part[r][m][c] * (c < nkv*D ? scale : 1)), fixed summation order.
__global__ __launch_bounds__(256) void dkdv_reduce_kernel(const float* __restrict__ part, u16* __restrict__ dqkv,
                                                          int total, int nq, int nkv, int rep, float scale) {
  const int C = 2 * nkv * D;
  const long nvec = (long)total * C / 8;
  const long ld = (long)(nq + 2 * nkv) * D;
  const long stride = (long)total * C;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nvec; v += (long)gridDim.x * 256) {
    const long e = v * 8;
    const long m = e / C;
    const int c = (int)(e - m * C);
    float acc[8];
    *(float4*)&acc[0] = *(const float4*)(part + e);
    *(float4*)&acc[4] = *(const float4*)(part + e + 4);
    for (int r = 1; r < rep; ++r) {
      const float4 a = *(const float4*)(part + r * stride + e);
      const float4 b2 = *(const float4*)(part + r * stride + e + 4);
      acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
      acc[4] += b2.x; acc[5] += b2.y; acc[6] += b2.z; acc[7] += b2.w;
    }
    const float sc = c < nkv * D ? scale : 1.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= sc;
    *(uint4*)(dqkv + m * ld + (long)nq * D + c) = pack8(acc);
  }
}

// ============================================================================== v3 kernels
// VALU diet for the v2 structure (the v2 main loops issued ~7 VALU per MFMA: rocprofv3 showed
// SQ_INSTS_VALU ~ 10x the MFMA count). Changes, all wave-uniform:
// * LDS operand addresses are per-lane constants computed once: 4 row-read bases (one per
//   k-step) and 8 transposed-read bases (one per 16-column block); tile / k-step / half-tile
//   displacements are compile-time immediates of the ds_read instructions;
// * causal/length masks are applied only on tiles that straddle the diagonal or the sequence end;
// * the softmax scale is folded into the exponent (one FMA per score), the running max is taken
//   on raw scores (v_max3), and O/l are rescaled only when the row max grows by more than
//   THR = 8 (log2 domain; T13 deferred rescale: P stays <= 2^8, exact in bf16 exponent range);
// * full tiles are staged without per-row bounds checks; one LDS buffer (register prefetch).
constexpr float THR = 8.f;
constexpr float THR_FAST = 40.f;  // v6 fast loop: P = exp2(s - m) <= 2^40, o <= 2^49 |V|: far from fp32 / bf16 limits

struct Offs {
  int row[4];  // frag_row bases, k-step s
  int tr[8];   // frag_tr bases, column block dt
  __device__ __forceinline__ void init(int lane) {
    const int g = lane >> 4, r = lane & 15;
#pragma unroll
    for (int s = 0; s < 4; ++s) row[s] = img_off(r, 4 * s + g);
    const int q = r >> 2, p = r & 3, r0 = 4 * g + q;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) tr[dt] = img_off(r0, 2 * dt + (p >> 1)) + 8 * (p & 1);
  }
};

__device__ __forceinline__ bf16x8 lds_row(const char* base, int off) { return *(const bf16x8*)(base + off); }

__device__ __forceinline__ bf16x8 lds_tr(const char* base, int off) {
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + off));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + off + 16 * ROWB));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// vmcnt(0) as the builtin (not inline asm), so the waitcnt pass sees it: a kernel whose loop-invariant operands (Q /
// K fragments) are global loads issued before the loop must drain them there; otherwise the pass merges the loop-entry
// state with the back edge and puts a vmcnt(0) before the loop's first MFMA, which also waits for the NEXT tile's
// prefetch every iteration (its latency fully exposed: profiles/r3_attention.md).
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// max / sum over the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 (one query column's key groups) with VALU lane swaps
// (v_permlane32_swap / v_permlane16_swap) instead of ds_bpermute round trips through the LDS unit.
__device__ __forceinline__ float xmax4(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
// max of a 16-score tile in 8 v_max3_f32 (fmaxf's NaN canonicalisation doubles the VALU count; scores are finite
// or -inf here)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max16(const f32x4 (&v)[4]) {
  const float a = max3f(v[0][0], v[0][1], v[0][2]), b = max3f(v[0][3], v[1][0], v[1][1]);
  const float c = max3f(v[1][2], v[1][3], v[2][0]), d = max3f(v[2][1], v[2][2], v[2][3]);
  const float e = max3f(v[3][0], v[3][1], v[3][2]);
  return max3f(max3f(a, b, c), max3f(d, e, v[3][3]), -INFINITY);
}
__device__ __forceinline__ float xsum4(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <int R, int NT>
struct Stage {
  static constexpr int N = (R * 16) / NT;
  uint4 v[N];
  __device__ __forceinline__ void load(const u16* __restrict__ g, long ld, int nvalid, int tid) {
    const int r = tid >> 4, ch = tid & 15;
    const u16* p = g + (long)r * ld + ch * 8;
    if (nvalid >= R) {
#pragma unroll
      for (int it = 0; it < N; ++it) v[it] = *(const uint4*)(p + (long)it * (NT / 16) * ld);
    } else {
#pragma unroll
      for (int it = 0; it < N; ++it)
        v[it] = (r + it * (NT / 16) < nvalid) ? *(const uint4*)(p + (long)it * (NT / 16) * ld) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
    const int off = img_off(tid >> 4, tid & 15);  // rows advance by NT/16 (multiple of 16): same swizzle
#pragma unroll
    for (int it = 0; it < N; ++it) *(uint4*)(lds + off + it * (NT / 16) * ROWB) = v[it];
  }
};

// 16 B per lane HBM -> LDS (global_load_lds): lane-linear LDS destination, the image swizzle applied to the source
__device__ __forceinline__ void lds_dma16(const u16* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
}

// One 64-key tile of the LDS-DMA forward (fwd3 DIAG bit5): issue the next tile's K / V pieces into stage nxt, then
// S^T = K Q^T, the online softmax and O^T += V^T P^T from stage cur. cur / nxt are __restrict__ parameters of ONE
// frame, so the waitcnt pass knows the DMA (tracked by vmcnt) never feeds these LDS reads; as plain pointers it put
// a vmcnt(0) before the first V^T read, i.e. waited for the next tile inside this one.
__device__ __forceinline__ void fwd_step_dma(const char* __restrict__ cur, char* __restrict__ nxt, bool pre, bool active,
                                             const u16* kbase, const u16* vbase, long ld, long kvoff, int r0, int wave,
                                             int k0, int len, int causal, int wfirst, int qrow, int g, float sl2,
                                             const Offs& off, const bf16x8 (&qf)[4], f32x4 (&o)[8], float& m,
                                             float& l, int ahead = 64) {
  constexpr int TB = 64 * ROWB;
  if (pre) {  // the tile `ahead` keys past this one
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long row = min(k0 + ahead + r0 + 32 * j, len - 1);
      lds_dma16(kbase + row * ld + kvoff, nxt + (wave + 8 * j) * 1024);
      lds_dma16(vbase + row * ld + kvoff, nxt + TB + (wave + 8 * j) * 1024);
    }
  }
  if (!active) return;
  const char* Ks = cur;
  const char* Vs = cur + TB;
  f32x4 sc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) sc[nt] = mfma(lds_row(Ks, off.row[s] + nt * 16 * ROWB), qf[s], sc[nt]);
  }
  if ((k0 + 64 > len) || (causal && k0 + 63 > wfirst)) {
    const int lim = (causal ? min(len - 1, qrow) : len - 1) - k0 - 4 * g;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) sc[nt][i] = 16 * nt + i > lim ? -INFINITY : sc[nt][i];
  }
  const float tmax = xmax4(max16(sc)) * sl2;
  if (__any(tmax > m + THR)) {
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
    m = mnew;
  }
  f32x2 acc = {0.f, 0.f};
  const f32x2 sl = {sl2, sl2}, nm = {-m, -m};
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      const f32x2 t = __builtin_elementwise_fma(f32x2{sc[nt][i], sc[nt][i + 1]}, sl, nm);
      const f32x2 p = {exp2f(t.x), exp2f(t.y)};
      sc[nt][i] = p.x;
      sc[nt][i + 1] = p.y;
      acc += p;
    }
  l += acc.x + acc.y;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = mfma(lds_tr(Vs, off.tr[dt] + ks * 32 * ROWB), pb, o[dt]);
  }
}

// fwd7: 4 waves x 2 row groups of 16 queries (BM = 128), K / V by LDS-DMA into two stages. Every K fragment and V^T
// fragment read from LDS feeds two MFMAs (half fwd3's LDS bytes per MFMA), and each wave carries two independent
// softmax chains (ILP for the one wave per SIMD of each workgroup; 64 KB LDS -> 2 workgroups per CU).
// Opt-in: SFTAMD_ATTN_FWD7=1.
__device__ __forceinline__ void fwd7_step(const char* __restrict__ cur, char* __restrict__ nxt, bool pre,
                                          const u16* kbase, const u16* vbase, long ld, long kvoff, int r0, int wave,
                                          int k0, int len, int causal, int wfirst, int g, int ql, float sl2,
                                          const Offs& off, const bf16x8 (&qf)[2][4], f32x4 (&o)[2][8], float (&m)[2],
                                          float (&l)[2]) {
  constexpr int TB = 64 * ROWB;
  if (pre) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long row = min(k0 + 64 + r0 + 16 * j, len - 1);
      lds_dma16(kbase + row * ld + kvoff, nxt + (wave + 4 * j) * 1024);
      lds_dma16(vbase + row * ld + kvoff, nxt + TB + (wave + 4 * j) * 1024);
    }
  }
  if (causal && k0 > wfirst + 31) return;  // both row groups above this tile's diagonal
  const char* Ks = cur;
  const char* Vs = cur + TB;
  f32x4 sc[2][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    sc[0][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    sc[1][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 kf = lds_row(Ks, off.row[s] + nt * 16 * ROWB);
      sc[0][nt] = mfma(kf, qf[0][s], sc[0][nt]);
      sc[1][nt] = mfma(kf, qf[1][s], sc[1][nt]);
    }
  }
  bf16x8 pb[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int rfirst = wfirst + 16 * r, qrow = rfirst + ql;
    if ((k0 + 64 > len) || (causal && k0 + 63 > rfirst)) {
      const int lim = (causal ? min(len - 1, qrow) : len - 1) - k0 - 4 * g;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sc[r][nt][i] = 16 * nt + i > lim ? -INFINITY : sc[r][nt][i];
    }
    const float tmax = xmax4(max16(sc[r])) * sl2;
    if (__any(tmax > m[r] + THR)) {
      const float mnew = fmaxf(m[r], tmax);
      const float alpha = exp2f(m[r] - mnew);
      l[r] *= alpha;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) o[r][dt] *= alpha;
      m[r] = mnew;
    }
    f32x2 acc = {0.f, 0.f};
    const f32x2 sl = {sl2, sl2}, nm = {-m[r], -m[r]};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const f32x2 t = __builtin_elementwise_fma(f32x2{sc[r][nt][i], sc[r][nt][i + 1]}, sl, nm);
        const f32x2 p = {exp2f(t.x), exp2f(t.y)};
        sc[r][nt][i] = p.x;
        sc[r][nt][i + 1] = p.y;
        acc += p;
      }
    l[r] += acc.x + acc.y;
    pb[r][0] = pack_acc(sc[r][0], sc[r][1]);
    pb[r][1] = pack_acc(sc[r][2], sc[r][3]);
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const bf16x8 vf = lds_tr(Vs, off.tr[dt] + ks * 32 * ROWB);
      o[0][dt] = mfma(vf, pb[0][ks], o[0][dt]);
      o[1][dt] = mfma(vf, pb[1][ks], o[1][dt]);
    }
}

__global__ __launch_bounds__(256, 2) void fwd7_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                      float* __restrict__ lse, const int* __restrict__ cu, int nq,
                                                      int nkv, int total, float sl2, int causal) {
  constexpr int BM = 128, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];  // two stages of (K, V) images
  const int h = blockIdx.x, b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;  // LPT: heaviest q-block first
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * BM;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, ql = lane & 15;
  const int wfirst = q0 + wave * 32;
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* vbase = qkv + (long)start * ld + (nq + nkv + kvh) * D;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  Offs off;
  off.init(lane);
  bf16x8 qf[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int qrow = wfirst + 16 * r + ql;
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[r][s] = load_frag_global(qp + 32 * s, qrow < len);
  }
  const int r0 = 4 * wave + (lane >> 4);
  const long kvoff = 8 * swz(r0, lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long row = min(r0 + 16 * j, len - 1);
    lds_dma16(kbase + row * ld + kvoff, smem + (wave + 4 * j) * 1024);
    lds_dma16(vbase + row * ld + kvoff, smem + TB + (wave + 4 * j) * 1024);
  }
  vm_drain();
  f32x4 o[2][8];
  float m[2] = {-1e30f, -1e30f}, l[2] = {0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[r][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const bool pre = kt + 1 < nkt;
    fwd7_step(smem + (kt & 1) * 2 * TB, smem + ((kt + 1) & 1) * 2 * TB, pre, kbase, vbase, ld, kvoff, r0, wave, kt * 64,
              len, causal, wfirst, g, ql, sl2, off, qf, o, m, l);
    if (pre) vm_drain();
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const float lt = xsum4(l[r]);
    const int qrow = wfirst + 16 * r + ql;
    if (qrow < len) {
      const float inv = 1.f / lt;
      u16* op = out + (long)(start + qrow) * nq * D + h * D + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) store4(op + 16 * dt, o[r][dt], inv);
      if (g == 0) lse[(long)h * total + start + qrow] = (m[r] + log2f(lt)) * LN2;
    }
  }
}

// DIAG (timing-only ablations, wrong results): bit0 no next-tile loads/stores, bit1 no softmax math,
// bit2 no PV MFMAs, bit3 no QK MFMAs. bit4 (results exact): the round-2 schedule for A/B runs (no vm_drain before
// the loop, per-tile row-sum shuffles through ds_bpermute). bit5: K / V tiles by LDS-DMA into two stages (no VGPR
// staging / ds_write, one barrier per tile; NW = 8).
template <int NW, int DIAG = 0>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 4 : 2) void fwd3_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                       float* __restrict__ lse, const int* __restrict__ cu, int nq,
                                                       int nkv, int total, float sl2, int causal) {
  constexpr int NT = NW * 64, BM = NW * 16, TB = 64 * ROWB;
  constexpr bool DMA3 = DIAG & 64;  // three stages, two tiles in flight (implies DMA)
  constexpr bool DMA = (DIAG & 32) || DMA3;
  static_assert(!DMA || NW == 8, "LDS-DMA staging: 8 waves x 2 pieces per 64-row image");
  __shared__ __attribute__((aligned(16))) char smem[(DMA3 ? 6 : DMA ? 4 : 2) * TB];
  char* Ks = smem;
  char* Vs = smem + TB;
  // grid (heads, sequences, q-blocks) with the last (causally heaviest) q-block dispatched first: LPT order
  const int h = blockIdx.x, b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * BM;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wfirst = q0 + wave * 16;
  const int qrow = wfirst + (lane & 15);
  const bool qok = qrow < len;
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* vbase = qkv + (long)start * ld + (nq + nkv + kvh) * D;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  Offs off;
  off.init(lane);
  constexpr bool LEG = DIAG & 16;
  bf16x8 qf[4];
  if constexpr (!LEG) {  // Q first: the (in-order) wait for the first K / V tile then covers it
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = load_frag_global(qp + 32 * s, qok);
  }
  // DMA: lane (wave w, l) fills LDS rows 4 (w + 8 j) + (l >> 4), position l & 15 with the chunk swz(row, l & 15) of
  // that row (rows past the sequence end clamped to its last row: their keys are masked)
  const int r0 = 4 * wave + (lane >> 4);
  const long kvoff = 8 * swz(r0, lane & 15);
  if constexpr (DMA3) {
    // tiles 0 and 1 are issued by the loop's first two (compute-free) iterations: the same code instance as every
    // later DMA, so the waitcnt pass sees them in the loop's alias scopes and adds no vmcnt(0) before the loop
  } else if constexpr (DMA) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long row = min(r0 + 32 * j, len - 1);
      lds_dma16(kbase + row * ld + kvoff, smem + (wave + 8 * j) * 1024);
      lds_dma16(vbase + row * ld + kvoff, smem + TB + (wave + 8 * j) * 1024);
    }
  } else {
    Stage<64, NT> tk, tv;
    tk.load(kbase, ld, len, tid);
    tv.load(vbase, ld, len, tid);
    tk.store(Ks, tid);
    tv.store(Vs, tid);
  }
  if constexpr (LEG) {
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = load_frag_global(qp + 32 * s, qok);
  }
  if constexpr (!LEG) vm_drain();
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;  // l: this lane's partial row sum (its 16 keys per tile) unless LEG
  __syncthreads();
  if constexpr (DMA3) {
    int sc = 1;  // stage of tile kt (kt = -2, -1: no tile, the DMA of tiles 0, 1); tile kt + 2 -> stage (sc + 2) % 3
    for (int kt = -2; kt < nkt; ++kt) {
      const int k0 = kt * 64;
      const bool pre2 = kt + 2 < nkt;
      const int sn = sc == 0 ? 2 : sc - 1;
      fwd_step_dma(smem + sc * 2 * TB, smem + sn * 2 * TB, pre2, kt >= 0 && (!causal || k0 <= wfirst + 15), kbase,
                   vbase, ld, kvoff, r0, wave, k0, len, causal, wfirst, qrow, g, sl2, off, qf, o, m, l, 128);
      // vmcnt(4) + lgkmcnt(0): tile kt + 1 landed (kt + 2's 4 pieces may fly), this wave's LDS reads are done; a
      // plain s_barrier, as __syncthreads' fence would wait for the in-flight DMA too (vmcnt(0))
      if (pre2) __builtin_amdgcn_s_waitcnt(0x0074);
      else __builtin_amdgcn_s_waitcnt(0x0070);
      __builtin_amdgcn_s_barrier();
      sc = sc == 2 ? 0 : sc + 1;
    }
  } else if constexpr (DMA) {
    for (int kt = 0; kt < nkt; ++kt) {
      const int k0 = kt * 64;
      const bool pre = kt + 1 < nkt;
      // stage (kt + 1) & 1's last reads ended at the previous iteration's barrier
      fwd_step_dma(smem + (kt & 1) * 2 * TB, smem + ((kt + 1) & 1) * 2 * TB, pre, !causal || k0 <= wfirst + 15,
                   kbase, vbase, ld, kvoff, r0, wave, k0, len, causal, wfirst, qrow, g, sl2, off, qf, o, m, l);
      if (pre) vm_drain();  // this lane's pieces of the next tile landed ...
      __syncthreads();      // ... and every lane's; every wave is done reading this stage
    }
  }
  for (int kt = 0; kt < (DMA ? 0 : nkt); ++kt) {
    const int k0 = kt * 64;
    const bool pre = !(DIAG & 1) && kt + 1 < nkt;
    Stage<64, NT> tk, tv;
    if (pre) {
      tk.load(kbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
      tv.load(vbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
    }
    if (!causal || k0 <= wfirst + 15) {
      f32x4 sc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (!(DIAG & 8)) sc[nt] = mfma(lds_row(Ks, off.row[s] + nt * 16 * ROWB), qf[s], sc[nt]);
      }
      if constexpr (!(DIAG & 2)) {
      const bool need_mask = (k0 + 64 > len) || (causal && k0 + 63 > wfirst);
      if (need_mask) {
        if constexpr (LEG) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int key = k0 + 16 * nt + 4 * g + i;
              if (key >= len || (causal && key > qrow)) sc[nt][i] = -INFINITY;
            }
        } else {  // one compare + select per score: key offset 16 nt + i against the lane's last visible key
          const int lim = (causal ? min(len - 1, qrow) : len - 1) - k0 - 4 * g;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) sc[nt][i] = 16 * nt + i > lim ? -INFINITY : sc[nt][i];
        }
      }
      float tmax;
      if constexpr (LEG) {
        tmax = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                     fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
        tmax = fmaxf(tmax, fmaxf(fmaxf(fmaxf(sc[2][0], sc[2][1]), fmaxf(sc[2][2], sc[2][3])),
                                 fmaxf(fmaxf(sc[3][0], sc[3][1]), fmaxf(sc[3][2], sc[3][3]))));
      } else {
        tmax = max16(sc);
      }
      if constexpr (LEG) {
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      } else {
        tmax = xmax4(tmax);
      }
      tmax *= sl2;
      if (__any(tmax > m + THR)) {  // deferred rescale (rare after the first tiles)
        const float mnew = fmaxf(m, tmax);
        const float alpha = exp2f(m - mnew);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
        m = mnew;
      }
      float rs = 0.f;
      if constexpr (LEG) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = exp2f(fmaf(sc[nt][i], sl2, -m));
            sc[nt][i] = p;
            rs += p;
          }
        rs += __shfl_xor(rs, 16, 64);
        rs += __shfl_xor(rs, 32, 64);
      } else {  // packed fp32 (v_pk_fma_f32 / v_pk_add_f32): two scores per VALU op around the exp2
        f32x2 acc = {0.f, 0.f};
        const f32x2 sl = {sl2, sl2}, nm = {-m, -m};
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const f32x2 t = __builtin_elementwise_fma(f32x2{sc[nt][i], sc[nt][i + 1]}, sl, nm);
            const f32x2 p = {exp2f(t.x), exp2f(t.y)};
            sc[nt][i] = p.x;
            sc[nt][i + 1] = p.y;
            acc += p;
          }
        rs = acc.x + acc.y;
      }
      l += rs;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
          if (!(DIAG & 4)) o[dt] = mfma(lds_tr(Vs, off.tr[dt] + ks * 32 * ROWB), pb, o[dt]);
      }
    }
    if (pre) {
      __syncthreads();
      tk.store(Ks, tid);
      tv.store(Vs, tid);
    }
    __syncthreads();
  }
  if constexpr (!LEG) l = xsum4(l);
  if (qok) {
    const float inv = 1.f / l;
    u16* op = out + (long)(start + qrow) * nq * D + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(op + 16 * dt, o[dt], inv);
    if (g == 0) lse[(long)h * total + start + qrow] = (m + log2f(l)) * LN2;
  }
}

// v4 forward: every wave owns RG = 2 row groups of 16 queries, so each K fragment (row read) and V
// fragment (transposed read) fetched from LDS feeds RG MFMAs — v3 reads 1 KB of LDS per MFMA, twice
// what the LDS can deliver at the MFMA rate (256 B/clk/CU vs 4 SIMDs x 16x16x32 per 16 clk); v4 reads
// 0.5 KB. Otherwise v3's structure: one LDS K/V buffer with register prefetch, masks only on
// diagonal / tail tiles, exp2 with the scale folded in, deferred rescale (THR).
template <int NW, int RG>
__global__ __launch_bounds__(NW * 64) void fwd4_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                       float* __restrict__ lse, const int* __restrict__ cu, int nq,
                                                       int nkv, int total, float sl2, int causal) {
  constexpr int NT = NW * 64, BM = NW * 16 * RG, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * TB];
  char* Ks = smem;
  char* Vs = smem + TB;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * BM;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wfirst = q0 + wave * 16 * RG;  // first query row of the wave
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* vbase = qkv + (long)start * ld + (nq + nkv + kvh) * D;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  Offs off;
  off.init(lane);
  {
    Stage<64, NT> tk, tv;
    tk.load(kbase, ld, len, tid);
    tv.load(vbase, ld, len, tid);
    tk.store(Ks, tid);
    tv.store(Vs, tid);
  }
  bf16x8 qf[RG][4];
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    const int qrow = wfirst + 16 * r + (lane & 15);
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) qf[r][s2] = load_frag_global(qp + 32 * s2, qrow < len);
  }
  f32x4 o[RG][8];
  float m[RG], l[RG];
#pragma unroll
  for (int r = 0; r < RG; ++r) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[r][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[r] = -1e30f;
    l[r] = 0.f;
  }
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const bool pre = kt + 1 < nkt;
    Stage<64, NT> tk, tv;
    if (pre) {
      tk.load(kbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
      tv.load(vbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
    }
    if (!causal || k0 <= wfirst + 16 * RG - 1) {
      f32x4 sc[RG][4];
#pragma unroll
      for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) sc[r][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const bf16x8 kf = lds_row(Ks, off.row[s2] + nt * 16 * ROWB);
#pragma unroll
          for (int r = 0; r < RG; ++r) sc[r][nt] = mfma(kf, qf[r][s2], sc[r][nt]);
        }
      bf16x8 pb[RG][2];
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const int rfirst = wfirst + 16 * r;
        const int qrow = rfirst + (lane & 15);
        const bool need_mask = (k0 + 64 > len) || (causal && k0 + 63 > rfirst);
        if (need_mask) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int key = k0 + 16 * nt + 4 * g + i;
              if (key >= len || (causal && key > qrow)) sc[r][nt][i] = -INFINITY;
            }
        }
        float tmax = fmaxf(fmaxf(fmaxf(sc[r][0][0], sc[r][0][1]), fmaxf(sc[r][0][2], sc[r][0][3])),
                           fmaxf(fmaxf(sc[r][1][0], sc[r][1][1]), fmaxf(sc[r][1][2], sc[r][1][3])));
        tmax = fmaxf(tmax, fmaxf(fmaxf(fmaxf(sc[r][2][0], sc[r][2][1]), fmaxf(sc[r][2][2], sc[r][2][3])),
                                 fmaxf(fmaxf(sc[r][3][0], sc[r][3][1]), fmaxf(sc[r][3][2], sc[r][3][3]))));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        tmax *= sl2;
        if (__any(tmax > m[r] + THR)) {
          const float mnew = fmaxf(m[r], tmax);
          const float alpha = exp2f(m[r] - mnew);
          l[r] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) o[r][dt] *= alpha;
          m[r] = mnew;
        }
        float rs = 0.f;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = exp2f(fmaf(sc[r][nt][i], sl2, -m[r]));
            sc[r][nt][i] = p;
            rs += p;
          }
        rs += __shfl_xor(rs, 16, 64);
        rs += __shfl_xor(rs, 32, 64);
        l[r] += rs;
        pb[r][0] = pack_acc(sc[r][0], sc[r][1]);
        pb[r][1] = pack_acc(sc[r][2], sc[r][3]);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const bf16x8 vf = lds_tr(Vs, off.tr[dt] + ks * 32 * ROWB);
#pragma unroll
          for (int r = 0; r < RG; ++r) o[r][dt] = mfma(vf, pb[r][ks], o[r][dt]);
        }
    }
    if (pre) {
      __syncthreads();
      tk.store(Ks, tid);
      tv.store(Vs, tid);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    const int qrow = wfirst + 16 * r + (lane & 15);
    if (qrow < len) {
      const float inv = 1.f / l[r];
      u16* op = out + (long)(start + qrow) * nq * D + h * D + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) store4(op + 16 * dt, o[r][dt], inv);
      if (g == 0) lse[(long)h * total + start + qrow] = (m[r] + log2f(l[r])) * LN2;
    }
  }
}

// v6 forward (GQA-stacked): one workgroup per (kv head, sequence, 64-query block), 4 waves; wave w owns query
// positions q0 + 16 w .. + 15 for ALL REP query heads of the kv head. A K fragment (S^T = K Q^T) and a V^T fragment
// (O^T += V^T P^T) are read from LDS once and feed REP MFMAs, one per head — REP x fewer LDS bytes per MFMA than v3,
// whose 1 KB per MFMA is twice what the LDS delivers at the MFMA rate. The causal / length masks are shared by the REP
// heads (same positions). K / V tiles (64 keys) go HBM -> LDS by global_load_lds (16 B per lane, lane-linear LDS
// writes: the image swizzle is applied to the SOURCE chunk, rows past the sequence end clamped to its last row so
// nothing outside the sequence is read) into two stages, the next tile's DMA in flight under the current tile's math.
// The row sums stay per-lane partials until the end (the running max is the only per-tile cross-lane reduction).
// REP x (32 o + 16 Q) registers per lane: one wave per SIMD, one workgroup per CU; grid (nkv, nseq, q-blocks) with the
// causally heaviest q-blocks dispatched first (LPT: a CU that drew block 4 of 8 takes block 3 next).
__device__ __forceinline__ void glds16(const u16* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
}

// O^T += V^T P^T with the accumulator tied to an AGPR: REP x 8 accumulators stay put across the K loop (as builtins,
// hipcc shuffled them between AGPRs and VGPRs every tile: ~1250 v_accvgpr moves per tile at REP 4). The compiler does
// not see these as MFMAs: VALU reads of the accumulators (rescale, epilogue) sit behind nop_mfma() wait states.
// The leading s_nop 1: P arrives from VALU packs (VALU write -> MFMA operand read: 2 wait states hipcc does not pad
// inside asm, cdna_hip_programming.md §5.7 item 2).
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// S^T = K Q^T into VGPRs (the softmax reads them): hipcc's builtin put them in AGPRs and copied them back every tile.
// Chains accumulate D -> C whole (0 wait states); the VALU readers sit behind nop_mfma().
__device__ __forceinline__ f32x4 mfma_v0(const bf16x8& a, const bf16x8& b) {
  f32x4 d;
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ void mfma_v(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void pin_acc(f32x4& c) { asm volatile("" : "+a"(c)); }  // (re)home a value in AGPRs
__device__ __forceinline__ void nop_mfma() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

template <int REP>
__global__ __launch_bounds__(256, 1) void fwd6_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                      float* __restrict__ lse, const int* __restrict__ cu, int nq,
                                                      int nkv, int total, float sl2, int causal) {
  constexpr int TB = 64 * ROWB;  // one 64-row image: 16 KB
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];  // stage s: K image at 2 s TB, V image at (2 s + 1) TB
  const int kvh = blockIdx.x, b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * 64;
  if (q0 >= len) return;
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int wfirst = q0 + 16 * w, qrow = wfirst + (lane & 15);
  const bool qok = qrow < len;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min(qb + 1, nkb) : nkb;
  // DMA: piece j < 4 of wave w = image rows 4 (w + 4 j) .. + 3 of K and of V (1 KB each); lane -> row r0 + 16 j,
  // LDS chunk lane & 15 = source chunk swz(row, lane & 15) — the same for every j (row & 3 and (row >> 2) & 3 are)
  const int r0 = 4 * w + (lane >> 4);
  const u16* kvsrc = qkv + (long)start * ld + (nq + kvh) * D + 8 * swz(r0, lane & 15);
  auto dma = [&](int kt, char* stage) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u16* src = kvsrc + (long)min(kt * 64 + r0 + 16 * j, len - 1) * ld;
      glds16(src, stage + (w + 4 * j) * 1024);
      glds16(src + nkv * D, stage + TB + (w + 4 * j) * 1024);
    }
  };
  dma(0, smem);
  Offs off;
  off.init(lane);
  bf16x8 qf[REP][4];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    const u16* qp = qkv + (long)(start + qrow) * ld + (kvh * REP + h) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[h][s] = load_frag_global(qp + 32 * s, qok);
  }
  f32x4 o[REP][8];
  float m[REP], l[REP];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      o[h][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
      pin_acc(o[h][dt]);
    }
    m[h] = 0.f;  // set from tile 0
    l[h] = 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0);  // tile 0 landed (vmcnt / lgkmcnt 0)
  __syncthreads();
  // One K/V tile. FAST: no accumulator rescale — the running max m is set from tile 0 (o = 0 then) and P =
  // exp2(s - m) may grow up to 2^THR_FAST (bf16 / fp32 hold that exactly enough: only the exponent grows); a tile
  // whose max exceeds m + THR_FAST returns false BEFORE touching any state and the rest of the row block runs the
  // SLOW variant (rescale by alpha, v3's deferred scheme). Keeping the rescale out of the fast loop keeps the
  // accumulators in AGPRs there (a VALU rescale in the loop made hipcc copy all of them to VGPRs every tile).
  auto tile = [&](int kt, auto slow_t) -> bool {
    constexpr bool SLOW = decltype(slow_t)::value;
    const int k0 = kt * 64;
    const char* Ks = smem + (kt & 1) * 2 * TB;
    const char* Vs = Ks + TB;
    f32x4 sc[REP][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = lds_row(Ks, off.row[s] + nt * 16 * ROWB);
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          if (s == 0) sc[h][nt] = mfma_v0(kf, qf[h][s]);
          else mfma_v(sc[h][nt], kf, qf[h][s]);
        }
      }
    nop_mfma();  // MFMA D -> VALU: 12 wait states for the 8-pass MFMA
    if ((k0 + 64 > len) || (causal && k0 + 63 > wfirst)) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = k0 + 16 * nt + 4 * g + i;
          if (key >= len || (causal && key > qrow)) {
#pragma unroll
            for (int h = 0; h < REP; ++h) sc[h][nt][i] = -INFINITY;
          }
        }
    }
    float tmax[REP];
    bool big = false;
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      float t = fmaxf(fmaxf(fmaxf(sc[h][0][0], sc[h][0][1]), fmaxf(sc[h][0][2], sc[h][0][3])),
                      fmaxf(fmaxf(sc[h][1][0], sc[h][1][1]), fmaxf(sc[h][1][2], sc[h][1][3])));
      t = fmaxf(t, fmaxf(fmaxf(fmaxf(sc[h][2][0], sc[h][2][1]), fmaxf(sc[h][2][2], sc[h][2][3])),
                         fmaxf(fmaxf(sc[h][3][0], sc[h][3][1]), fmaxf(sc[h][3][2], sc[h][3][3]))));
      t = fmaxf(t, __shfl_xor(t, 16, 64));
      t = fmaxf(t, __shfl_xor(t, 32, 64));
      tmax[h] = t * sl2;
      if constexpr (!SLOW) {
        if (kt == 0) m[h] = tmax[h];  // o and l are still 0: no rescale
        big |= tmax[h] > m[h] + THR_FAST;
      }
    }
    if constexpr (!SLOW) {
      if (__any(big)) return false;
    }
    bf16x8 pb[REP][2];
#pragma unroll
    for (int h = 0; h < REP; ++h) {
      if constexpr (SLOW) {
        if (__any(tmax[h] > m[h] + THR)) {
          nop_mfma();
          const float mnew = fmaxf(m[h], tmax[h]);
          const float alpha = exp2f(m[h] - mnew);
          l[h] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) o[h][dt] *= alpha;
          m[h] = mnew;
        }
      }
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = exp2f(fmaf(sc[h][nt][i], sl2, -m[h]));
          sc[h][nt][i] = p;
          rs += p;
        }
      l[h] += rs;  // per-lane partial: the 4 lanes of a query share m, so their partials add up at the end
      pb[h][0] = pack_acc(sc[h][0], sc[h][1]);
      pb[h][1] = pack_acc(sc[h][2], sc[h][3]);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const bf16x8 vf = lds_tr(Vs, off.tr[dt] + ks * 32 * ROWB);
#pragma unroll
        for (int h = 0; h < REP; ++h) mfma_acc(o[h][dt], vf, pb[h][ks]);
      }
    return true;
  };
  int kt = 0;
#pragma nounroll
  for (; kt < nkt; ++kt) {
    if (kt + 1 < nkt) dma(kt + 1, smem + ((kt + 1) & 1) * 2 * TB);  // that stage's last reads: before the barrier
    if (!tile(kt, std::false_type())) break;
    __builtin_amdgcn_s_waitcnt(0);  // the next tile's DMA landed (this wave's pieces) ...
    __syncthreads();                 // ... and every wave's; every wave is done reading this stage
  }
  if (kt < nkt) {  // rare: a score jumped past m + THR_FAST; tile kt again with rescaling, then the rest
    nop_mfma();
#pragma nounroll
    for (int k2 = kt; k2 < nkt; ++k2) {
      if (k2 > kt && k2 + 1 < nkt) dma(k2 + 1, smem + ((k2 + 1) & 1) * 2 * TB);
      tile(k2, std::true_type());
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
  }
  nop_mfma();
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    float lt = l[h];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (qok) {
      const int hq = kvh * REP + h;
      u16* op = out + (long)(start + qrow) * nq * D + hq * D + 4 * g;
      const float inv = 1.f / lt;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) store4(op + 16 * dt, o[h][dt], inv);
      if (g == 0) lse[(long)hq * total + start + qrow] = (m[h] + log2f(lt)) * LN2;
    }
  }
}

// v6 dQ (recompute, GQA-stacked): the fwd6 geometry — one workgroup per (kv head, sequence, 64-query block), wave w
// owns positions q0 + 16 w .. + 15 for all REP query heads — recomputing S^T = K Q^T and dP^T = V dO^T per 64-key
// tile, dS^T = P o (dP - delta) with P = exp2(S sl2 - lse) (lse and delta are per-lane scalars in this layout: lane
// (g, r) holds query r), and dQ^T += K^T dS^T. Every K row / V row / K^T fragment read from LDS feeds REP MFMAs. Against
// dq4 it triples the MFMA work but drops the lp x lp bf16 dS^T round trip through HBM (stores in the dK/dV kernel,
// loads here). Q and dO fragments and the dQ accumulators live in AGPRs (MFMA B / C operands), S and dP in VGPRs.
__device__ __forceinline__ void pin_frag(bf16x8& x) { asm volatile("" : "+a"(x)); }
__device__ __forceinline__ f32x4 mfma_v0_a(const bf16x8& a, const bf16x8& b) {
  f32x4 d;
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "a"(b));
  return d;
}
__device__ __forceinline__ void mfma_v_a(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "a"(b));
}

template <int REP>
__global__ __launch_bounds__(256, 1) void dq6_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     const int* __restrict__ cu, u16* __restrict__ dqkv, int nq,
                                                     int nkv, int total, float sl2, float scale, int causal,
                                                     const float* __restrict__ rcos, const float* __restrict__ rsin) {
  constexpr int TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];  // stage s: K image at 2 s TB, V image at (2 s + 1) TB
  const int kvh = blockIdx.x, b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * 64;
  if (q0 >= len) return;
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int wfirst = q0 + 16 * w, qrow = wfirst + (lane & 15);
  const bool qok = qrow < len;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min(qb + 1, nkb) : nkb;
  const int r0 = 4 * w + (lane >> 4);  // DMA as fwd6
  const u16* kvsrc = qkv + (long)start * ld + (nq + kvh) * D + 8 * swz(r0, lane & 15);
  auto dma = [&](int kt, char* stage) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u16* src = kvsrc + (long)min(kt * 64 + r0 + 16 * j, len - 1) * ld;
      glds16(src, stage + (w + 4 * j) * 1024);
      glds16(src + nkv * D, stage + TB + (w + 4 * j) * 1024);
    }
  };
  dma(0, smem);
  Offs off;
  off.init(lane);
  bf16x8 qf[REP][4], df[REP][4];
  float lse2[REP], dl[REP];
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    const int hq = kvh * REP + h;
    const u16* qp = qkv + (long)(start + qrow) * ld + hq * D + 8 * g;
    const u16* dp = dout + (long)(start + qrow) * ldo + hq * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[h][s] = load_frag_global(qp + 32 * s, qok);
      df[h][s] = load_frag_global(dp + 32 * s, qok);
      pin_frag(qf[h][s]);
      pin_frag(df[h][s]);
    }
    lse2[h] = qok ? lse[(long)hq * total + start + qrow] * LOG2E : 0.f;
    dl[h] = qok ? delta[(long)hq * total + start + qrow] : 0.f;
  }
  f32x4 dq[REP][8];
#pragma unroll
  for (int h = 0; h < REP; ++h)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      dq[h][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
      pin_acc(dq[h][dt]);
    }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  nop_mfma();  // AGPR writes of the Q / dO fragments -> MFMA operand reads
#pragma nounroll
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const char* Ks = smem + (kt & 1) * 2 * TB;
    const char* Vs = Ks + TB;
    if (kt + 1 < nkt) dma(kt + 1, smem + ((kt + 1) & 1) * 2 * TB);
    f32x4 sc[REP][4], dp[REP][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = lds_row(Ks, off.row[s] + nt * 16 * ROWB);
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          if (s == 0) sc[h][nt] = mfma_v0_a(kf, qf[h][s]);
          else mfma_v_a(sc[h][nt], kf, qf[h][s]);
        }
      }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 vf = lds_row(Vs, off.row[s] + nt * 16 * ROWB);
#pragma unroll
        for (int h = 0; h < REP; ++h) {
          if (s == 0) dp[h][nt] = mfma_v0_a(vf, df[h][s]);
          else mfma_v_a(dp[h][nt], vf, df[h][s]);
        }
      }
    nop_mfma();
    const bool need_mask = (k0 + 64 > len) || (causal && k0 + 63 > wfirst);
    bf16x8 db[REP][2];
#pragma unroll
    for (int h = 0; h < REP; ++h) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float p = exp2f(fmaf(sc[h][nt][i], sl2, -lse2[h]));
          if (need_mask) {
            const int key = k0 + 16 * nt + 4 * g + i;
            if (key >= len || (causal && key > qrow)) p = 0.f;
          }
          dp[h][nt][i] = p * (dp[h][nt][i] - dl[h]);
        }
      db[h][0] = pack_acc(dp[h][0], dp[h][1]);
      db[h][1] = pack_acc(dp[h][2], dp[h][3]);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const bf16x8 kt_f = lds_tr(Ks, off.tr[dt] + ks * 32 * ROWB);
#pragma unroll
        for (int h = 0; h < REP; ++h) mfma_acc(dq[h][dt], kt_f, db[h][ks]);
      }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  nop_mfma();
  if (!qok) return;
#pragma unroll
  for (int h = 0; h < REP; ++h) {
    u16* qp = dqkv + (long)(start + qrow) * ld + (kvh * REP + h) * D + 4 * g;
    if (rcos != nullptr) {
      const long tr = (long)(start + qrow) * (D / 2) + 4 * g;
      store4_rope_bwd(qp, dq[h], scale, rcos + tr, rsin + tr);
    } else {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) store4(qp + 16 * dt, dq[h][dt], scale);
    }
  }
}

// One key tile of the LDS-DMA dq4 (bwd_dq4_kernel<8, false, true>): issue the next tile's K / dS^T pieces into stage
// nxt (2 x 1 KB per image per wave, source-swizzled; rows past the sequence end are ZERO-filled with LDS stores, as
// dQ sums K x dS^T over keys and the dS^T rows there were never written), then dQ^T += K^T dS^T from stage cur.
// cur / nxt: __restrict__ parameters of one frame (see fwd_step_dma).
__device__ __forceinline__ void dq_step_dma(const char* __restrict__ cur, char* __restrict__ nxt, bool pre, bool active,
                                            const u16* ksrc, const u16* ssrc, long ld, long lp, int row0, int len,
                                            long coff, int wave, int lane, int trw, const Offs& off, f32x4 (&dq)[8]) {
  constexpr int TB = 64 * ROWB;
  if (pre) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = row0 + 32 * j;
      char* dk = nxt + (wave + 8 * j) * 1024;
      if (row < len) {
        lds_dma16(ksrc + row * ld + coff, dk);
        lds_dma16(ssrc + row * lp + coff, dk + TB);
      } else {
        *(uint4*)(dk + 16 * lane) = make_uint4(0, 0, 0, 0);
        *(uint4*)(dk + TB + 16 * lane) = make_uint4(0, 0, 0, 0);
      }
    }
  }
  if (!active) return;
  const char* Ks = cur;
  const char* Ss = cur + TB;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bf16x8 db = lds_tr(Ss, trw + ks * 32 * ROWB);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) dq[dt] = mfma(lds_tr(Ks, off.tr[dt] + ks * 32 * ROWB), db, dq[dt]);
  }
}

// dQ from the materialised dS (v4 backward): bwd_dkdv3_kernel already computes dS = P o (dP - delta) for
// every (query, key) pair of a head; it stores it transposed, dS^T[b][h][key][query] (bf16, lp x lp per head),
// so dQ^T = K^T dS^T is ONE MFMA product per 64-key tile here — 16 MFMA per wave per tile instead of the 48 of
// dq3 (which recomputes S and dP), no exp2 / softmax VALU, no lse / delta reads. The dS^T tile [64 keys][128
// queries] is staged exactly like a K/V image and read with the same transposed reads (query column block =
// the wave's 16 rows), so both MFMA operands come from LDS. Rows past the sequence end are zero-filled by the
// stager; entries never written by dkdv (queries past the last 64-query tile, key tiles above a wave's causal
// diagonal) are never used: a wave skips tiles above its diagonal and each query column is independent.
template <int NW, bool LEG = false, bool DMA = false>
__global__ __launch_bounds__(NW * 64, 4) void bwd_dq4_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dst,
                                                          const int* __restrict__ cu, u16* __restrict__ dqkv, int nq,
                                                          int nkv, int lp, float scale, int causal,
                                                          const float* __restrict__ rcos = nullptr,
                                                          const float* __restrict__ rsin = nullptr) {
  static_assert(NW == 8, "the dS^T image is 128 queries wide: 8 waves x 16 rows");
  constexpr int NT = NW * 64, BM = NW * 16, TB = 64 * ROWB;
  static_assert(!DMA || !LEG, "the LDS-DMA variant has the current schedule only");
  __shared__ __attribute__((aligned(16))) char smem[(DMA ? 4 : 2) * TB];  // DMA: two stages of (K, dS^T) images
  char* Ks = smem;
  char* Ss = smem + TB;
  // grid (heads, sequences, q-blocks) with the last (causally heaviest) q-block dispatched first: LPT order
  const int h = blockIdx.x, b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int q0 = qb * BM;
  if (q0 >= len) return;
  SFT_DASSERT(q0 + BM <= lp);
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wfirst = q0 + wave * 16;
  const int qrow = wfirst + (lane & 15);
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* sbase = dst + (long)(b * nq + h) * lp * lp + q0;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  Offs off;
  off.init(lane);
  // the wave's own dS^T column block: computed, not off.tr[wave] (a runtime index into a register array sends
  // the array to scratch, and the scratch load in the loop waited on the next tile's prefetch: vmcnt(0))
  int trw;
  if constexpr (LEG) {
    trw = off.tr[wave];
  } else {
    const int r = lane & 15, q = r >> 2, p = r & 3;
    trw = img_off(4 * g + q, 2 * wave + (p >> 1)) + 8 * (p & 1);
  }
  f32x4 dq[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // DMA: lane (wave w, l) fills image rows 4 (w + 8 j) + (l >> 4), position l & 15 with chunk swz(row, l & 15)
  const int r0 = 4 * wave + (lane >> 4);
  const long coff = 8 * swz(r0, lane & 15);
  if constexpr (DMA) {  // tile 0 into stage 0 (the "next" tile of a virtual tile -1)
    dq_step_dma(smem + 2 * TB, smem, true, false, kbase, sbase, ld, lp, r0, len, coff, wave, lane, trw, off, dq);
  } else {
    Stage<64, NT> tk, ts;
    tk.load(kbase, ld, len, tid);
    ts.load(sbase, lp, len, tid);
    tk.store(Ks, tid);
    ts.store(Ss, tid);
  }
  if constexpr (DMA) vm_drain();
  __syncthreads();
  if constexpr (DMA) {
    for (int kt = 0; kt < nkt; ++kt) {
      const int k0 = kt * 64;
      const bool pre = kt + 1 < nkt;
      dq_step_dma(smem + (kt & 1) * 2 * TB, smem + ((kt + 1) & 1) * 2 * TB, pre, !causal || k0 <= wfirst + 15, kbase,
                  sbase, ld, lp, k0 + 64 + r0, len, coff, wave, lane, trw, off, dq);
      if (pre) vm_drain();  // this lane's pieces of the next tile landed ...
      __syncthreads();      // ... and every lane's (LDS zero stores too); every wave is done reading this stage
    }
  }
  for (int kt = 0; kt < (DMA ? 0 : nkt); ++kt) {
    const int k0 = kt * 64;
    const bool pre = kt + 1 < nkt;
    Stage<64, NT> tk, ts;
    if (pre) {
      tk.load(kbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
      ts.load(sbase + (long)(k0 + 64) * lp, lp, len - k0 - 64, tid);
    }
    if (!causal || k0 <= wfirst + 15) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 db = lds_tr(Ss, trw + ks * 32 * ROWB);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) dq[dt] = mfma(lds_tr(Ks, off.tr[dt] + ks * 32 * ROWB), db, dq[dt]);
      }
    }
    if (pre) {
      __syncthreads();
      tk.store(Ks, tid);
      ts.store(Ss, tid);
    }
    __syncthreads();
  }
  if (qrow < len) {
    u16* qp = dqkv + (long)(start + qrow) * ld + h * D + 4 * g;
    if (rcos != nullptr) {
      const long tr = (long)(start + qrow) * (D / 2) + 4 * g;
      store4_rope_bwd(qp, dq, scale, rcos + tr, rsin + tr);
    } else {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) store4(qp + 16 * dt, dq[dt], scale);
    }
  }
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void bwd_dq3_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta, const int* __restrict__ cu,
                                                          u16* __restrict__ dqkv, int nq, int nkv, int total,
                                                          float sl2, float scale, int causal) {
  constexpr int NT = NW * 64, BM = NW * 16, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * TB];
  char* Ks = smem;
  char* Vs = smem + TB;
  // grid (heads, sequences, q-blocks) with the last (causally heaviest) q-block dispatched first: LPT order
  const int h = blockIdx.x, b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * BM;
  if (q0 >= len) return;
  const int kvh = h / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wfirst = q0 + wave * 16;
  const int qrow = wfirst + (lane & 15);
  const bool qok = qrow < len;
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* vbase = qkv + (long)start * ld + (nq + nkv + kvh) * D;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((q0 + BM + 63) / 64, nkb) : nkb;
  Offs off;
  off.init(lane);
  {
    Stage<64, NT> tk, tv;
    tk.load(kbase, ld, len, tid);
    tv.load(vbase, ld, len, tid);
    tk.store(Ks, tid);
    tv.store(Vs, tid);
  }
  bf16x8 qf[4], df[4];
  {
    const u16* qp = qkv + (long)(start + qrow) * ld + h * D + 8 * g;
    const u16* dp = dout + (long)(start + qrow) * ldo + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = load_frag_global(qp + 32 * s, qok);
      df[s] = load_frag_global(dp + 32 * s, qok);
    }
  }
  const float lse2 = qok ? lse[(long)h * total + start + qrow] * LOG2E : 0.f;
  const float dl = qok ? delta[(long)h * total + start + qrow] : 0.f;
  f32x4 dq[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const bool pre = kt + 1 < nkt;
    Stage<64, NT> tk, tv;
    if (pre) {
      tk.load(kbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
      tv.load(vbase + (long)(k0 + 64) * ld, ld, len - k0 - 64, tid);
    }
    if (!causal || k0 <= wfirst + 15) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc[nt] = mfma(lds_row(Ks, off.row[s] + nt * 16 * ROWB), qf[s], sc[nt]);
          dp[nt] = mfma(lds_row(Vs, off.row[s] + nt * 16 * ROWB), df[s], dp[nt]);
        }
      }
      const bool need_mask = (k0 + 64 > len) || (causal && k0 + 63 > wfirst) || (q0 + BM > len);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float p = exp2f(fmaf(sc[nt][i], sl2, -lse2));
          if (need_mask) {
            const int key = k0 + 16 * nt + 4 * g + i;
            if (key >= len || (causal && key > qrow) || !qok) p = 0.f;
          }
          dp[nt][i] = p * (dp[nt][i] - dl);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) dq[dt] = mfma(lds_tr(Ks, off.tr[dt] + ks * 32 * ROWB), db, dq[dt]);
      }
    }
    if (pre) {
      __syncthreads();
      tk.store(Ks, tid);
      tv.store(Vs, tid);
    }
    __syncthreads();
  }
  if (qok) {
    u16* qp = dqkv + (long)(start + qrow) * ld + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(qp + 16 * dt, dq[dt], scale);
  }
}

__global__ __launch_bounds__(256, 2) void bwd_dkdv3_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           const int* __restrict__ cu, float* __restrict__ part,
                                                           u16* __restrict__ dqkv, int nq, int nkv, int total,
                                                           float sl2, float scale, int causal,
                                                           u16* __restrict__ dst = nullptr, int lp = 0) {
  constexpr int NT = 256, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * TB + 2 * 64 * 4];
  char* Qs = smem;
  char* Os = smem + TB;
  float* Ls = (float*)(smem + 2 * TB);
  float* Dl = Ls + 64;
  // grid (heads, sequences, key blocks): key block 0 (causally heaviest: every query tile) dispatched first
  const int h = blockIdx.x, b = blockIdx.y, kb = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int k0 = kb * 64;
  if (k0 >= len) return;
  const int rep = nq / nkv;
  const int kvh = h / rep, r = h - kvh * rep;
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wfirst = k0 + wave * 16;
  const int key = wfirst + (lane & 15);
  const bool kok = key < len;
  const u16* qbase = qkv + (long)start * ld + h * D;
  const u16* obase = dout + (long)start * ldo + h * D;
  const float* lbase = lse + (long)h * total + start;
  const float* dbase = delta + (long)h * total + start;
  const int qt0 = causal ? kb : 0;
  const int nqt = (len + 63) / 64;
  Offs off;
  off.init(lane);
  {
    const int q0 = qt0 * 64, qv = len - q0;
    Stage<64, NT> tq, to;
    tq.load(qbase + (long)q0 * ld, ld, qv, tid);
    to.load(obase + (long)q0 * ldo, ldo, qv, tid);
    tq.store(Qs, tid);
    to.store(Os, tid);
    if (tid < 64) {
      Ls[tid] = tid < qv ? lbase[q0 + tid] * LOG2E : 0.f;
      Dl[tid] = tid < qv ? dbase[q0 + tid] : 0.f;
    }
  }
  bf16x8 kf[4], vf[4];
  {
    const u16* kp = qkv + (long)(start + key) * ld + (nq + kvh) * D + 8 * g;
    const u16* vp = qkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = load_frag_global(kp + 32 * s, kok);
      vf[s] = load_frag_global(vp + 32 * s, kok);
    }
  }
  f32x4 dk[8], dv[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  for (int qt = qt0; qt < nqt; ++qt) {
    const int q0 = qt * 64;
    const bool pre = qt + 1 < nqt;
    Stage<64, NT> tq, to;
    float pl = 0.f, pd = 0.f;
    if (pre) {
      const int qn = q0 + 64, qv = len - qn;
      tq.load(qbase + (long)qn * ld, ld, qv, tid);
      to.load(obase + (long)qn * ldo, ldo, qv, tid);
      if (tid < 64 && tid < qv) {
        pl = lbase[qn + tid] * LOG2E;
        pd = dbase[qn + tid];
      }
    }
    if (!causal || wfirst <= q0 + 63) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc[mt] = mfma(lds_row(Qs, off.row[s] + mt * 16 * ROWB), kf[s], sc[mt]);
          dp[mt] = mfma(lds_row(Os, off.row[s] + mt * 16 * ROWB), vf[s], dp[mt]);
        }
      }
      const bool need_mask = (q0 + 64 > len) || (causal && wfirst + 15 > q0);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const float4 L4 = *(const float4*)(Ls + 16 * mt + 4 * g);
        const float4 D4 = *(const float4*)(Dl + 16 * mt + 4 * g);
        const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float p = exp2f(fmaf(sc[mt][i], sl2, -Lv[i]));
          if (need_mask) {
            const int q = q0 + 16 * mt + 4 * g + i;
            if (q >= len || (causal && key > q)) p = 0.f;
          }
          sc[mt][i] = p;
          dp[mt][i] = p * (dp[mt][i] - Dv[i]);
        }
      }
      if (dst != nullptr && kok) {  // dS^T row of this lane's key: 4 consecutive queries per fragment (bf16)
        u16* drow = dst + ((long)(b * nq + h) * lp + key) * lp + q0 + 4 * g;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store4(drow + 16 * mt, dp[mt], 1.f);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
        const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          dv[dt] = mfma(lds_tr(Os, off.tr[dt] + ks * 32 * ROWB), pb, dv[dt]);
          dk[dt] = mfma(lds_tr(Qs, off.tr[dt] + ks * 32 * ROWB), db, dk[dt]);
        }
      }
    }
    if (pre) {
      __syncthreads();
      tq.store(Qs, tid);
      to.store(Os, tid);
      if (tid < 64) {
        Ls[tid] = pl;
        Dl[tid] = pd;
      }
    }
    __syncthreads();
  }
  if (!kok) return;
  if (rep == 1) {
    u16* kp = dqkv + (long)(start + key) * ld + (nq + kvh) * D + 4 * g;
    u16* vp = dqkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      store4(kp + 16 * dt, dk[dt], scale);
      store4(vp + 16 * dt, dv[dt], 1.f);
    }
    return;
  }
  const long pld = 2L * nkv * D;
  float* pk = part + ((long)r * total + start + key) * pld + kvh * D + 4 * g;
  float* pv = pk + (long)nkv * D;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    *(float4*)(pk + 16 * dt) = make_float4(dk[dt][0], dk[dt][1], dk[dt][2], dk[dt][3]);
    *(float4*)(pv + 16 * dt) = make_float4(dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
  }
}

// GQA-grouped dK/dV (v5): one workgroup per (kv head, sequence, 64-key block) walks the query tiles of ALL
// rep = nq / nkv query heads that share the kv head, keeping K/V fragments and the dK/dV accumulators in
// registers across heads. dK/dV are written once, in bf16, straight into dqkv: no rep x [total, 2*nkv*128] fp32
// partial slabs (134 MB written + re-read at 16 x 512 tokens, 16q/4kv) and no dkdv_reduce pass. The per-tile
// math (S^T, dP^T, dS^T store for dq4) is bwd_dkdv3_kernel's; the iteration space is flattened over
// (head, query tile) so the register prefetch of the next tile crosses head boundaries.
// G = 2 (default when rep is even): the workgroup is two 4-wave groups over the SAME 64 keys, each walking half
// of the heads with its own Q/dO LDS images; group 1 hands its fp32 dK/dV to group 0 through LDS at the end.
// That halves the serial chain of the causally heaviest key block (block 0 walks rep x nqt tiles), which is what
// bounds this kernel: at 16 x 512 tokens the MFMA work alone is ~18 us, one tile step ~3 us of latency.
// blockIdx.z = key block, heaviest first.
// One query tile of the LDS-DMA GQA dK/dV kernel (bwd_dkdv5_kernel<G, false, true>): issue the next tile's Q / dO
// pieces (4 x 1 KB per image per wave, source-swizzled, rows past the sequence end clamped: their P and dS are masked
// to 0) and its lse / delta loads, compute this tile from stage cur, then park lse (x LOG2E) / delta in stage nxt.
// cur / nxt are __restrict__ parameters of one frame (see fwd_step_dma). Stage: Q image, dO image, lse[64], delta[64].
__device__ __forceinline__ void dkdv_step_dma(const char* __restrict__ cur, char* __restrict__ nxt, bool pre, bool active,
                                              const u16* qsrc, const u16* osrc, long ld, long ldo, int qrow0, int qlast,
                                              long kvoff, int wave, const float* lsrc, const float* dsrc, int gtid,
                                              int q0, int len, int causal, int key, int wfirst, int g, float sl2,
                                              u16* drow, const Offs& off, const bf16x8 (&kf)[4],
                                              const bf16x8 (&vf)[4], f32x4 (&dk)[8], f32x4 (&dv)[8]) {
  constexpr int TB = 64 * ROWB;
  float pl = 0.f, pd = 0.f;
  if (pre) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long row = min(qrow0 + 16 * j, qlast);
      lds_dma16(qsrc + row * ld + kvoff, nxt + (wave + 4 * j) * 1024);
      lds_dma16(osrc + row * ldo + kvoff, nxt + TB + (wave + 4 * j) * 1024);
    }
    if (gtid < 64 && lsrc != nullptr) {
      pl = lsrc[gtid];
      pd = dsrc[gtid];
    }
  }
  if (active) {
    const char* Qs = cur;
    const char* Os = cur + TB;
    const float* Ls = (const float*)(cur + 2 * TB);
    const float* Dl = Ls + 64;
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc[mt] = mfma(lds_row(Qs, off.row[s] + mt * 16 * ROWB), kf[s], sc[mt]);
        dp[mt] = mfma(lds_row(Os, off.row[s] + mt * 16 * ROWB), vf[s], dp[mt]);
      }
    }
    const bool need_mask = (q0 + 64 > len) || (causal && wfirst + 15 > q0);
    const int qb0 = q0 + 4 * g;
    const int lo = (causal ? key : 0) - qb0, hi = len - 1 - qb0;
    const f32x2 sl = {sl2, sl2};
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const float4 L4 = *(const float4*)(Ls + 16 * mt + 4 * g);
      const float4 D4 = *(const float4*)(Dl + 16 * mt + 4 * g);
      const f32x2 L[2] = {{-L4.x, -L4.y}, {-L4.z, -L4.w}}, Dd[2] = {{D4.x, D4.y}, {D4.z, D4.w}};
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const f32x2 t = __builtin_elementwise_fma(f32x2{sc[mt][i], sc[mt][i + 1]}, sl, L[i / 2]);
        f32x2 p = {exp2f(t.x), exp2f(t.y)};
        if (need_mask) {
          const int o = 16 * mt + i;
          p.x = (o < lo || o > hi) ? 0.f : p.x;
          p.y = (o + 1 < lo || o + 1 > hi) ? 0.f : p.y;
        }
        const f32x2 d = p * (f32x2{dp[mt][i], dp[mt][i + 1]} - Dd[i / 2]);
        sc[mt][i] = p.x;
        sc[mt][i + 1] = p.y;
        dp[mt][i] = d.x;
        dp[mt][i + 1] = d.y;
      }
    }
    if (drow != nullptr) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) store4(drow + 16 * mt, dp[mt], 1.f);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
      const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        dv[dt] = mfma(lds_tr(Os, off.tr[dt] + ks * 32 * ROWB), pb, dv[dt]);
        dk[dt] = mfma(lds_tr(Qs, off.tr[dt] + ks * 32 * ROWB), db, dk[dt]);
      }
    }
  }
  if (pre && gtid < 64) {  // the next stage's lse / delta (that stage's last reads ended at the previous barrier)
    float* Ln = (float*)(nxt + 2 * TB);
    asm volatile("" : "+v"(pl));  // keeps the multiply (and the loads' wait) after this tile's math
    Ln[gtid] = pl * LOG2E;
    Ln[64 + gtid] = pd;
  }
}

template <int G, bool LEG = false, bool DMA = false>
__global__ __launch_bounds__(256 * G, G == 1 ? 2 : 1) void bwd_dkdv5_kernel(
    const u16* __restrict__ qkv, const u16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, const int* __restrict__ cu, u16* __restrict__ dqkv, int nq, int nkv, int total,
    float sl2, float scale, int causal, u16* __restrict__ dst, int lp, const float* __restrict__ rcos,
    const float* __restrict__ rsin) {
  constexpr int NT = 256, TB = 64 * ROWB, GB = 2 * TB + 2 * 64 * 4;  // per group: Q, dO images + lse, delta
  static_assert(!DMA || !LEG, "the LDS-DMA variant has the current schedule only");
  __shared__ __attribute__((aligned(16))) char smem[G * GB * (DMA ? 2 : 1)];  // DMA: two stages per group
  const int tid = threadIdx.x, grp = tid >> 8, gtid = tid & 255;
  char* Qs = smem + grp * GB * (DMA ? 2 : 1);
  char* Os = Qs + TB;
  float* Ls = (float*)(Qs + 2 * TB);
  float* Dl = Ls + 64;
  const int kvh = blockIdx.x, b = blockIdx.y, kb = blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int k0 = kb * 64;
  if (k0 >= len) return;
  const int rep = nq / nkv, hpg = rep / G;  // heads per group
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int lane = tid & 63, wave = (tid >> 6) & 3, g = lane >> 4;
  const int wfirst = k0 + wave * 16;
  const int key = wfirst + (lane & 15);
  const bool kok = key < len;
  const int qt0 = causal ? kb : 0;
  const int nqt = (len + 63) / 64;
  const int nt = nqt - qt0;        // query tiles per head
  const int niter = hpg * nt;      // the same in every group: the loop's barriers line up
  Offs off;
  off.init(lane);
  // iteration it -> head h = kvh * rep + grp * hpg + it / nt, query tile qt0 + it % nt (kept incrementally)
  int h = kvh * rep + grp * hpg, qt = qt0;
  // DMA: lane (wave w, l) fills image rows 4 (w + 4 j) + (l >> 4), position l & 15 with chunk swz(row, l & 15)
  const int qr0 = 4 * wave + (lane >> 4);
  const long qoff = 8 * swz(qr0, lane & 15);
  {
    const int q0 = qt0 * 64, qv = len - q0;
    if constexpr (DMA) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long row = start + min(q0 + qr0 + 16 * j, len - 1);
        lds_dma16(qkv + row * ld + h * D + qoff, Qs + (wave + 4 * j) * 1024);
        lds_dma16(dout + row * ldo + h * D + qoff, Os + (wave + 4 * j) * 1024);
      }
    } else {
      Stage<64, NT> tq, to;
      tq.load(qkv + (long)(start + q0) * ld + h * D, ld, qv, gtid);
      to.load(dout + (long)(start + q0) * ldo + h * D, ldo, qv, gtid);
      tq.store(Qs, gtid);
      to.store(Os, gtid);
    }
    if (gtid < 64) {
      Ls[gtid] = gtid < qv ? lse[(long)h * total + start + q0 + gtid] * LOG2E : 0.f;
      Dl[gtid] = gtid < qv ? delta[(long)h * total + start + q0 + gtid] : 0.f;
    }
  }
  bf16x8 kf[4], vf[4];
  {
    const u16* kp = qkv + (long)(start + key) * ld + (nq + kvh) * D + 8 * g;
    const u16* vp = qkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = load_frag_global(kp + 32 * s, kok);
      vf[s] = load_frag_global(vp + 32 * s, kok);
    }
  }
  if constexpr (!LEG) vm_drain();  // see vm_drain: K / V fragments are loop-invariant MFMA operands
  f32x4 dk[8], dv[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  if constexpr (DMA) {
    for (int it = 0; it < niter; ++it) {
      const int q0 = qt * 64;
      const bool pre = it + 1 < niter;
      int hn = h, qtn = qt + 1;
      if (qtn == nqt) {
        qtn = qt0;
        ++hn;
      }
      const int qn = qtn * 64;
      const long lo = (long)hn * total + start + qn;
      const bool lok = pre && qn + gtid < len;
      char* cur = Qs + (it & 1) * GB;
      char* nxt = Qs + ((it + 1) & 1) * GB;
      u16* drow = (dst != nullptr && kok) ? dst + ((long)(b * nq + h) * lp + key) * lp + q0 + 4 * g : nullptr;
      dkdv_step_dma(cur, nxt, pre, !causal || wfirst <= q0 + 63, qkv + (long)start * ld + hn * D,
                    dout + (long)start * ldo + hn * D, ld, ldo, qn + qr0, len - 1, qoff, wave,
                    lok ? lse + lo : nullptr, delta + lo, gtid, q0, len, causal, key, wfirst, g, sl2, drow, off, kf,
                    vf, dk, dv);
      if (pre) vm_drain();  // this lane's pieces of the next tile landed ...
      __syncthreads();      // ... and every lane's; every wave is done reading this stage
      h = hn;
      qt = qtn;
    }
  }
  for (int it = 0; it < (DMA ? 0 : niter); ++it) {
    const int q0 = qt * 64;
    const bool pre = it + 1 < niter;
    int hn = h, qtn = qt + 1;
    if (qtn == nqt) {
      qtn = qt0;
      ++hn;
    }
    Stage<64, NT> tq, to;
    float pl = 0.f, pd = 0.f;
    if (pre) {
      const int qn = qtn * 64, qv = len - qn;
      tq.load(qkv + (long)(start + qn) * ld + hn * D, ld, qv, gtid);
      to.load(dout + (long)(start + qn) * ldo + hn * D, ldo, qv, gtid);
      if (gtid < 64 && gtid < qv) {
        // the LOG2E scaling happens at the LDS store: a multiply here made the compiler wait for this load, and
        // with it (in-order vmcnt) for the Q / dO prefetch issued just before
        pl = lse[(long)hn * total + start + qn + gtid];
        if constexpr (LEG) pl *= LOG2E;
        pd = delta[(long)hn * total + start + qn + gtid];
      }
    }
    if (!causal || wfirst <= q0 + 63) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        sc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc[mt] = mfma(lds_row(Qs, off.row[s] + mt * 16 * ROWB), kf[s], sc[mt]);
          dp[mt] = mfma(lds_row(Os, off.row[s] + mt * 16 * ROWB), vf[s], dp[mt]);
        }
      }
      const bool need_mask = (q0 + 64 > len) || (causal && wfirst + 15 > q0);
      if constexpr (LEG) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const float4 L4 = *(const float4*)(Ls + 16 * mt + 4 * g);
          const float4 D4 = *(const float4*)(Dl + 16 * mt + 4 * g);
          const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float p = exp2f(fmaf(sc[mt][i], sl2, -Lv[i]));
            if (need_mask) {
              const int q = q0 + 16 * mt + 4 * g + i;
              if (q >= len || (causal && key > q)) p = 0.f;
            }
            sc[mt][i] = p;
            dp[mt][i] = p * (dp[mt][i] - Dv[i]);
          }
        }
      } else {  // packed fp32 pairs around the exp2; the mask as one compare per score (query offset 16 mt + i
                // visible iff first <= it <= last)
        const int qb0 = q0 + 4 * g;
        const int lo = (causal ? key : 0) - qb0, hi = len - 1 - qb0;
        const f32x2 sl = {sl2, sl2};
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const float4 L4 = *(const float4*)(Ls + 16 * mt + 4 * g);
          const float4 D4 = *(const float4*)(Dl + 16 * mt + 4 * g);
          const f32x2 L[2] = {{-L4.x, -L4.y}, {-L4.z, -L4.w}}, Dd[2] = {{D4.x, D4.y}, {D4.z, D4.w}};
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const f32x2 t = __builtin_elementwise_fma(f32x2{sc[mt][i], sc[mt][i + 1]}, sl, L[i / 2]);
            f32x2 p = {exp2f(t.x), exp2f(t.y)};
            if (need_mask) {
              const int o = 16 * mt + i;
              p.x = (o < lo || o > hi) ? 0.f : p.x;
              p.y = (o + 1 < lo || o + 1 > hi) ? 0.f : p.y;
            }
            const f32x2 d = p * (f32x2{dp[mt][i], dp[mt][i + 1]} - Dd[i / 2]);
            sc[mt][i] = p.x;
            sc[mt][i + 1] = p.y;
            dp[mt][i] = d.x;
            dp[mt][i + 1] = d.y;
          }
        }
      }
      if (dst != nullptr && kok) {
        u16* drow = dst + ((long)(b * nq + h) * lp + key) * lp + q0 + 4 * g;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store4(drow + 16 * mt, dp[mt], 1.f);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack_acc(sc[2 * ks], sc[2 * ks + 1]);
        const bf16x8 db = pack_acc(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          dv[dt] = mfma(lds_tr(Os, off.tr[dt] + ks * 32 * ROWB), pb, dv[dt]);
          dk[dt] = mfma(lds_tr(Qs, off.tr[dt] + ks * 32 * ROWB), db, dk[dt]);
        }
      }
    }
    if (pre) {
      __syncthreads();
      tq.store(Qs, gtid);
      to.store(Os, gtid);
      if (gtid < 64) {
        if constexpr (!LEG) asm volatile("" : "+v"(pl));  // keeps the multiply (and the load's wait) here
        Ls[gtid] = LEG ? pl : pl * LOG2E;
        Dl[gtid] = pd;
      }
    }
    __syncthreads();
    h = hn;
    qt = qtn;
  }
  if constexpr (G == 2) {
    // group 1 -> LDS (fp32, [wave][dt][lane] float4: consecutive lanes, conflict-free) -> group 0 adds.
    // 2 x 4 waves x 8 x 64 x 16 B = 64 KB = both groups' Q/dO images, free after the loop's last barrier.
    float4* xk = (float4*)smem;
    float4* xv = xk + 4 * 8 * 64;
    if (grp == 1) {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        xk[(wave * 8 + dt) * 64 + lane] = make_float4(dk[dt][0], dk[dt][1], dk[dt][2], dk[dt][3]);
        xv[(wave * 8 + dt) * 64 + lane] = make_float4(dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
      }
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const float4 a = xk[(wave * 8 + dt) * 64 + lane], c = xv[(wave * 8 + dt) * 64 + lane];
      dk[dt] += f32x4{a.x, a.y, a.z, a.w};
      dv[dt] += f32x4{c.x, c.y, c.z, c.w};
    }
  }
  if (!kok) return;
  u16* kp = dqkv + (long)(start + key) * ld + (nq + kvh) * D + 4 * g;
  u16* vp = dqkv + (long)(start + key) * ld + (nq + nkv + kvh) * D + 4 * g;
  if (rcos != nullptr) {
    const long tr = (long)(start + key) * (D / 2) + 4 * g;
    store4_rope_bwd(kp, dk, scale, rcos + tr, rsin + tr);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) store4(vp + 16 * dt, dv[dt], 1.f);
    return;
  }
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    store4(kp + 16 * dt, dk[dt], scale);
    store4(vp + 16 * dt, dv[dt], 1.f);
  }
}

// SFTAMD_ATTN_LEGWAIT=1: the round-2 instruction schedule of fwd3 / dq4 / dK-dV v5 (prefetch latency exposed by
// compiler-inserted vmcnt(0) waits), kept for same-process A/B timing only (tools/bench_attention.py ATTN_LEG=1)
static bool attn_legacy_wait() {
  const char* e = std::getenv("SFTAMD_ATTN_LEGWAIT");
  return e && e[0] == '1';
}

// host launcher: G = 2 head groups when rep is even (SFTAMD_ATTN_GQA_SPLIT=0 forces 1)
static void launch_dkdv5(const u16* qkv, const u16* dout, const float* lse, const float* delta, const int* cu,
                         u16* dqkv, int nq, int nkv, int total, int nseq, int max_seqlen, float sl2, float scale,
                         int causal, u16* dst, int lp, hipStream_t st, const float* rcos = nullptr,
                         const float* rsin = nullptr) {
  const int rep = nq / nkv;
  const char* e = std::getenv("SFTAMD_ATTN_GQA_SPLIT");
  const bool split = rep % 2 == 0 && !(e && e[0] == '0');
  dim3 grid(nkv, nseq, (max_seqlen + 63) / 64);
  const bool leg = attn_legacy_wait();
  const char* ed = std::getenv("SFTAMD_ATTN_BWD_DMA");
  const bool dma = !leg && !(ed && ed[0] == '0');
  if (split && dma)
    bwd_dkdv5_kernel<2, false, true><<<grid, 512, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2,
                                                           scale, causal, dst, lp, rcos, rsin);
  else if (split && leg)
    bwd_dkdv5_kernel<2, true><<<grid, 512, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale,
                                                    causal, dst, lp, rcos, rsin);
  else if (split)
    bwd_dkdv5_kernel<2><<<grid, 512, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
                                              dst, lp, rcos, rsin);
  else
    bwd_dkdv5_kernel<1><<<grid, 256, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
                                              dst, lp, rcos, rsin);
}

}  // namespace attn

// SFTAMD_ATTN_GQA=0: per-query-head dK/dV + fp32 partials + dkdv_reduce (v4) instead of the GQA-grouped v5 kernel
static bool attn_gqa_grouped() {
  const char* e = std::getenv("SFTAMD_ATTN_GQA");
  return !(e && e[0] == '0');
}

static void check_attn_args(const at::Tensor& qkv, const at::Tensor& cu, int64_t nq, int64_t nkv, int64_t hd) {
  SFT_CHECK_CUDA(qkv);
  SFT_CHECK_BF16(qkv);
  SFT_CHECK_CONTIG(qkv);
  SFT_CHECK(hd == attn::D, "flash attention kernel is built for head_dim 128, got ", hd);
  SFT_CHECK(nq % nkv == 0, "nq must be a multiple of nkv");
  SFT_CHECK(qkv.dim() == 2 && qkv.size(1) == (nq + 2 * nkv) * hd, "qkv must be [M, (nq+2nkv)*hd]");
  SFT_CHECK(cu.scalar_type() == at::kInt && cu.is_cuda() && cu.dim() == 1 && cu.numel() >= 2, "cu_seqlens int32");
}

// variant: 1 = ds_read_b64_tr_b16 transposed operand reads (default), 0 = scalar LDS gathers
// implementation: 2 = double-buffered v2 kernels (default), 1 = v1 (single-buffered)
// SFTAMD_ATTN_CONC=1: dq and dK/dV backward kernels concurrently on two HIP streams (they write disjoint
// column ranges of dqkv). Measured neutral at the SmolLM3 shape (bwd 266.5 vs 262.5 us serial, end to end
// within noise: profiles/r1_attention_microbench.txt), so serial is the default.
static bool attn_concurrent_bwd() {
  const char* e = std::getenv("SFTAMD_ATTN_CONC");
  return e && e[0] == '1';
}

static long attn_ds_budget() {  // read per call (cheap next to the kernels): tests switch paths in-process
  const char* e = std::getenv("SFTAMD_ATTN_DS_MB");
  return (e && e[0] ? atol(e) : 2048L) * 1024L * 1024L;
}

// SFTAMD_ATTN_DQ6=1: backward v6 (dK/dV without dS^T stores + the recomputing GQA-stacked dQ kernel)
static bool attn_dq6() {
  const char* e = std::getenv("SFTAMD_ATTN_DQ6");
  return e && e[0] == '1';
}

// SFTAMD_ATTN_FWD6=1: the GQA-stacked v6 forward where it applies (2 or 4 query heads per kv head)
static bool attn_fwd6() {
  const char* e = std::getenv("SFTAMD_ATTN_FWD6");
  return e && e[0] == '1';
}

// SFTAMD_ATTN_FWD7=1: the 4-wave, two-row-group LDS-DMA forward (fwd7_kernel)
static bool attn_fwd7() {
  const char* e = std::getenv("SFTAMD_ATTN_FWD7");
  return e && e[0] == '1';
}

// fwd3 with K / V staged by LDS-DMA into two stages, one barrier per tile (default; SFTAMD_ATTN_FWD_DMA=0: register
// staging). B16 x T512: 46.0 vs 51.8 us, ragged 16 x ~640: 65.0 vs 71.8 us (profiles/r3_attention.md)
static bool attn_fwd_dma() {
  const char* e = std::getenv("SFTAMD_ATTN_FWD_DMA");
  return !(e && e[0] == '0');
}

static int attn_impl() {
  const char* e = std::getenv("SFTAMD_ATTN_IMPL");
  if (e && e[0] == '6') return 6;
  if (e && e[0] == '1') return 1;
  if (e && e[0] == '2') return 2;
  if (e && e[0] == '4') return 4;  // forward v4 (measured slower, kept selectable: profiles/r1_attention_microbench.txt)
  return 3;
}

// launch geometry for the v2 kernels: SFTAMD_ATTN_CFG="<waves fwd/dq: 4|8>,<LDS buffers: 1|2>"
static void attn_cfg(int& nw, int& nbuf) {
  nw = 8;
  nbuf = 2;
  const char* e = std::getenv("SFTAMD_ATTN_CFG");
  if (e && e[0]) {
    nw = (e[0] == '4') ? 4 : 8;
    const char* c = std::strchr(e, ',');
    if (c && c[1] == '1') nbuf = 1;
  }
}

static int attn_variant() {
  const char* e = std::getenv("SFTAMD_ATTN_TR");
  return (e && e[0] == '0') ? 0 : 1;
}

std::tuple<at::Tensor, at::Tensor> flash_fwd(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_seqlen,
                                             int64_t nq, int64_t nkv, int64_t hd, double scale, bool causal) {
  check_attn_args(qkv, cu, nq, nkv, hd);
  const int total = qkv.size(0);
  const int nseq = cu.numel() - 1;
  auto out = at::empty({total, nq * hd}, qkv.options());
  auto lse = at::empty({nq, total}, qkv.options().dtype(at::kFloat));
  if (total == 0 || max_seqlen == 0) return {out, lse};
  dim3 grid((max_seqlen + 63) / 64, nq, nseq);
  const float sl2 = (float)scale * attn::LOG2E;
  auto cu_c = cu.contiguous();
  if (attn_impl() == 4) {  // forward v4 (2 row groups per wave); backward stays on v3
    constexpr int NW = 4, RG = 2;
    dim3 g4((max_seqlen + NW * 16 * RG - 1) / (NW * 16 * RG), nq, nseq);
    attn::fwd4_kernel<NW, RG><<<g4, NW * 64, 0, cur_stream()>>>((const u16*)qkv.data_ptr(), (u16*)out.data_ptr(),
                                                               lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv,
                                                               total, sl2, causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
    return {out, lse};
  }
  const int rep = (int)(nq / nkv);
  if (attn_impl() == 6 || (attn_impl() == 3 && attn_fwd6() && (rep == 2 || rep == 4))) {
    SFT_CHECK(rep == 2 || rep == 4, "attention forward v6: 2 or 4 query heads per kv head");
    SFT_TRACE("attn.fwd6");
    dim3 g6(nkv, nseq, (max_seqlen + 63) / 64);
    auto go6 = [&](auto r) {
      attn::fwd6_kernel<decltype(r)::value><<<g6, 256, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (u16*)out.data_ptr(), lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv, total,
          sl2, causal ? 1 : 0);
    };
    if (rep == 4) go6(std::integral_constant<int, 4>()); else go6(std::integral_constant<int, 2>());
    SFT_LAUNCH_CHECK();
    return {out, lse};
  }
  if (attn_impl() == 3 && std::getenv("SFTAMD_ATTN_DIAG")) {  // timing-only ablations of fwd v3 (8 waves)
    const int diag = atoi(std::getenv("SFTAMD_ATTN_DIAG"));
    dim3 g3(nq, nseq, (max_seqlen + 127) / 128);
    auto gd = [&](auto dg) {
      attn::fwd3_kernel<8, decltype(dg)::value><<<g3, 512, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (u16*)out.data_ptr(), lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv, total,
          sl2, causal ? 1 : 0);
    };
    switch (diag) {
      case 1: gd(std::integral_constant<int, 1>()); break;
      case 2: gd(std::integral_constant<int, 2>()); break;
      case 4: gd(std::integral_constant<int, 4>()); break;
      case 8: gd(std::integral_constant<int, 8>()); break;
      case 12: gd(std::integral_constant<int, 12>()); break;
      case 15: gd(std::integral_constant<int, 15>()); break;
      default: gd(std::integral_constant<int, 0>()); break;
    }
    SFT_LAUNCH_CHECK();
    return {out, lse};
  }
  if (attn_impl() == 3 && attn_fwd7() && !attn::attn_legacy_wait()) {
    SFT_TRACE("attn.fwd7");
    dim3 g7(nq, nseq, (max_seqlen + 127) / 128);
    attn::fwd7_kernel<<<g7, 256, 0, cur_stream()>>>((const u16*)qkv.data_ptr(), (u16*)out.data_ptr(),
                                                    lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv, total, sl2,
                                                    causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
    return {out, lse};
  }
  if (attn_impl() == 3) {
    int nw, nbuf;
    attn_cfg(nw, nbuf);
    SFT_TRACE(nw == 8 ? "attn.fwd3" : "attn.fwd3.w4");
    auto go3 = [&](auto w) {
      constexpr int NW = decltype(w)::value;
      dim3 g3(nq, nseq, (max_seqlen + NW * 16 - 1) / (NW * 16));
      const char* e3 = std::getenv("SFTAMD_ATTN_FWD_DMA3");
      if (NW == 8 && e3 && e3[0] == '1' && !attn::attn_legacy_wait())
        attn::fwd3_kernel<8, 64><<<g3, 512, 0, cur_stream()>>>(
            (const u16*)qkv.data_ptr(), (u16*)out.data_ptr(), lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv,
            total, sl2, causal ? 1 : 0);
      else if (NW == 8 && attn_fwd_dma() && !attn::attn_legacy_wait())
        attn::fwd3_kernel<8, 32><<<g3, 512, 0, cur_stream()>>>(
            (const u16*)qkv.data_ptr(), (u16*)out.data_ptr(), lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv,
            total, sl2, causal ? 1 : 0);
      else if (NW == 8 && attn::attn_legacy_wait())
        attn::fwd3_kernel<NW, 16><<<g3, NW * 64, 0, cur_stream()>>>(
            (const u16*)qkv.data_ptr(), (u16*)out.data_ptr(), lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv,
            total, sl2, causal ? 1 : 0);
      else
        attn::fwd3_kernel<NW><<<g3, NW * 64, 0, cur_stream()>>>((const u16*)qkv.data_ptr(), (u16*)out.data_ptr(),
                                                               lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv,
                                                               total, sl2, causal ? 1 : 0);
    };
    if (nw == 4) go3(std::integral_constant<int, 4>()); else go3(std::integral_constant<int, 8>());
    SFT_LAUNCH_CHECK();
    return {out, lse};
  }
  if (attn_impl() == 2) {
    int nw, nbuf;
    attn_cfg(nw, nbuf);
    auto go = [&](auto tr, auto w, auto b) {
      constexpr bool TR = decltype(tr)::value;
      constexpr int NW = decltype(w)::value, NB = decltype(b)::value;
      dim3 g2((max_seqlen + NW * 16 - 1) / (NW * 16), nq, nseq);
      attn::fwd2_kernel<TR, NW, NB><<<g2, NW * 64, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (u16*)out.data_ptr(), lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv,
          total, sl2, causal ? 1 : 0);
    };
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using B1 = std::integral_constant<int, 1>;
    using B2 = std::integral_constant<int, 2>;
    if (!attn_variant()) go(std::false_type(), I8(), B2());
    else if (nw == 8 && nbuf == 2) go(std::true_type(), I8(), B2());
    else if (nw == 8) go(std::true_type(), I8(), B1());
    else if (nbuf == 2) go(std::true_type(), I4(), B2());
    else go(std::true_type(), I4(), B1());
    SFT_LAUNCH_CHECK();
    return {out, lse};
  }
  if (attn_variant())
    attn::fwd_kernel<true><<<grid, 256, 0, cur_stream()>>>((const u16*)qkv.data_ptr(), (u16*)out.data_ptr(),
                                                           lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv, total,
                                                           sl2, causal ? 1 : 0);
  else
    attn::fwd_kernel<false><<<grid, 256, 0, cur_stream()>>>((const u16*)qkv.data_ptr(), (u16*)out.data_ptr(),
                                                            lse.data_ptr<float>(), cu_c.data_ptr<int>(), nq, nkv, total,
                                                            sl2, causal ? 1 : 0);
  SFT_LAUNCH_CHECK();
  return {out, lse};
}

// rcos / rsin (optional, [total, hd / 2] fp32): apply the inverse rotate_half RoPE to the dq and dk heads in the
// epilogues (v4 dq path + GQA-grouped dK/dV); sets rope_done. Other paths leave it to the caller.
static at::Tensor flash_bwd_impl(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out,
                                 const at::Tensor& lse, const at::Tensor& cu, int64_t max_seqlen, int64_t nq,
                                 int64_t nkv, int64_t hd, double scale, bool causal, const float* rcos,
                                 const float* rsin, bool& rope_done) {
  rope_done = false;
  check_attn_args(qkv, cu, nq, nkv, hd);
  SFT_CHECK_CONTIG(dout);
  SFT_CHECK_CONTIG(out);
  SFT_CHECK(dout.sizes() == out.sizes() && out.size(1) == nq * hd, "dout/out shape");
  const int total = qkv.size(0);
  const int nseq = cu.numel() - 1;
  auto dqkv = at::empty_like(qkv);
  if (total == 0 || max_seqlen == 0) return dqkv;
  auto delta = at::empty({nq, total}, qkv.options().dtype(at::kFloat));
  const long rows = (long)total * nq;
  attn::delta_kernel<<<(rows + 15) / 16, 256, 0, cur_stream()>>>((const u16*)dout.data_ptr(), (const u16*)out.data_ptr(),
                                                                  delta.data_ptr<float>(), total, nq);
  SFT_LAUNCH_CHECK();
  const float sl2 = (float)scale * attn::LOG2E;
  auto cu_c = cu.contiguous();
  dim3 gk((max_seqlen + 63) / 64, nkv, nseq);
  dim3 gq((max_seqlen + 63) / 64, nq, nseq);
  auto run = [&](auto tr) {
    constexpr bool TR = decltype(tr)::value;
    attn::bwd_dkdv_kernel<TR><<<gk, 256, 0, cur_stream()>>>(
        (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
        cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, sl2, (float)scale, causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
    attn::bwd_dq_kernel<TR><<<gq, 256, 0, cur_stream()>>>(
        (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
        cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, sl2, (float)scale, causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
  };
  int nw, nbuf;
  attn_cfg(nw, nbuf);
  auto run2 = [&](auto tr, auto w, auto bb) {
    constexpr bool TR = decltype(tr)::value;
    constexpr int NW = decltype(w)::value, NB = decltype(bb)::value;
    const int rep = nq / nkv;
    at::Tensor part;
    if (rep > 1) part = at::empty({(long)rep * total * 2 * nkv * hd}, qkv.options().dtype(at::kFloat));
    dim3 gk2((max_seqlen + 63) / 64, nq, nseq);
    attn::bwd_dkdv2_kernel<TR, NB><<<gk2, 256, 0, cur_stream()>>>(
        (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
        cu_c.data_ptr<int>(), rep > 1 ? part.data_ptr<float>() : nullptr, (u16*)dqkv.data_ptr(), nq, nkv, total, sl2,
        (float)scale, causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
    if (rep > 1) {
      const long nvec = (long)total * 2 * nkv * hd / 8;
      const int grid = (int)std::min<long>((nvec + 255) / 256, 2048);
      attn::dkdv_reduce_kernel<<<grid, 256, 0, cur_stream()>>>(part.data_ptr<float>(), (u16*)dqkv.data_ptr(), total,
                                                               nq, nkv, rep, (float)scale);
      SFT_LAUNCH_CHECK();
    }
    dim3 gq2((max_seqlen + NW * 16 - 1) / (NW * 16), nq, nseq);
    attn::bwd_dq2_kernel<TR, NW, NB><<<gq2, NW * 64, 0, cur_stream()>>>(
        (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
        cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, sl2, (float)scale, causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
  };
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  using B1 = std::integral_constant<int, 1>;
  using B2 = std::integral_constant<int, 2>;
  // side stream for the dq kernel: forked after the delta kernel, joined before returning
  hipStream_t dq_stream = cur_stream();
  static thread_local hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  c10::optional<c10::hip::HIPStream> side;
  if (attn_impl() >= 3 && attn_concurrent_bwd()) {
    if (!ev_fork) {
      C10_HIP_CHECK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
      C10_HIP_CHECK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    }
    side = c10::hip::getStreamFromPool(false, qkv.device().index());
    dq_stream = side->stream();
    C10_HIP_CHECK(hipEventRecord(ev_fork, cur_stream()));
    C10_HIP_CHECK(hipStreamWaitEvent(dq_stream, ev_fork, 0));
  }
  // v4 backward: dkdv3 stores dS^T, dQ = one product per tile (bwd_dq4_kernel). Needs the lp x lp bf16 dS^T
  // blocks of every (sequence, head) — 134 MB for 16 x 512 tokens, 16 heads — so it is used when they fit
  // SFTAMD_ATTN_DS_MB (default 2048); otherwise dq3 recomputes S / dP.
  const long lp = (max_seqlen + 127) / 128 * 128;
  const long ds_bytes = (long)nseq * nq * lp * lp * 2;
  const int rep6 = nq / nkv;
  if (attn_impl() >= 3 && !side && attn_dq6() && (rep6 == 2 || rep6 == 4) && attn_gqa_grouped()) {
    // v6 backward: GQA-grouped dK/dV without the dS^T stores + the recomputing GQA-stacked dQ (no HBM round trip)
    const bool rope = rcos != nullptr;
    SFT_TRACE("attn.dkdv5");
    SFT_TRACE("attn.dq6");
    if (rope) SFT_TRACE("attn.bwd_rope_epi");
    attn::launch_dkdv5((const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(),
                       delta.data_ptr<float>(), cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, nseq,
                       max_seqlen, sl2, (float)scale, causal ? 1 : 0, nullptr, 0, cur_stream(), rcos, rsin);
    SFT_LAUNCH_CHECK();
    dim3 g6(nkv, nseq, (max_seqlen + 63) / 64);
    auto go6 = [&](auto r) {
      attn::dq6_kernel<decltype(r)::value><<<g6, 256, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
          cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, sl2, (float)scale, causal ? 1 : 0, rcos, rsin);
    };
    if (rep6 == 4) go6(std::integral_constant<int, 4>()); else go6(std::integral_constant<int, 2>());
    SFT_LAUNCH_CHECK();
    rope_done = rope;
    return dqkv;
  }
  if (attn_impl() >= 3 && !side && ds_bytes <= attn_ds_budget() && hd == 128) {
    const int rep = nq / nkv;
    auto dst = at::empty({ds_bytes / 2}, qkv.options());
    const bool grouped = rep > 1 && attn_gqa_grouped();
    const bool rope = grouped && rcos != nullptr;
    at::Tensor part;
    SFT_TRACE(grouped ? "attn.dkdv5" : "attn.dkdv3");
    SFT_TRACE("attn.dq4");
    if (rope) SFT_TRACE("attn.bwd_rope_epi");
    if (grouped) {
      attn::launch_dkdv5((const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(),
                         delta.data_ptr<float>(), cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, nseq,
                         max_seqlen, sl2, (float)scale, causal ? 1 : 0, (u16*)dst.data_ptr(), (int)lp, cur_stream(),
                         rope ? rcos : nullptr, rope ? rsin : nullptr);
      SFT_LAUNCH_CHECK();
    } else {
      if (rep > 1) part = at::empty({(long)rep * total * 2 * nkv * hd}, qkv.options().dtype(at::kFloat));
      dim3 gk3(nq, nseq, (max_seqlen + 63) / 64);
      attn::bwd_dkdv3_kernel<<<gk3, 256, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
          cu_c.data_ptr<int>(), rep > 1 ? part.data_ptr<float>() : nullptr, (u16*)dqkv.data_ptr(), nq, nkv, total, sl2,
          (float)scale, causal ? 1 : 0, (u16*)dst.data_ptr(), (int)lp);
      SFT_LAUNCH_CHECK();
    }
    if (rep > 1 && !grouped) {
      const long nvec = (long)total * 2 * nkv * hd / 8;
      const int grid = (int)std::min<long>((nvec + 255) / 256, 2048);
      attn::dkdv_reduce_kernel<<<grid, 256, 0, cur_stream()>>>(part.data_ptr<float>(), (u16*)dqkv.data_ptr(), total,
                                                               nq, nkv, rep, (float)scale);
      SFT_LAUNCH_CHECK();
    }
    dim3 gq4(nq, nseq, (max_seqlen + 127) / 128);
    // SFTAMD_ATTN_DQ_DMA=1: K / dS^T by LDS-DMA (measured neutral: 130.2 vs 129.9 us bwd at B16 x T512, r3_run40;
    // this kernel streams dS^T at ~60 % of HBM bandwidth, the staging is not its limit)
    const char* edq = std::getenv("SFTAMD_ATTN_DQ_DMA");
    if (!attn::attn_legacy_wait() && edq && edq[0] == '1')
      attn::bwd_dq4_kernel<8, false, true><<<gq4, 512, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (const u16*)dst.data_ptr(), cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv,
          (int)lp, (float)scale, causal ? 1 : 0, rope ? rcos : nullptr, rope ? rsin : nullptr);
    else if (attn::attn_legacy_wait())
      attn::bwd_dq4_kernel<8, true><<<gq4, 512, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (const u16*)dst.data_ptr(), cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv,
          (int)lp, (float)scale, causal ? 1 : 0, rope ? rcos : nullptr, rope ? rsin : nullptr);
    else
      attn::bwd_dq4_kernel<8><<<gq4, 512, 0, cur_stream()>>>((const u16*)qkv.data_ptr(), (const u16*)dst.data_ptr(),
                                                             cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv,
                                                             (int)lp, (float)scale, causal ? 1 : 0,
                                                             rope ? rcos : nullptr, rope ? rsin : nullptr);
    SFT_LAUNCH_CHECK();
    rope_done = rope;
    return dqkv;
  }
  auto run3 = [&](auto w) {
    constexpr int NW = decltype(w)::value;
    const int rep = nq / nkv;
    SFT_TRACE("attn.dq3");
    // dq first: on the side stream it starts filling the GPU while dK/dV is enqueued
    dim3 gq3(nq, nseq, (max_seqlen + NW * 16 - 1) / (NW * 16));
    attn::bwd_dq3_kernel<NW><<<gq3, NW * 64, 0, dq_stream>>>(
        (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
        cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, sl2, (float)scale, causal ? 1 : 0);
    SFT_LAUNCH_CHECK();
    const bool grouped = rep > 1 && attn_gqa_grouped();
    at::Tensor part;
    if (grouped) {
      attn::launch_dkdv5((const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(),
                         delta.data_ptr<float>(), cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total, nseq,
                         max_seqlen, sl2, (float)scale, causal ? 1 : 0, nullptr, 0, cur_stream());
      SFT_LAUNCH_CHECK();
    } else {
      if (rep > 1) part = at::empty({(long)rep * total * 2 * nkv * hd}, qkv.options().dtype(at::kFloat));
      dim3 gk3(nq, nseq, (max_seqlen + 63) / 64);
      attn::bwd_dkdv3_kernel<<<gk3, 256, 0, cur_stream()>>>(
          (const u16*)qkv.data_ptr(), (const u16*)dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
          cu_c.data_ptr<int>(), rep > 1 ? part.data_ptr<float>() : nullptr, (u16*)dqkv.data_ptr(), nq, nkv, total, sl2,
          (float)scale, causal ? 1 : 0);
      SFT_LAUNCH_CHECK();
    }
    if (rep > 1 && !grouped) {
      const long nvec = (long)total * 2 * nkv * hd / 8;
      const int grid = (int)std::min<long>((nvec + 255) / 256, 2048);
      attn::dkdv_reduce_kernel<<<grid, 256, 0, cur_stream()>>>(part.data_ptr<float>(), (u16*)dqkv.data_ptr(), total,
                                                               nq, nkv, rep, (float)scale);
      SFT_LAUNCH_CHECK();
    }
  };
  if (attn_impl() >= 3) {
    if (nw == 4) run3(I4()); else run3(I8());
    if (side) {  // join: everything after this op on the current stream sees dq
      C10_HIP_CHECK(hipEventRecord(ev_join, dq_stream));
      C10_HIP_CHECK(hipStreamWaitEvent(cur_stream(), ev_join, 0));
    }
  } else if (attn_impl() == 2) {
    if (!attn_variant()) run2(std::false_type(), I8(), B2());
    else if (nw == 8 && nbuf == 2) run2(std::true_type(), I8(), B2());
    else if (nw == 8) run2(std::true_type(), I8(), B1());
    else if (nbuf == 2) run2(std::true_type(), I4(), B2());
    else run2(std::true_type(), I4(), B1());
  } else if (attn_variant()) {
    run(std::true_type());
  } else {
    run(std::false_type());
  }
  return dqkv;
}

at::Tensor flash_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& lse,
                     const at::Tensor& cu, int64_t max_seqlen, int64_t nq, int64_t nkv, int64_t hd, double scale,
                     bool causal) {
  bool rope_done;
  return flash_bwd_impl(dout, qkv, out, lse, cu, max_seqlen, nq, nkv, hd, scale, causal, nullptr, nullptr, rope_done);
}

void rope_(at::Tensor qkv, const at::Tensor& cos, const at::Tensor& sin, int64_t n_q, int64_t n_kv, int64_t head_dim,
           bool inverse);  // elementwise.hip

// flash_bwd for a qkv whose q / k heads were rotated (RoPE) by the producing GEMM: returns the gradient w.r.t. the
// UNROTATED qkv. The inverse rotation rides in the dq / dK epilogues on the default path; otherwise the rope kernel
// runs after the backward.
at::Tensor flash_bwd_rope(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& lse,
                          const at::Tensor& cu, int64_t max_seqlen, int64_t nq, int64_t nkv, int64_t hd, double scale,
                          bool causal, const at::Tensor& cos, const at::Tensor& sin) {
  SFT_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                sin.is_contiguous() && cos.is_cuda() && sin.is_cuda(),
            "flash_bwd_rope: contiguous fp32 cos / sin");
  SFT_CHECK(cos.numel() == qkv.size(0) * hd / 2 && sin.numel() == cos.numel(), "flash_bwd_rope: cos / sin [total, hd/2]");
  bool rope_done;
  auto dqkv = flash_bwd_impl(dout, qkv, out, lse, cu, max_seqlen, nq, nkv, hd, scale, causal, cos.data_ptr<float>(),
                             sin.data_ptr<float>(), rope_done);
  if (!rope_done) rope_(dqkv, cos, sin, nq, nkv, hd, true);
  return dqkv;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("flash_fwd", &flash_fwd);
  m.impl("flash_bwd", &flash_bwd);
  m.impl("flash_bwd_rope", &flash_bwd_rope);
}

}  // namespace sftamd
