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

// Buffer-descriptor forms (the 32x32 kernels): the tile's base and byte range in a wave-uniform descriptor, the lane's
// row / chunk in a loop-invariant VGPR offset, the tile's row offset in an SGPR. Rows past the sequence end fall
// outside the range and read as ZERO (no clamps, no per-row branches, no 64-bit VALU address math per piece).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const unsigned n = __builtin_amdgcn_readfirstlane((unsigned)(bytes < 0 ? 0 : bytes));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, n, 0x00020000);
}
__device__ __forceinline__ void bdma16(rsrc_t r, char* dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ bf16x8 bload16(rsrc_t r, unsigned voff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return __builtin_bit_cast(bf16x8, v);
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

// ============================================================================== fwd32: 32x32x16 forward
// v_mfma_f32_32x32x16_bf16 lane maps (hi = lane >> 5, c = lane & 31, j = 0..7, i = 0..15):
//   A[row c][k 8hi+j], B[k 8hi+j][col c], C[row crow(i, hi)][col c], crow(i, hi) = (i & 3) + 8 (i >> 2) + 4 hi.
// S^T = K Q^T with the query on the lane: lane (hi, c) holds 16 keys of each 32-key block for query c, so the row max
// and sum are lane-local plus ONE permlane32 swap, and the accumulator registers 8 sub .. 8 sub + 7 of block kb are
// already the B operand (P^T) of k-step 2 kb + sub of O^T += V^T P^T: they hold keys 16 ks + 4 hi + {0..3} and
// 16 ks + 8 + 4 hi + {0..3}, so the V^T A operand is read with that key order (two ds_read_b64_tr_b16, rows
// 16 ks + 4 hi + q and 16 ks + 8 + 4 hi + q). Per 64-key tile and 32 queries: 16 + 16 MFMAs (each 2x the work of a
// 16x16x32), 16 ds_read_b128 + 32 ds_read_b64_tr_b16 — half fwd3's LDS bytes per FLOP.
// A workgroup = 4 waves = HW query heads of one kv head x (4 / HW) 32-query position blocks (HW = gcd(rep, 4)): at
// GQA rep 4 the four waves share their positions, so the key range, the K / V tiles and the causal work are the same
// for every wave and a 32-key half tile past the diagonal is skipped by all of them.
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

struct Offs32 {
  int k[8];  // K row reads (A of S^T), k-step s: image row c, chunk 2 s + hi
  int v[8];  // V^T transposed reads, [2 db + part]: rows 8 part + 4 hi + q, columns 32 db + 16 (a & 1) + 4 p ..
  __device__ __forceinline__ void init(int lane) {
    const int c = lane & 31, hi = lane >> 5, a = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int s = 0; s < 8; ++s) k[s] = img_off(c, 2 * s + hi);
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int part = 0; part < 2; ++part)
        v[2 * db + part] = img_off(8 * part + 4 * hi + q, 4 * db + 2 * (a & 1) + (p >> 1)) + 8 * (p & 1);
  }
};

__device__ __forceinline__ bf16x8 lds_tr2(const char* base, int lo, int hi) {
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + lo));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + hi));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& t, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)t[base + j];
  return r;
}

__device__ __forceinline__ float swap32max(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
__device__ __forceinline__ float swap32sum(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}

// T21 epilogue of a 32x32 accumulator row: lane (hi, c) holds columns 32 db + 8 m + 4 hi + {0..3} (registers
// 4 m .. 4 m + 3 of block db) of row c; one permlane32 swap per dword pair (m = 2u, 2u + 1) gives each half 8
// consecutive columns -> 8 x 16-B stores per lane. row: the row's first column; every lane must call (the swaps).
__device__ __forceinline__ void store_t21(u16* row, const f32x16 (&a)[4], float s, bool ok) {
  const int hi = (threadIdx.x >> 5) & 1;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i0 = 8 * u;
      const unsigned ax = (unsigned)f2bf(a[db][i0] * s) | ((unsigned)f2bf(a[db][i0 + 1] * s) << 16);
      const unsigned ay = (unsigned)f2bf(a[db][i0 + 2] * s) | ((unsigned)f2bf(a[db][i0 + 3] * s) << 16);
      const unsigned bx = (unsigned)f2bf(a[db][i0 + 4] * s) | ((unsigned)f2bf(a[db][i0 + 5] * s) << 16);
      const unsigned by = (unsigned)f2bf(a[db][i0 + 6] * s) | ((unsigned)f2bf(a[db][i0 + 7] * s) << 16);
      const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
      if (ok) *(uint4*)(row + 32 * db + 16 * u + 8 * hi) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
}

// One 64-key tile: issue the next tile's K / V pieces into nxt (4 x 1 KB per image per wave, source-swizzled, rows
// past the sequence end clamped: their keys are masked), then S^T, the online softmax and O^T += V^T P^T from cur.
// lastkey: the wave's last visible key (causal: its last query); rel: this lane's last visible key - k0 - 4 hi.
__device__ __forceinline__ void fwd32_step(const char* __restrict__ cur, char* __restrict__ nxt, bool pre, rsrc_t kv,
                                           unsigned voffk, unsigned voffv, unsigned rowb, int wave, int k0, int lastkey,
                                           bool need_mask, int rel, float sl2, const Offs32& off,
                                           const bf16x8 (&qf)[8], f32x16 (&o)[4], float& m, float& l) {
  constexpr int TB = 64 * ROWB;
  if (pre) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned so = (unsigned)(k0 + 64 + 16 * j) * rowb;
      bdma16(kv, nxt + (wave + 4 * j) * 1024, voffk, so);
      bdma16(kv, nxt + TB + (wave + 4 * j) * 1024, voffv, so);
    }
  }
  if (k0 > lastkey) return;
  const bool two = k0 + 32 <= lastkey;  // wave-uniform: the second 32-key half has a visible key
  const char* Ks = cur;
  const char* Vs = cur + TB;
  f32x16 s[2];
  s[0] = mfma32(lds_row(Ks, off.k[0]), qf[0], f32x16{});
#pragma unroll
  for (int st = 1; st < 8; ++st) s[0] = mfma32(lds_row(Ks, off.k[st]), qf[st], s[0]);
  if (two) {  // (each path writes s[1] itself: a zero-filled s[1] before the branch costs 48 moves per tile)
    s[1] = mfma32(lds_row(Ks, off.k[0] + 32 * ROWB), qf[0], f32x16{});
#pragma unroll
    for (int st = 1; st < 8; ++st) s[1] = mfma32(lds_row(Ks, off.k[st] + 32 * ROWB), qf[st], s[1]);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[1][i] = -INFINITY;
  }
  if (need_mask) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        s[kb][i] = 32 * kb + (i & 3) + 8 * (i >> 2) > rel ? -INFINITY : s[kb][i];
  }
  float mx = max3f(s[0][0], s[0][1], s[0][2]);
#pragma unroll
  for (int i = 3; i < 15; i += 2) mx = max3f(mx, s[0][i], s[0][i + 1]);
  mx = max3f(mx, s[0][15], s[1][0]);
#pragma unroll
  for (int i = 1; i < 15; i += 2) mx = max3f(mx, s[1][i], s[1][i + 1]);
  mx = fmaxf(mx, s[1][15]);
  const float tmax = swap32max(mx) * sl2;
  if (__any(tmax > m + THR)) {  // deferred rescale (T13): P stays <= 2^THR
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);
    l *= alpha;
#pragma unroll
    for (int db = 0; db < 4; ++db) o[db] *= alpha;
    m = mnew;
  }
  float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const float p0 = exp2f(__builtin_fmaf(s[kb][i], sl2, -m));
      const float p1 = exp2f(__builtin_fmaf(s[kb][i + 1], sl2, -m));
      s[kb][i] = p0;
      s[kb][i + 1] = p1;
      acc0 += p0;
      acc1 += p1;
    }
  l += acc0 + acc1;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if (ks >= 2 && !two) break;
    const bf16x8 pb = pack8(s[ks >> 1], 8 * (ks & 1));
#pragma unroll
    for (int db = 0; db < 4; ++db)
      o[db] = mfma32(lds_tr2(Vs, off.v[2 * db] + 16 * ks * ROWB, off.v[2 * db + 1] + 16 * ks * ROWB), pb, o[db]);
  }
}

// grid (nq / HW, sequences, position blocks of 32 (4 / HW)) with the last (causally heaviest) block first; 256 threads
template <int HW>
__global__ __launch_bounds__(256, 2) void fwd32_kernel(const u16* __restrict__ qkv, u16* __restrict__ out,
                                                       float* __restrict__ lse, const int* __restrict__ cu, int nq,
                                                       int nkv, int total, float sl2, int causal) {
  constexpr int PB = 4 / HW, TB = 64 * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];
  const int b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int q0 = qb * 32 * PB;
  if (q0 >= len) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), hi = lane >> 5;
  const int h = blockIdx.x * HW + wave % HW;
  const int kvh = (blockIdx.x * HW) / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int wq0 = q0 + 32 * (wave / HW);
  const int qi = wq0 + (lane & 31);
  const bool qok = qi < len;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((min(q0 + 32 * PB, len) - 1) / 64 + 1, nkb) : nkb;
  const int lastkey = causal ? min(wq0 + 31, len - 1) : len - 1;
  const int lim = causal ? min(len - 1, qi) : len - 1;
  Offs32 off;
  off.init(lane);
  const unsigned rowb = (unsigned)ld * 2;
  bf16x8 qf[8];
  {  // Q rows past the sequence end read as zero (outside the descriptor's range)
    const rsrc_t qr = make_rsrc(qkv + (long)start * ld + h * D, (long)(len - 1) * ld * 2 + ROWB);
    const unsigned vo = (unsigned)qi * rowb + 16 * hi;
#pragma unroll
    for (int st = 0; st < 8; ++st) qf[st] = bload16(qr, vo + 32 * st);
  }
  // K and V of rows [0, len) of this kv head in one descriptor (V = K + nkv * D); DMA lane (wave w, l) fills LDS
  // rows 4 (w + 4 j) + (l >> 4), position l & 15, with the chunk swz(row, l & 15)
  const rsrc_t kv = make_rsrc(qkv + (long)start * ld + (nq + kvh) * D, (long)len * ld * 2 - (long)(nq + kvh) * ROWB);
  const int r0 = 4 * wave + (lane >> 4);
  const unsigned voffk = (unsigned)r0 * rowb + 16 * swz(r0, lane & 15), voffv = voffk + nkv * ROWB;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bdma16(kv, smem + (wave + 4 * j) * 1024, voffk, 16 * j * rowb);
    bdma16(kv, smem + TB + (wave + 4 * j) * 1024, voffv, 16 * j * rowb);
  }
  vm_drain();
  f32x16 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[db][i] = 0.f;
  float m = -1e30f, l = 0.f;  // l: this lane's partial row sum (its 16 keys of each 32-key block)
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const bool pre = kt + 1 < nkt;
    const bool need_mask = (k0 + 64 > len) || (causal && k0 + 63 > wq0);
    fwd32_step(smem + (kt & 1) * 2 * TB, smem + ((kt + 1) & 1) * 2 * TB, pre, kv, voffk, voffv, rowb, wave, k0,
               lastkey, need_mask, lim - k0 - 4 * hi, sl2, off, qf, o, m, l);
    if (pre) vm_drain();
    __syncthreads();
  }
  l = swap32sum(l);
  const float inv = 1.f / l;
  store_t21(out + (long)(start + qi) * nq * D + h * D, o, inv, qok);
  if (qok && hi == 0) lse[(long)h * total + start + qi] = (m + log2f(l)) * LN2;
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
// ============================================================================== dQ with 32x32x16 MFMAs
// dQ^T = K^T dS^T over the key tiles of the materialised dS^T (written by bwd_dkdv32): the query on the lane, so the
// accumulator is the forward's O^T layout (T21 stores). A workgroup = 4 waves = HW query heads of one kv head x
// (4 / HW) 32-query position blocks (as fwd32): the K tile is shared, each wave stages its own [64 keys][32 queries]
// dS^T block (64-B rows: a transposed read's four rows x 64 B of a 32-lane half cover the 64 banks once, no swizzle).
// Rows past the sequence end read as zero (the dS^T rows there were never written; buffer-descriptor range). Per tile and wave: 16 MFMAs,
// 32 + 8 ds_read_b64_tr_b16.
__device__ __forceinline__ void rope_bwd32(f32x16 (&a)[4], const float* cs, const float* sn, float s) {
  const int hi = (threadIdx.x >> 5) & 1;
#pragma unroll
  for (int d4 = 0; d4 < 2; ++d4)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int d = 32 * d4 + 8 * m + 4 * hi;
      const float4 c4 = *(const float4*)(cs + d), s4 = *(const float4*)(sn + d);
      const float c[4] = {c4.x, c4.y, c4.z, c4.w}, n[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = 4 * m + t;
        const float x = a[d4][i] * s, y = a[d4 + 2][i] * s;
        a[d4][i] = x * c[t] + y * n[t];
        a[d4 + 2][i] = y * c[t] - x * n[t];
      }
    }
}

__device__ __forceinline__ void dq32_step(const char* __restrict__ cur, char* __restrict__ nxt, bool pre, bool active,
                                          rsrc_t kr, rsrc_t sr, unsigned voffk, unsigned voffs, unsigned rowb,
                                          unsigned rows, int k0n, int wave, const Offs32& off, int sofs,
                                          f32x16 (&dq)[4]) {
  constexpr int TB = 64 * ROWB, SB = 64 * 64;  // K image, per-wave dS^T block
  if (pre) {  // the next tile (keys k0n ..): K pieces wave + 4 j, this wave's dS^T pieces j (rows 16 j + lane / 4);
              // rows past the sequence end read as zero (outside the descriptors' ranges)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bdma16(kr, nxt + (wave + 4 * j) * 1024, voffk, (unsigned)(k0n + 16 * j) * rowb);
      bdma16(sr, nxt + TB + wave * SB + j * 1024, voffs, (unsigned)(k0n + 16 * j) * rows);
    }
  }
  if (!active) return;
  const char* Ks = cur;
  const char* Ss = cur + TB + wave * SB;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8 sb = lds_tr2(Ss, sofs + ks * 16 * 64, sofs + ks * 16 * 64 + 8 * 64);
#pragma unroll
    for (int d4 = 0; d4 < 4; ++d4)
      dq[d4] = mfma32(lds_tr2(Ks, off.v[2 * d4] + ks * 16 * ROWB, off.v[2 * d4 + 1] + ks * 16 * ROWB), sb, dq[d4]);
  }
}

template <int HW>
__global__ __launch_bounds__(256, 2) void bwd_dq32_kernel(const u16* __restrict__ qkv, const u16* __restrict__ dst,
                                                          const int* __restrict__ cu, u16* __restrict__ dqkv, int nq,
                                                          int nkv, int lp, float scale, int causal,
                                                          const float* __restrict__ rcos,
                                                          const float* __restrict__ rsin) {
  constexpr int PB = 4 / HW, TB = 64 * ROWB, SB = 64 * 64, STG = TB + 4 * SB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int b = blockIdx.y, qb = gridDim.z - 1 - blockIdx.z;
  const int start = cu[b], len = cu[b + 1] - start;
  const int q0 = qb * 32 * PB;
  if (q0 >= len) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), hi = lane >> 5;
  const int h = blockIdx.x * HW + wave % HW;
  const int kvh = (blockIdx.x * HW) / (nq / nkv);
  const long ld = (long)(nq + 2 * nkv) * D;
  const int wq0 = q0 + 32 * (wave / HW);
  const int qi = wq0 + (lane & 31);
  SFT_DASSERT(wq0 + 32 <= lp);
  const int lastq = min(wq0 + 31, len - 1);  // the wave's last query: keys past it are causally invisible
  const u16* kbase = qkv + (long)start * ld + (nq + kvh) * D;
  const u16* sbase = dst + (long)(b * nq + h) * lp * lp + wq0;
  const int nkb = (len + 63) / 64;
  const int nkt = causal ? min((min(q0 + 32 * PB, len) - 1) / 64 + 1, nkb) : nkb;
  Offs32 off;
  off.init(lane);
  // this lane's dS^T transposed read: group a = lane >> 4 reads rows 4 hi + q (+ 8) of a 16-key step, columns
  // 16 (a & 1) + 4 p .. + 3 (64-B rows)
  const int sofs = (4 * hi + ((lane & 15) >> 2)) * 64 + 32 * ((lane >> 4) & 1) + 8 * (lane & 3);
  const int r0 = 4 * wave + (lane >> 4);
  const unsigned rowb = (unsigned)ld * 2, rows = (unsigned)lp * 2;
  const rsrc_t kr = make_rsrc(kbase, (long)(len - 1) * ld * 2 + ROWB);
  const rsrc_t sr = make_rsrc(sbase, (long)(len - 1) * lp * 2 + 64);
  const unsigned voffk = (unsigned)r0 * rowb + 16 * swz(r0, lane & 15);
  const unsigned voffs = (unsigned)(lane >> 2) * rows + 16 * (lane & 3);
  f32x16 dq[4];
#pragma unroll
  for (int d4 = 0; d4 < 4; ++d4)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[d4][i] = 0.f;
  dq32_step(smem + STG, smem, true, false, kr, sr, voffk, voffs, rowb, rows, 0, wave, off, sofs, dq);
  vm_drain();
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    const bool pre = kt + 1 < nkt;
    dq32_step(smem + (kt & 1) * STG, smem + ((kt + 1) & 1) * STG, pre, !causal || k0 <= lastq, kr, sr, voffk, voffs,
              rowb, rows, k0 + 64, wave, off, sofs, dq);
    if (pre) vm_drain();  // this lane's pieces of the next tile landed ...
    __syncthreads();      // ... and every lane's (LDS zero stores too); every wave is done reading this stage
  }
  const bool qok = qi < len;
  float s = scale;
  if (rcos != nullptr && qok) {
    const long tr = (long)(start + qi) * (D / 2);
    rope_bwd32(dq, rcos + tr, rsin + tr, scale);
    s = 1.f;
  }
  store_t21(dqkv + (long)(start + qi) * ld + h * D, dq, s, qok);
}

// ============================================================================== dK / dV with 32x32x16 MFMAs
// S = Q K^T and dP = dO V^T with the KEY on the lane (the K / V fragments are loop-invariant B operands in registers):
// lane (hi, c) holds S[q = crow(i, hi)][key c], so its accumulator registers 8 sub .. 8 sub + 7 are already the B
// operand (k = query) of dV^T += dO^T P and dK^T += Q^T dS, whose A operands are transposed reads of the dO / Q
// images (the forward's V^T read). P = exp2(S sl2 - lse log2 e) needs no row max; lse / delta of the tile's 64 queries
// ride with the Q / dO images. A workgroup = 64 keys of one kv head = 2 key halves x G head groups (G = 2 when rep is
// even; the groups' dK / dV are summed through LDS at the end), 64-query tiles of Q / dO by LDS-DMA in two stages per
// group, one wave per SIMD (dK^T / dV^T: 128 fp32 accumulators per lane). Per tile and wave: 64 MFMAs (32 keys x 64
// queries x 4 products), 32 ds_read_b128 + 64 ds_read_b64_tr_b16 — half dkdv5's LDS bytes per FLOP.
// dS^T ([b][h][key][q], row stride lp) is written for bwd_dq4 when drow is given (T21-paired 16-B stores).
__device__ __forceinline__ void dkdv32_step(const char* __restrict__ cur, char* __restrict__ nxt, bool pre,
                                            rsrc_t qr, rsrc_t orr, unsigned vq0, unsigned vq1, unsigned vo0,
                                            unsigned vo1, unsigned qso, unsigned oso, unsigned rowb, unsigned rowo,
                                            int wv, const float* lsrc, const float* dsrc, int gl, int q0, int len,
                                            int causal, int kw0, int key, float sl2, u16* drow, bool dok,
                                            const Offs32& off, const bf16x8 (&kf)[8], const char* Vk,
                                            f32x16 (&dk)[4], f32x16 (&dv)[4]) {
  constexpr int TB = 64 * ROWB;
  float pl = 0.f, pd = 0.f;
  if (pre) {  // the next tile (rows from qso / oso): image rows 4 (wv + 2 j) + (lane >> 4); rows past the sequence
              // end read as zero (outside the descriptors' ranges)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bdma16(qr, nxt + (wv + 2 * j) * 1024, (j & 1) ? vq1 : vq0, qso + 16 * (j >> 1) * rowb);
      bdma16(orr, nxt + TB + (wv + 2 * j) * 1024, (j & 1) ? vo1 : vo0, oso + 16 * (j >> 1) * rowo);
    }
    if (gl < 64 && lsrc != nullptr) {
      pl = lsrc[gl];
      pd = dsrc[gl];
    }
  }
  const char* Qs = cur;
  const char* Os = cur + TB;
  const float* Ls = (const float*)(cur + 2 * TB);
  const float* Dl = Ls + 64;
  const int hi = (threadIdx.x >> 5) & 1;
#pragma unroll 1
  for (int qb = 0; qb < 2; ++qb) {  // (not unrolled: hoisting the second half's LDS reads ran out of VGPRs)
    f32x16 s, dp;
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = dp[i] = 0.f;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      s = mfma32(lds_row(Qs, off.k[st] + qb * 32 * ROWB), kf[st], s);
      dp = mfma32(lds_row(Os, off.k[st] + qb * 32 * ROWB), lds_row(Vk, off.k[st]), dp);
    }
    // query q = q0 + 32 qb + 4 hi + o, o = 8 m + t for register 4 m + t; visible iff lo <= o <= hq
    const int qbase = q0 + 32 * qb + 4 * hi;
    const int lo = (causal ? key : 0) - qbase, hq = len - 1 - qbase;
    const bool need_mask = (q0 + 32 * qb + 31 >= len) || (causal && kw0 + 31 > q0 + 32 * qb);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 L4 = *(const float4*)(Ls + 32 * qb + 8 * m + 4 * hi);
      const float4 D4 = *(const float4*)(Dl + 32 * qb + 8 * m + 4 * hi);
      const float L[4] = {L4.x, L4.y, L4.z, L4.w}, Dd[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = 4 * m + t, o = 8 * m + t;
        float p = exp2f(__builtin_fmaf(s[i], sl2, -L[t]));
        if (need_mask) p = (o < lo || o > hq) ? 0.f : p;
        dp[i] = p * (dp[i] - Dd[t]);
        s[i] = p;
      }
    }
    if (drow != nullptr) {  // dS^T[key][q]: registers 8 u .. 8 u + 7 = queries 16 u + 4 hi + {0..3, 8..11}
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i0 = 8 * u;
        const unsigned ax = (unsigned)f2bf(dp[i0]) | ((unsigned)f2bf(dp[i0 + 1]) << 16);
        const unsigned ay = (unsigned)f2bf(dp[i0 + 2]) | ((unsigned)f2bf(dp[i0 + 3]) << 16);
        const unsigned bx = (unsigned)f2bf(dp[i0 + 4]) | ((unsigned)f2bf(dp[i0 + 5]) << 16);
        const unsigned by = (unsigned)f2bf(dp[i0 + 6]) | ((unsigned)f2bf(dp[i0 + 7]) << 16);
        const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
        if (dok) *(uint4*)(drow + 32 * qb + 16 * u + 8 * hi) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
      }
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const bf16x8 pb = pack8(s, 8 * sub), db = pack8(dp, 8 * sub);
      const int ko = (2 * qb + sub) * 16 * ROWB;
#pragma unroll
      for (int d4 = 0; d4 < 4; ++d4) {
        dv[d4] = mfma32(lds_tr2(Os, off.v[2 * d4] + ko, off.v[2 * d4 + 1] + ko), pb, dv[d4]);
        dk[d4] = mfma32(lds_tr2(Qs, off.v[2 * d4] + ko, off.v[2 * d4 + 1] + ko), db, dk[d4]);
      }
    }
  }
  if (pre && gl < 64) {  // the next stage's lse / delta (that stage's last reads ended at the previous barrier)
    float* Ln = (float*)(nxt + 2 * TB);
    asm volatile("" : "+v"(pl));  // keeps the multiply (and the loads' wait) after this tile's math
    Ln[gl] = pl * LOG2E;
    Ln[64 + gl] = pd;
  }
}

template <int G>
__global__ __launch_bounds__(128 * G, 1) void bwd_dkdv32_kernel(
    const u16* __restrict__ qkv, const u16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, const int* __restrict__ cu, u16* __restrict__ dqkv, int nq, int nkv, int total,
    float sl2, float scale, int causal, u16* __restrict__ dst, int lp, const float* __restrict__ rcos,
    const float* __restrict__ rsin) {
  constexpr int TB = 64 * ROWB, GB = 2 * TB + 2 * 64 * 4;  // per stage: Q, dO images + lse, delta
  __shared__ __attribute__((aligned(16))) char smem[G * 2 * GB + TB];  // + the workgroup's V image (64 keys)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), grp = w >> 1, kh = w & 1;
  const int gl = tid & 127;
  const int hi = lane >> 5;
  char* base = smem + grp * 2 * GB;
  const int kvh = blockIdx.x, b = blockIdx.y, kb = blockIdx.z;  // z = 0 first: the causally heaviest key blocks
  const int start = cu[b], len = cu[b + 1] - start;
  SFT_DASSERT(start >= 0 && len >= 0 && start + len <= total);
  const int k0 = kb * 64;
  if (k0 >= len) return;
  const int rep = nq / nkv, hpg = rep / G;
  const long ld = (long)(nq + 2 * nkv) * D;
  const long ldo = (long)nq * D;
  const int kw0 = k0 + 32 * kh, key = kw0 + (lane & 31);
  const bool kok = key < len;
  const int qt0 = causal ? kb : 0, nqt = (len + 63) / 64, nt = nqt - qt0, niter = hpg * nt;
  Offs32 off;
  off.init(lane);
  int h = kvh * rep + grp * hpg, qt = qt0;
  // DMA: lane (wave kh, l) fills image rows 4 (kh + 2 j) + (l >> 4), position l & 15, with chunk swz(row, l & 15)
  const int qr0 = 4 * kh + (lane >> 4);
  const unsigned rowb = (unsigned)ld * 2, rowo = (unsigned)ldo * 2;
  // Q rows [0, len) of every head of the sequence (rows past it fall outside the range: zero), dO likewise
  const rsrc_t qr = make_rsrc(qkv + (long)start * ld, (long)(len - 1) * ld * 2 + (long)nq * ROWB);
  const rsrc_t orr = make_rsrc(dout + (long)start * ldo, (long)len * ldo * 2);
  // lane offsets of the even / odd pieces (image rows qr0 + 16 u and qr0 + 8 + 16 u: two swizzles)
  const unsigned sw0 = 16 * swz(qr0, lane & 15), sw1 = 16 * swz(qr0 + 8, lane & 15);
  const unsigned vq0 = (unsigned)qr0 * rowb + sw0, vq1 = (unsigned)(qr0 + 8) * rowb + sw1;
  const unsigned vo0 = (unsigned)qr0 * rowo + sw0, vo1 = (unsigned)(qr0 + 8) * rowo + sw1;
  {
    const int q0 = qt0 * 64, qv = len - q0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // piece j: rows qr0 + 8 j (vq1 / vo1 carry the + 8 of odd j)
      bdma16(qr, base + (kh + 2 * j) * 1024, (j & 1) ? vq1 : vq0, (unsigned)(q0 + 16 * (j >> 1)) * rowb + h * ROWB);
      bdma16(orr, base + TB + (kh + 2 * j) * 1024, (j & 1) ? vo1 : vo0, (unsigned)(q0 + 16 * (j >> 1)) * rowo + h * ROWB);
    }
    if (gl < 64) {
      float* Ls = (float*)(base + 2 * TB);
      Ls[gl] = gl < qv ? lse[(long)h * total + start + q0 + gl] * LOG2E : 0.f;
      Ls[64 + gl] = gl < qv ? delta[(long)h * total + start + q0 + gl] : 0.f;
    }
  }
  // K fragments (B of S = Q K^T) in registers; the V rows (B of dP = dO V^T) read from an LDS image of the
  // workgroup's 64 keys (keeping them in registers too pushed the accumulators through v_accvgpr moves every tile)
  bf16x8 kf[8];
  char* Vk = smem + G * 2 * GB + kh * 32 * ROWB;
  {
    const rsrc_t kr = make_rsrc(qkv + (long)start * ld + (nq + kvh) * D, (long)(len - 1) * ld * 2 + (long)(nkv + 1) * ROWB);
    const unsigned vo = (unsigned)key * rowb + 16 * hi;
#pragma unroll
    for (int st = 0; st < 8; ++st) kf[st] = bload16(kr, vo + 32 * st);
    // V image rows 4 p + (lane >> 4) of piece p = w + 2 G j (keys k0 + row; past the sequence end: zero)
    // (G = 1: pieces w + 2 j, rows vr + 8 j — odd j is 8 rows on, with the swizzle of vr + 8)
    const int vr = 4 * w + (lane >> 4);
    const unsigned vv0 = (unsigned)(k0 + vr) * rowb + nkv * ROWB + 16 * swz(vr, lane & 15);
    const unsigned vv1 = (unsigned)(k0 + vr) * rowb + nkv * ROWB + 16 * swz(vr + 8, lane & 15);
#pragma unroll
    for (int j = 0; j < 8 / G; ++j)
      bdma16(kr, smem + G * 2 * GB + (w + 2 * G * j) * 1024, (G == 1 && (j & 1)) ? vv1 : vv0,
             (unsigned)(8 * G * j) * rowb);
  }
  vm_drain();
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int d4 = 0; d4 < 4; ++d4)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[d4][i] = dv[d4][i] = 0.f;
  __syncthreads();
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
    const bool lok = pre && qn + gl < len;
    u16* drow = dst != nullptr ? dst + ((long)(b * nq + h) * lp + key) * lp + q0 : nullptr;
    dkdv32_step(base + (it & 1) * GB, base + ((it + 1) & 1) * GB, pre, qr, orr, vq0, vq1, vo0, vo1,
                (unsigned)qn * rowb + hn * ROWB, (unsigned)qn * rowo + hn * ROWB, rowb, rowo, kh,
                lok ? lse + lo : nullptr, delta + lo, gl, q0, len, causal, kw0, key, sl2, drow, kok, off, kf, Vk, dk,
                dv);
    if (pre) vm_drain();  // this lane's pieces of the next tile landed ...
    __syncthreads();      // ... and every lane's; every wave is done reading this stage
    h = hn;
    qt = qtn;
  }
  if constexpr (G == 2) {  // group 1 hands its dK / dV partial sums to group 0 through the (now idle) stages
    float4* xk = (float4*)smem;
    float4* xv = xk + 2 * 16 * 64;
    if (grp == 1) {
#pragma unroll
      for (int d4 = 0; d4 < 4; ++d4)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int ix = (kh * 16 + 4 * d4 + v) * 64 + lane;
          xk[ix] = make_float4(dk[d4][4 * v], dk[d4][4 * v + 1], dk[d4][4 * v + 2], dk[d4][4 * v + 3]);
          xv[ix] = make_float4(dv[d4][4 * v], dv[d4][4 * v + 1], dv[d4][4 * v + 2], dv[d4][4 * v + 3]);
        }
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int d4 = 0; d4 < 4; ++d4)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int ix = (kh * 16 + 4 * d4 + v) * 64 + lane;
        const float4 a = xk[ix], c = xv[ix];
        dk[d4][4 * v] += a.x;
        dk[d4][4 * v + 1] += a.y;
        dk[d4][4 * v + 2] += a.z;
        dk[d4][4 * v + 3] += a.w;
        dv[d4][4 * v] += c.x;
        dv[d4][4 * v + 1] += c.y;
        dv[d4][4 * v + 2] += c.z;
        dv[d4][4 * v + 3] += c.w;
      }
  }
  float ks = scale;
  if (rcos != nullptr && kok) {  // inverse rotate_half RoPE on dK: columns d and d + 64 are blocks d4 and d4 + 2
    const long tr = (long)(start + key) * (D / 2);
    rope_bwd32(dk, rcos + tr, rsin + tr, scale);
    ks = 1.f;
  }
  store_t21(dqkv + (long)(start + key) * ld + (nq + kvh) * D, dk, ks, kok);
  store_t21(dqkv + (long)(start + key) * ld + (nq + nkv + kvh) * D, dv, 1.f, kok);
}

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

// host launcher of the GQA-grouped dK/dV: G = 2 head groups (Q / dO by LDS-DMA) when rep is even, else G = 1
static void launch_dkdv5(const u16* qkv, const u16* dout, const float* lse, const float* delta, const int* cu,
                         u16* dqkv, int nq, int nkv, int total, int nseq, int max_seqlen, float sl2, float scale,
                         int causal, u16* dst, int lp, hipStream_t st, const float* rcos = nullptr,
                         const float* rsin = nullptr) {
  const int rep = nq / nkv;
  dim3 grid(nkv, nseq, (max_seqlen + 63) / 64);
  const char* e5 = std::getenv("SFTAMD_ATTN_DKDV5");  // A/B against the 16x16x32 dkdv5 (read per call)
  if (!(e5 && std::strcmp(e5, "1") == 0)) {
    if (rep % 2 == 0)
      bwd_dkdv32_kernel<2><<<grid, 256, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
                                                 dst, lp, rcos, rsin);
    else
      bwd_dkdv32_kernel<1><<<grid, 128, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
                                                 dst, lp, rcos, rsin);
    return;
  }
  if (rep % 2 == 0)
    bwd_dkdv5_kernel<2, false, true><<<grid, 512, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2,
                                                           scale, causal, dst, lp, rcos, rsin);
  else
    bwd_dkdv5_kernel<1><<<grid, 256, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
                                              dst, lp, rcos, rsin);
}

}  // namespace attn

static void check_attn_args(const at::Tensor& qkv, const at::Tensor& cu, int64_t nq, int64_t nkv, int64_t hd) {
  SFT_CHECK_CUDA(qkv);
  SFT_CHECK_BF16(qkv);
  SFT_CHECK_CONTIG(qkv);
  SFT_CHECK(hd == attn::D, "flash attention kernel is built for head_dim 128, got ", hd);
  SFT_CHECK(nq % nkv == 0, "nq must be a multiple of nkv");
  SFT_CHECK(qkv.dim() == 2 && qkv.size(1) == (nq + 2 * nkv) * hd, "qkv must be [M, (nq+2nkv)*hd]");
  SFT_CHECK(cu.scalar_type() == at::kInt && cu.is_cuda() && cu.dim() == 1 && cu.numel() >= 2, "cu_seqlens int32");
}

// The dq4 backward stores the bf16 dS^T blocks of every (sequence, head) — nseq x nq x lp^2 x 2 bytes (134 MB for
// 16 x 512 tokens, 16 heads); past SFTAMD_ATTN_DS_MB (default 2048, read per call so tests can switch paths
// in-process) the dq3 kernel recomputes S / dP instead (long contexts).
static long attn_ds_budget() {
  const char* e = std::getenv("SFTAMD_ATTN_DS_MB");
  return (e && e[0] ? atol(e) : 2048L) * 1024L * 1024L;
}

// forward: fwd3 (8 waves x 16 query rows, K / V staged by LDS-DMA into two stages, one barrier per 64-key tile)
std::tuple<at::Tensor, at::Tensor> flash_fwd(const at::Tensor& qkv, const at::Tensor& cu, int64_t max_seqlen,
                                             int64_t nq, int64_t nkv, int64_t hd, double scale, bool causal) {
  check_attn_args(qkv, cu, nq, nkv, hd);
  const int total = qkv.size(0);
  const int nseq = cu.numel() - 1;
  auto out = at::empty({total, nq * hd}, qkv.options());
  auto lse = at::empty({nq, total}, qkv.options().dtype(at::kFloat));
  if (total == 0 || max_seqlen == 0) return {out, lse};
  const float sl2 = (float)scale * attn::LOG2E;
  auto cu_c = cu.contiguous();
  const char* e16 = std::getenv("SFTAMD_ATTN_FWD16");  // A/B against the 16x16x32 fwd3 (read per call)
  const bool use16 = e16 && std::strcmp(e16, "1") == 0;
  const u16* q = (const u16*)qkv.data_ptr();
  u16* o = (u16*)out.data_ptr();
  float* lp = lse.data_ptr<float>();
  const int* cp = cu_c.data_ptr<int>();
  const int ca = causal ? 1 : 0;
  if (use16) {
    SFT_TRACE("attn.fwd3");
    dim3 g3(nq, nseq, (max_seqlen + 127) / 128);
    attn::fwd3_kernel<8, 32><<<g3, 512, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
  } else {
    SFT_TRACE("attn.fwd32");
    const int rep = nq / nkv, hw = rep % 4 == 0 ? 4 : rep % 2 == 0 ? 2 : 1, span = 32 * (4 / hw);
    dim3 g(nq / hw, nseq, (max_seqlen + span - 1) / span);
    if (hw == 4) attn::fwd32_kernel<4><<<g, 256, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
    else if (hw == 2) attn::fwd32_kernel<2><<<g, 256, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
    else attn::fwd32_kernel<1><<<g, 256, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
  }
  SFT_LAUNCH_CHECK();
  return {out, lse};
}

// backward: delta = rowsum(dO * O); GQA-grouped dK/dV (bwd_dkdv5: all query heads of a kv head in one workgroup, no
// partials) writing dS^T, then dQ = one product per tile (bwd_dq4); past the dS^T budget dK/dV + the recomputing dq3.
// rcos / rsin (optional, [total, hd / 2] fp32): the inverse rotate_half RoPE applied to the dq and dk heads in the
// dq4 / dK epilogues (sets rope_done); the dq3 path leaves it to the caller.
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
  const u16* q = (const u16*)qkv.data_ptr();
  const u16* dO = (const u16*)dout.data_ptr();
  const long lp = (max_seqlen + 127) / 128 * 128;
  const long ds_bytes = (long)nseq * nq * lp * lp * 2;
  if (ds_bytes <= attn_ds_budget()) {
    auto dst = at::empty({ds_bytes / 2}, qkv.options());
    const bool rope = rcos != nullptr;
    SFT_TRACE("attn.dkdv5");
    SFT_TRACE("attn.dq4");
    if (rope) SFT_TRACE("attn.bwd_rope_epi");
    attn::launch_dkdv5(q, dO, lse.data_ptr<float>(), delta.data_ptr<float>(), cu_c.data_ptr<int>(),
                       (u16*)dqkv.data_ptr(), nq, nkv, total, nseq, max_seqlen, sl2, (float)scale, causal ? 1 : 0,
                       (u16*)dst.data_ptr(), (int)lp, cur_stream(), rcos, rsin);
    SFT_LAUNCH_CHECK();
    const char* e5 = std::getenv("SFTAMD_ATTN_DKDV5");  // A/B: the 16x16x32 dkdv5 + dq4 pair (read per call)
    if (e5 && std::strcmp(e5, "1") == 0) {
      dim3 gq4(nq, nseq, (max_seqlen + 127) / 128);
      attn::bwd_dq4_kernel<8><<<gq4, 512, 0, cur_stream()>>>(q, (const u16*)dst.data_ptr(), cu_c.data_ptr<int>(),
                                                             (u16*)dqkv.data_ptr(), nq, nkv, (int)lp, (float)scale,
                                                             causal ? 1 : 0, rcos, rsin);
    } else {
      const int rep = nq / nkv, hw = rep % 4 == 0 ? 4 : rep % 2 == 0 ? 2 : 1, span = 32 * (4 / hw);
      dim3 g(nq / hw, nseq, (max_seqlen + span - 1) / span);
      const u16* ds = (const u16*)dst.data_ptr();
      u16* dx = (u16*)dqkv.data_ptr();
      const int* cp = cu_c.data_ptr<int>();
      const int ca = causal ? 1 : 0;
      if (hw == 4) attn::bwd_dq32_kernel<4><<<g, 256, 0, cur_stream()>>>(q, ds, cp, dx, nq, nkv, (int)lp, (float)scale, ca, rcos, rsin);
      else if (hw == 2) attn::bwd_dq32_kernel<2><<<g, 256, 0, cur_stream()>>>(q, ds, cp, dx, nq, nkv, (int)lp, (float)scale, ca, rcos, rsin);
      else attn::bwd_dq32_kernel<1><<<g, 256, 0, cur_stream()>>>(q, ds, cp, dx, nq, nkv, (int)lp, (float)scale, ca, rcos, rsin);
    }
    SFT_LAUNCH_CHECK();
    rope_done = rope;
    return dqkv;
  }
  SFT_TRACE("attn.dq3");
  dim3 gq3(nq, nseq, (max_seqlen + 127) / 128);
  attn::bwd_dq3_kernel<8><<<gq3, 512, 0, cur_stream()>>>(q, dO, lse.data_ptr<float>(), delta.data_ptr<float>(),
                                                         cu_c.data_ptr<int>(), (u16*)dqkv.data_ptr(), nq, nkv, total,
                                                         sl2, (float)scale, causal ? 1 : 0);
  SFT_LAUNCH_CHECK();
  attn::launch_dkdv5(q, dO, lse.data_ptr<float>(), delta.data_ptr<float>(), cu_c.data_ptr<int>(),
                     (u16*)dqkv.data_ptr(), nq, nkv, total, nseq, max_seqlen, sl2, (float)scale, causal ? 1 : 0,
                     nullptr, 0, cur_stream());
  SFT_LAUNCH_CHECK();
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
