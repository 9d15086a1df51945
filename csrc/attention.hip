// Varlen causal GQA flash-attention forward/backward for gfx950.
//
// Layout: the packed QKV GEMM output qkv[M, (nq + 2*nkv) * 128] (bf16, token-major, no
// transposes anywhere); sequences are [cu[b], cu[b+1]). Output o[M, nq*128], lse[nq, M] (fp32,
// natural log). Backward returns dqkv in the same packed layout, ready for the fused QKV
// linear's backward.
//
// Kernels (all on gfx950 MFMA, fp32 accumulate, bf16 I/O):
// * fwd32_kernel: v_mfma_f32_32x32x16_bf16, S^T = K Q^T with the query on the lane (row max / sum lane-local + one
//   permlane32 swap), P^T fed to O^T += V^T P^T straight from the accumulator registers; the GQA heads of a kv head
//   share each K / V tile (LDS-DMA, two stages, buffer descriptors: rows past the sequence end read as zero);
// * bwd: delta_kernel (rowsum dO . O), bwd_dkdv32_kernel (S and dP with the KEY on the lane, P / dS as the register
//   B operands of dV^T / dK^T, dS^T materialised for dQ), bwd_dq32_kernel (dQ^T = K^T dS^T). Past the dS^T budget
//   (SFTAMD_ATTN_DS_MB) the recomputing bwd_dq3_kernel (16x16x32) replaces dq32.
// * LDS images [rows][128] bf16 with an XOR swizzle that is conflict-free for both the 16-byte row reads and the
//   gfx950 transposed read ds_read_b64_tr_b16 (tools/lds_swizzle_check.py).
//
// mfma_f32_16x16x32_bf16 lane maps (dq3; g = lane >> 4, r = lane & 15, j = 0..7, i = 0..3):
//   A[row r][k 8g+j], B[k 8g+j][col r], C[row 4g+i][col r].
// Accumulator-as-operand: two 16-row C tiles (t0, t1) give lane (g, r) the k values
//   {4g+i} from t0 and {16+4g+i} from t1; we use that order as the k permutation
//   p(8g+j) = j<4 ? 4g+j : 16+4g+(j-4) on BOTH operands of the next MFMA.
// The 32x32x16 lane maps are at fwd32 below.
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
  typedef __attribute__((ext_vector_type(4))) unsigned w4;
  return __builtin_bit_cast(bf16x8, w4{pk2bf(t0[0], t0[1]), pk2bf(t0[2], t0[3]), pk2bf(t1[0], t1[1]), pk2bf(t1[2], t1[3])});
}

__device__ __forceinline__ bf16x8 load_frag_global(const u16* p, bool ok) {
  if (!ok) return bf16x8{};
  return __builtin_bit_cast(bf16x8, *(const uint4*)p);
}

__device__ __forceinline__ void store4(u16* p, const f32x4& v, float s) {
  uint2 w;
  w.x = pk2bf(v[0] * s, v[1] * s);
  w.y = pk2bf(v[2] * s, v[3] * s);
  *(uint2*)p = w;
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

typedef float f32x2 __attribute__((ext_vector_type(2)));
// v_max3_f32 (fmaxf's NaN canonicalisation doubles the VALU count; scores are finite or -inf here)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
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

// ============================================================================== fwd32: 32x32x16 forward
// v_mfma_f32_32x32x16_bf16 lane maps (hi = lane >> 5, c = lane & 31, j = 0..7, i = 0..15):
//   A[row c][k 8hi+j], B[k 8hi+j][col c], C[row crow(i, hi)][col c], crow(i, hi) = (i & 3) + 8 (i >> 2) + 4 hi.
// S^T = K Q^T with the query on the lane: lane (hi, c) holds 16 keys of each 32-key block for query c, so the row max
// and sum are lane-local plus ONE permlane32 swap, and the accumulator registers 8 sub .. 8 sub + 7 of block kb are
// already the B operand (P^T) of k-step 2 kb + sub of O^T += V^T P^T: they hold keys 16 ks + 4 hi + {0..3} and
// 16 ks + 8 + 4 hi + {0..3}, so the V^T A operand is read with that key order (two ds_read_b64_tr_b16, rows
// 16 ks + 4 hi + q and 16 ks + 8 + 4 hi + q). Per 64-key tile and 32 queries: 16 + 16 MFMAs (each 2x the work of a
// 16x16x32), 16 ds_read_b128 + 32 ds_read_b64_tr_b16 — half the LDS bytes per FLOP of the 16x16x32 forward it
// replaced (46 -> 35 us at 16 x 512, SmolLM3 heads).
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

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
__device__ __forceinline__ u32x4 pack8w(const f32x16& t, int base) {  // t[base .. base + 7] as 4 bf16 pairs
  return u32x4{pk2bf(t[base], t[base + 1]), pk2bf(t[base + 2], t[base + 3]), pk2bf(t[base + 4], t[base + 5]),
               pk2bf(t[base + 6], t[base + 7])};
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& t, int base) {
  return __builtin_bit_cast(bf16x8, pack8w(t, base));
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
      const unsigned ax = pk2bf(a[db][i0] * s, a[db][i0 + 1] * s);
      const unsigned ay = pk2bf(a[db][i0 + 2] * s, a[db][i0 + 3] * s);
      const unsigned bx = pk2bf(a[db][i0 + 4] * s, a[db][i0 + 5] * s);
      const unsigned by = pk2bf(a[db][i0 + 6] * s, a[db][i0 + 7] * s);
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

// dQ past the dS^T budget (long contexts): per 64-key tile S^T and dP^T are recomputed from Q, K, V, dO, lse and delta
// (16x16x32 MFMAs, 48 per tile and wave instead of dq32's 16) and dQ^T += K^T dS^T; 8 waves x 16 queries.
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
// queries x 4 products), 32 ds_read_b128 + 64 ds_read_b64_tr_b16 — half the LDS bytes per FLOP of the 16x16x32
// dK/dV kernel it replaced. dS^T ([b][h][key][q], row stride lp) is written for bwd_dq32 when drow is given
// (T21-paired 16-B stores).
__device__ __forceinline__ void dkdv32_step(const char* __restrict__ cur, char* __restrict__ nxt, bool pre,
                                            rsrc_t qr, rsrc_t orr, unsigned vq0, unsigned vq1, unsigned vo0,
                                            unsigned vo1, unsigned qso, unsigned oso, unsigned rowb, unsigned rowo,
                                            int wv, const float* lsrc, const float* dsrc, int gl, int q0, int len,
                                            int causal, int kw0, int key, float sl2, u16* drow,
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
  const bool wds = __builtin_amdgcn_readfirstlane((int)(drow != nullptr));  // (drow is per lane, the test uniform)
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
        const int i = 4 * m + t;
        const float p = exp2f(__builtin_fmaf(s[i], sl2, -L[t]));
        dp[i] = p * (dp[i] - Dd[t]);
        s[i] = p;
      }
    }
    // The mask as a real (wave-uniform) branch: only the diagonal and the sequence-end tiles take it. Folded into the
    // loop above as selects it cost 50 of the ~245 VALU per half tile on every tile, and this loop is VALU-bound
    // (~10 VALU per 32x32x16 MFMA, PMC in profiles/r6_attention.md). A masked element's p (possibly inf / NaN from an
    // unmasked exp) is replaced, so the result is the select form's.
    if (need_mask) {
      int vlo = lo, vhi = hq;
      asm volatile("" : "+v"(vlo), "+v"(vhi));  // the compares depend on volatile code: not hoisted out of the branch
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = 8 * (i >> 2) + (i & 3);
        if (o < vlo || o > vhi) s[i] = dp[i] = 0.f;
      }
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const u32x4 dw = pack8w(dp, 8 * sub);  // dS (bf16) once, for the MFMA operand and the dS^T store
      if (wds) {  // dS^T[key][q]: registers 8 sub .. 8 sub + 7 = queries 16 sub + 4 hi + {0..3, 8..11}
        const auto rx = __builtin_amdgcn_permlane32_swap(dw[0], dw[2], false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(dw[1], dw[3], false, false);
        // (also for keys past the sequence end: their rows are inside the [lp][lp] block, key < k0 + 64 <= lp, and
        // bwd_dq32 never reads them — no divergent branch around the store)
        *(uint4*)(drow + 32 * qb + 16 * sub + 8 * hi) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
      }
      const bf16x8 pb = pack8(s, 8 * sub), db = __builtin_bit_cast(bf16x8, dw);
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
                lok ? lse + lo : nullptr, delta + lo, gl, q0, len, causal, kw0, key, sl2, drow, off, kf, Vk, dk,
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

// host launcher of the GQA-grouped dK/dV: G = 2 head groups when rep is even, else G = 1
static void launch_dkdv(const u16* qkv, const u16* dout, const float* lse, const float* delta, const int* cu,
                        u16* dqkv, int nq, int nkv, int total, int nseq, int max_seqlen, float sl2, float scale,
                        int causal, u16* dst, int lp, hipStream_t st, const float* rcos = nullptr,
                        const float* rsin = nullptr) {
  dim3 grid(nkv, nseq, (max_seqlen + 63) / 64);
  if ((nq / nkv) % 2 == 0)
    bwd_dkdv32_kernel<2><<<grid, 256, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
                                               dst, lp, rcos, rsin);
  else
    bwd_dkdv32_kernel<1><<<grid, 128, 0, st>>>(qkv, dout, lse, delta, cu, dqkv, nq, nkv, total, sl2, scale, causal,
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

// The default backward stores the bf16 dS^T blocks of every (sequence, head) — nseq x nq x lp^2 x 2 bytes (134 MB for
// 16 x 512 tokens, 16 heads); past SFTAMD_ATTN_DS_MB (default 2048, read per call so tests can switch paths
// in-process) the dq3 kernel recomputes S / dP instead (long contexts).
static long attn_ds_budget() {
  const char* e = std::getenv("SFTAMD_ATTN_DS_MB");
  return (e && e[0] ? atol(e) : 2048L) * 1024L * 1024L;
}

// forward: fwd32 (4 waves = HW GQA heads x 4 / HW 32-query blocks sharing each K / V tile)
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
  const u16* q = (const u16*)qkv.data_ptr();
  u16* o = (u16*)out.data_ptr();
  float* lp = lse.data_ptr<float>();
  const int* cp = cu_c.data_ptr<int>();
  const int ca = causal ? 1 : 0;
  SFT_TRACE("attn.fwd32");
  const int rep = nq / nkv, hw = rep % 4 == 0 ? 4 : rep % 2 == 0 ? 2 : 1, span = 32 * (4 / hw);
  dim3 g(nq / hw, nseq, (max_seqlen + span - 1) / span);
  if (hw == 4) attn::fwd32_kernel<4><<<g, 256, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
  else if (hw == 2) attn::fwd32_kernel<2><<<g, 256, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
  else attn::fwd32_kernel<1><<<g, 256, 0, cur_stream()>>>(q, o, lp, cp, nq, nkv, total, sl2, ca);
  SFT_LAUNCH_CHECK();
  return {out, lse};
}

// backward: delta = rowsum(dO * O); GQA-grouped dK/dV (bwd_dkdv32: all query heads of a kv head in one workgroup, no
// partials) writing dS^T, then dQ = one product per tile (bwd_dq32); past the dS^T budget dK/dV + the recomputing dq3.
// rcos / rsin (optional, [total, hd / 2] fp32): the inverse rotate_half RoPE applied to the dq and dk heads in the
// dq32 / dK epilogues (sets rope_done); the dq3 path leaves it to the caller.
static at::Tensor flash_bwd_impl(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out,
                                 const at::Tensor& lse, const at::Tensor& cu, int64_t max_seqlen, int64_t nq,
                                 int64_t nkv, int64_t hd, double scale, bool causal, const float* rcos,
                                 const float* rsin, bool& rope_done, const c10::optional<at::Tensor>& delta_in) {
  rope_done = false;
  check_attn_args(qkv, cu, nq, nkv, hd);
  SFT_CHECK_CONTIG(dout);
  SFT_CHECK_CONTIG(out);
  SFT_CHECK(dout.sizes() == out.sizes() && out.size(1) == nq * hd, "dout/out shape");
  const int total = qkv.size(0);
  const int nseq = cu.numel() - 1;
  auto dqkv = at::empty_like(qkv);
  if (total == 0 || max_seqlen == 0) return dqkv;
  at::Tensor delta;
  if (delta_in.has_value() && delta_in->defined()) {  // computed by the producer of dO (dgrad_gemm_delta's epilogue)
    delta = *delta_in;
    SFT_CHECK(delta.scalar_type() == at::kFloat && delta.is_contiguous() && delta.dim() == 2 && delta.size(0) == nq &&
                  delta.size(1) == total && delta.device() == qkv.device(),
              "flash_bwd: delta must be contiguous fp32 [n_q, total]");
  } else {
    SFT_TRACE("attn.delta_kernel");
    delta = at::empty({nq, total}, qkv.options().dtype(at::kFloat));
    const long rows = (long)total * nq;
    attn::delta_kernel<<<(rows + 15) / 16, 256, 0, cur_stream()>>>((const u16*)dout.data_ptr(),
                                                                    (const u16*)out.data_ptr(), delta.data_ptr<float>(),
                                                                    total, nq);
    SFT_LAUNCH_CHECK();
  }
  const float sl2 = (float)scale * attn::LOG2E;
  auto cu_c = cu.contiguous();
  const u16* q = (const u16*)qkv.data_ptr();
  const u16* dO = (const u16*)dout.data_ptr();
  const long lp = (max_seqlen + 127) / 128 * 128;
  const long ds_bytes = (long)nseq * nq * lp * lp * 2;
  if (ds_bytes <= attn_ds_budget()) {
    auto dst = at::empty({ds_bytes / 2}, qkv.options());
    const bool rope = rcos != nullptr;
    SFT_TRACE("attn.dkdv32");
    SFT_TRACE("attn.dq32");
    if (rope) SFT_TRACE("attn.bwd_rope_epi");
    attn::launch_dkdv(q, dO, lse.data_ptr<float>(), delta.data_ptr<float>(), cu_c.data_ptr<int>(),
                       (u16*)dqkv.data_ptr(), nq, nkv, total, nseq, max_seqlen, sl2, (float)scale, causal ? 1 : 0,
                       (u16*)dst.data_ptr(), (int)lp, cur_stream(), rcos, rsin);
    SFT_LAUNCH_CHECK();
    {
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
  attn::launch_dkdv(q, dO, lse.data_ptr<float>(), delta.data_ptr<float>(), cu_c.data_ptr<int>(),
                     (u16*)dqkv.data_ptr(), nq, nkv, total, nseq, max_seqlen, sl2, (float)scale, causal ? 1 : 0,
                     nullptr, 0, cur_stream());
  SFT_LAUNCH_CHECK();
  return dqkv;
}

at::Tensor flash_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& lse,
                     const at::Tensor& cu, int64_t max_seqlen, int64_t nq, int64_t nkv, int64_t hd, double scale,
                     bool causal, const c10::optional<at::Tensor>& delta) {
  bool rope_done;
  return flash_bwd_impl(dout, qkv, out, lse, cu, max_seqlen, nq, nkv, hd, scale, causal, nullptr, nullptr, rope_done,
                        delta);
}

void rope_(at::Tensor qkv, const at::Tensor& cos, const at::Tensor& sin, int64_t n_q, int64_t n_kv, int64_t head_dim,
           bool inverse);  // elementwise.hip

// flash_bwd for a qkv whose q / k heads were rotated (RoPE) by the producing GEMM: returns the gradient w.r.t. the
// UNROTATED qkv. The inverse rotation rides in the dq / dK epilogues on the default path; otherwise the rope kernel
// runs after the backward.
at::Tensor flash_bwd_rope(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& lse,
                          const at::Tensor& cu, int64_t max_seqlen, int64_t nq, int64_t nkv, int64_t hd, double scale,
                          bool causal, const at::Tensor& cos, const at::Tensor& sin,
                          const c10::optional<at::Tensor>& delta) {
  SFT_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                sin.is_contiguous() && cos.is_cuda() && sin.is_cuda(),
            "flash_bwd_rope: contiguous fp32 cos / sin");
  SFT_CHECK(cos.numel() == qkv.size(0) * hd / 2 && sin.numel() == cos.numel(), "flash_bwd_rope: cos / sin [total, hd/2]");
  bool rope_done;
  auto dqkv = flash_bwd_impl(dout, qkv, out, lse, cu, max_seqlen, nq, nkv, hd, scale, causal, cos.data_ptr<float>(),
                             sin.data_ptr<float>(), rope_done, delta);
  if (!rope_done) rope_(dqkv, cos, sin, nq, nkv, hd, true);
  return dqkv;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("flash_fwd", &flash_fwd);
  m.impl("flash_bwd", &flash_bwd);
  m.impl("flash_bwd_rope", &flash_bwd_rope);
}

}  // namespace sftamd
