// 4-wave 256 x 256 MFMA GEMM for the two backward layouts on gfx950 (MI355X):
//
//   weight gradient  dW[N, K] (+)= dy[T, N]^T . x[T, K]      A = dy  (TR: reduction T is the ROW index)
//                                                             B = x   (TR)
//   input gradient   dX[M, N]   = dy[M, K] . W[K, N]          A = dy  (ROW: reduction K contiguous)
//                                                             B = W   (TR: reduction K is the row index)
//
// C[m][n] = sum_k A'[m][k] B'[n][k]. One workgroup = 4 waves = one wave per SIMD, each wave a 128 x 128 output
// tile whose 256 fp32 accumulators are pinned in the AGPR file: the MFMAs are inline asm with the accumulator TIED
// ("+a"), which is what lets hipcc keep 256 accumulators next to double-buffered fragments without renaming them
// through v_accvgpr_read / write or spilling (profiles/r3_gemm_4wave.md). Why 4 waves: a 128 x 128 wave tile reads 16
// fragments per 64 MFMAs instead of the 12 per 32 of 128 x 64 tiles — a third fewer LDS bytes per FLOP — and one
// wave per SIMD leaves the matrix pipe to a single in-order instruction stream (/opt/skills/guides/MI355X_MICROARCH.md
// "Two waves per SIMD", item 1). The 8-wave weight-gradient rings ran at 48-56 % MFMA busy inside the training step
// (profiles/r2_step_pmc.md).
//
// Main loop: 32-deep K-steps in NS = 4 LDS slots of 32 KB (128 KB), three steps in flight ahead of the one being
// computed. Per step u (slot u % 4):
//   vmcnt: this wave's pieces of step u + 1 landed (F(u) was read during step u - 1: the compiler's counted LDS waits)
//   MFMA group 0 | lgkmcnt(0), barrier (every wave's step u + 1 landed, every wave done reading slot u % 4)
//   MFMA on F(u) | ds_read F(u + 1) from slot (u + 1) % 4 | LDS-DMA of step u + 4 -> slot u % 4
// with the 16 fragment reads and 8 DMA pieces placed ONE PER MFMA GAP (op k after MFMA 8 + 7k/3, order B0 B1 D0 B2
// B3 D1 .. A6 A7 D7): one wave per SIMD issues in order, and a burst that outlasts the 16-cycle gap of
// v_mfma_f32_16x16x32_bf16 idles the matrix pipe (hipBLASLt's MT256x256x64 loop places one ds_read / buffer_load
// between consecutive MFMAs: profiles/r6_g4_interleave.md, +1.3 % in the step over 2 reads + 1 piece per 8 MFMAs).
// B fragments first: the next step's group 0 needs all 8 B and A0. The reduction length must be a multiple of 128 (one
// loop body = 4 steps on compile-time slot pointers).
//
// Operand staging (LDS-DMA through a buffer descriptor, 16 B per lane, 1 KB per wave instruction; the chunk swizzle is
// applied to the GLOBAL source address because the DMA writes LDS lane-linearly):
//   ROW operand: image [256 rows][32 k], 64-B rows, chunk c at slot c ^ S((row >> 2) & 3), S = {0, 2, 3, 1}: the
//                16-lane groups of ds_read_b128 conflict-free; a fragment is one ds_read_b128 per lane;
//   TR operand:  two images [32 k][128 columns], 256-B rows, chunk c of row r at slot c ^ 2 ((r & 3) | ((r >> 3) & 1)
//                << 2); a fragment is two ds_read_b64_tr_b16 per lane (rows 8g .. 8g + 3 and 8g + 4 .. 8g + 7), i.e.
//                the same k 8g .. 8g + 7 as the ROW side. Lane groups {0, 1} / {2, 3} of a 32-lane half read 8 rows
//                whose 32-byte column pairs the swizzle spreads over all 64 banks: conflict-free.
// MFMA v_mfma_f32_16x16x32_bf16 with the B fragment first (transposed C): each lane ends with 4 consecutive output
// columns of one row per fragment, and v_permlane16_swap pairs two fragments into 8 consecutive columns, so the
// epilogue writes 16-byte vectors straight from registers (no LDS round trip).
//
// Wave quantisation (weight gradients: down_proj 344 tiles = 1.34 rounds of 256 CUs, lm_head 4008 = 15.7): the tiles
// past the last whole round can be split S ways over the reduction (hybrid data-parallel + split-K, 128-deep blocks
// per split) into fp32 slabs summed in a fixed order by splitk_fixup_kernel (deterministic); small grids (qkv 96
// tiles, o_proj 64) split every tile. A stream-K partition of the last round (ranges crossing tile boundaries) was
// measured and dropped: no faster on any SmolLM3 shape (profiles/r6_gemm_routing.md).
#include <climits>

#include "common.h"
#include "g4_api.h"
#include "splitk_fixup.h"

namespace sftamd {
namespace g4 {

constexpr int BK32 = 32;
constexpr int OPB32 = 256 * BK32 * 2;  // one operand's 32-deep K-step: 16 KB
constexpr int SLOT32 = 2 * OPB32;      // 32 KB
constexpr int ROWB_T = 256;            // TR image row: 128 columns x bf16
constexpr int IMG32 = BK32 * ROWB_T;   // 8 KB
enum { ROW = 0, TR = 1 };

__device__ __forceinline__ int xt(int row) { return 2 * ((row & 3) | (((row >> 3) & 1) << 2)); }
__device__ __forceinline__ int sel4(int q) { return (0x78 >> (2 * q)) & 3; }

// LDS-DMA through a buffer descriptor: the tile's base in the (wave-uniform) descriptor, each lane's byte offset in a
// VGPR fixed for the whole loop, the piece / K-step offset in an SGPR — no per-piece 64-bit VALU address arithmetic
// (the global_load_lds form cost a v_lshl_add_u64 per piece), as hipBLASLt's MT256x256x64 loop does.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t tile_rsrc(const u16* p) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, 0xFFFFFFFFu, 0x00020000);
}
__device__ __forceinline__ void bldsx4(rsrc_t r, char* dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}

constexpr unsigned waitcnt_imm(int vm, int lgkm) {  // gfx9: vmcnt[3:0] expcnt[6:4] lgkmcnt[11:8] vmcnt[5:4]<<14
  return (unsigned)((vm & 15) | (7 << 4) | ((lgkm & 15) << 8) | ((vm >> 4) << 14));
}

typedef __attribute__((address_space(3))) s16x4 lds_s4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

__device__ __forceinline__ void mfma(f32x4& c, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}

// One operand: the lane's DMA source for the wave's first piece of a step, and its fragment read offsets.
// `sub` = which 128-wide half of the 256 tile the wave computes on this side (wm for A, wn for B).
template <int L>
struct Op32;

template <>
struct Op32<ROW> {
  rsrc_t r;
  unsigned voff, jst, koff, kmax;  // lane offset; bytes per 64 rows; K progress; its cap (the last step)
  int off;   // fragment 0 (fragment i is 1024 B further)
  __device__ __forceinline__ void init(const u16* base, long ld, int r0, long k0, int w, int lane, int sub) {
    // piece P = w + 4 j: 16 rows 16 P + lr (lr = lane >> 2), slot lane & 3; (row >> 2) & 3 = lr >> 2 for all pieces
    const int lr = lane >> 2, ch = (lane & 3) ^ sel4(lr >> 2);
    r = tile_rsrc(base + (long)r0 * ld + k0);
    voff = (unsigned)(((16 * w + lr) * ld + 8 * ch) * 2);
    jst = (unsigned)(128 * ld);
    koff = 0;
    kmax = 0xFFFFFFFFu;
    const int g = lane >> 4, ii = lane & 15;
    off = (128 * sub + ii) * 64 + 16 * (g ^ sel4(ii >> 2));
  }
  __device__ __forceinline__ void limit(int nsteps) { kmax = (unsigned)(nsteps - 1) * 2 * BK32; }
  __device__ __forceinline__ void advance() { koff = min(koff + 2 * BK32, kmax); }
  __device__ __forceinline__ void piece(char* opb, int w, int j) const {
    bldsx4(r, opb + (w + 4 * j) * 1024, voff, koff + j * jst);
  }
  __device__ __forceinline__ bf16x8 frag(const char* opb, int i) const { return *(const bf16x8*)(opb + off + 1024 * i); }
};

template <>
struct Op32<TR> {
  rsrc_t r;
  unsigned voff, jst, kst, koff, kmax;  // lane offset; bytes per 16 rows; per step (32 rows); K progress; its cap
  int ob, x2;
  __device__ __forceinline__ void init(const u16* base, long ld, int c0, long k0, int w, int lane, int sub) {
    // piece (image j >> 1, q = w + 4 (j & 1)): rows 4q + lr4; xt(row) = 2 (lr4 | ((w >> 1) & 1) << 2) for all
    const int lr4 = lane >> 4, row = 4 * w + lr4, ch = (lane & 15) ^ xt(row);
    r = tile_rsrc(base + k0 * ld + c0);
    voff = (unsigned)((row * ld + 8 * ch) * 2);
    jst = (unsigned)(32 * ld);
    kst = (unsigned)(2 * BK32 * ld);
    koff = 0;
    kmax = 0xFFFFFFFFu;
    const int g = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    x2 = qq | ((g & 1) << 2);
    ob = sub * IMG32 + (8 * g + qq) * ROWB_T + 8 * pp;
  }
  __device__ __forceinline__ void limit(int nsteps) { kmax = (unsigned)(nsteps - 1) * kst; }
  __device__ __forceinline__ void advance() { koff = min(koff + kst, kmax); }
  __device__ __forceinline__ void piece(char* opb, int w, int j) const {
    bldsx4(r, opb + (j >> 1) * IMG32 + (w + 4 * (j & 1)) * 1024, voff, koff + (j & 1) * jst + 256 * (j >> 1));
  }
  __device__ __forceinline__ bf16x8 frag(const char* opb, int i) const {
    const char* q = opb + ob + 32 * (i ^ x2);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)q);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(q + 4 * ROWB_T));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
};

struct Epi {
  u16* C;          // output rows [M, ldc]
  float* P;        // split slabs (+ parked whole-tile norm partials) or the norm slots (no split)
  long ldc;
  int flags;       // bit 0: accumulate into C (beta = 1); bit 1: gradient-norm partials; bit 2: attention delta
  const u16* O;    // flags & 4: the attention output [M, ldO] (C = dO, its gradient) ...
  float* Dl;       // ... and delta [C columns / 128][dM] = per-head rowsum(bf16(dO) * O)
  long ldO;
  int dM;
};

__device__ __forceinline__ float fbits(unsigned u) { return __uint_as_float(u); }

// TRC accumulators -> 8 consecutive fp32 columns per (fragment row i, fragment pair p) per lane: lane (g, ii) holds
// row 16 i + ii, columns 32 p + 16 (g & 1) + 8 (g >> 1) + 0..7 of the wave tile.
__device__ __forceinline__ void gather8(const f32x4 (&acc)[8][8], int i, int p, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][e]), __float_as_uint(acc[i][2 * p + 1][e]),
                                              false, false);
    v[e] = fbits(r[0]);
    v[4 + e] = fbits(r[1]);
  }
}

// Whole tile -> C (bf16, optionally + C); nrm: this wave's gradient-norm slot (sum of squares of the stored values).
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[8][8], const Epi& ea, int row0, int col0, int lane,
                                           float* nrm) {
  const int g = lane >> 4, ii = lane & 15;
  const int cofs = col0 + 16 * (g & 1) + 8 * (g >> 1);
  float ss = 0.f;
  if (ea.flags & 1) {
    // the accumulated C streams through a PD-deep register ring over the 32 (fragment row, column pair) units: unit
    // u + PD is loaded while unit u computes, instead of one exposed HBM round trip per unit (the fragment registers
    // of the main loop are free here)
    constexpr int U = 32, PD = 8;
    auto at = [&](int u) -> long { return (long)(row0 + 16 * (u >> 2) + ii) * ea.ldc + cofs + 32 * (u & 3); };
    uint4 rg[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u) rg[u] = *(const uint4*)(ea.C + at(u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[8], a[8];
      gather8(acc, u >> 2, u & 3, v);
      unpack8(rg[u % PD], a);
      if (u + PD < U) rg[u % PD] = *(const uint4*)(ea.C + at(u + PD));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += a[e];
      if (nrm != nullptr) {
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += v[e] * v[e];
      }
      *(uint4*)(ea.C + at(u)) = pack8(v);
    }
  } else if (ea.flags & 4) {
    // the input gradient of the attention output projection, dO, with flash attention's delta = rowsum(dO . O) per
    // head fused (the backward's first kernel otherwise: a full re-read of dO and O): the wave tile is 128 rows x ONE
    // head's 128 columns, each row on the 4 lanes ii + 16 g. O streams through a PD-deep register ring as C does above;
    // the products use the stored (bf16-rounded) dO, as the standalone kernel would read it.
    constexpr int U = 32, PD = 8;
    auto ato = [&](int u) -> long { return (long)(row0 + 16 * (u >> 2) + ii) * ea.ldO + cofs + 32 * (u & 3); };
    uint4 rg[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u) rg[u] = *(const uint4*)(ea.O + ato(u));
    float part = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[8], o[8], r[8];
      gather8(acc, u >> 2, u & 3, v);
      unpack8(rg[u % PD], o);
      if (u + PD < U) rg[u % PD] = *(const uint4*)(ea.O + ato(u + PD));
      const uint4 pk = pack8(v);
      *(uint4*)(ea.C + (long)(row0 + 16 * (u >> 2) + ii) * ea.ldc + cofs + 32 * (u & 3)) = pk;
      unpack8(pk, r);
#pragma unroll
      for (int e = 0; e < 8; ++e) part = __builtin_fmaf(r[e], o[e], part);
      if ((u & 3) == 3) {  // the row's 4 column pairs done: sum over the 4 lanes holding it
        part += __shfl_xor(part, 16, 64);
        part += __shfl_xor(part, 32, 64);
        if (g == 0) ea.Dl[(long)(col0 >> 7) * ea.dM + row0 + 16 * (u >> 2) + ii] = part;
        part = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long row = row0 + 16 * i + ii;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float v[8];
        gather8(acc, i, p, v);
        if (nrm != nullptr) {
#pragma unroll
          for (int e = 0; e < 8; ++e) ss += v[e] * v[e];
        }
        *(uint4*)(ea.C + row * ea.ldc + cofs + 32 * p) = pack8(v);
      }
    }
  }
  if (nrm != nullptr) {  // 8 slots per tile (the 8-wave kernels' layout): waves 0..3 write theirs and zero w + 4, so
    ss = wave_sum(ss);    // slots parked in an uninitialised split-K buffer (hybrid launches) are never garbage
    if (lane == 0) {
      nrm[0] = ss;
      nrm[4] = 0.f;
    }
  }
}

// split piece: fp32 wave tile -> the piece's tile-local slab P[256][256]
__device__ __forceinline__ void store_partial(const f32x4 (&acc)[8][8], float* __restrict__ P, int wm, int wn, int lane) {
  const int g = lane >> 4, ii = lane & 15;
  const int c = 128 * wn + 16 * (g & 1) + 8 * (g >> 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float* row = P + (long)(128 * wm + 16 * i + ii) * 256 + c;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v[8];
      gather8(acc, i, p, v);
      *(float4*)(row + 32 * p) = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(row + 32 * p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// One 32-deep step on F(u) = (fa, fb): MFMAs, and one memory op per MFMA gap after the barrier — the 16 reads of
// F(u + 1) from `nxt` into (ra, rb) and the 8 LDS-DMA pieces of step u + 4 into `cur` (op k after MFMA 8 + 7k/3, in the
// order B0 B1 D0 B2 B3 D1 .. A6 A7 D7).
template <int LA, int LB>
__device__ __forceinline__ void rstep(f32x4 (&acc)[8][8], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8],
                                      bf16x8 (&ra)[8], bf16x8 (&rb)[8], const char* __restrict__ nxt,
                                      char* __restrict__ cur, Op32<LA>& oa, Op32<LB>& ob, int w) {
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(16, 15));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mfma(acc[i][j], fb[j], fa[i]);
      if (i == 0 && j == 7) {  // this wave's reads of the slot the DMA below overwrites have retired
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(63, 0));
        __builtin_amdgcn_s_barrier();
      }
      const int n = 8 * i + j;
      const int k = n < 8 ? -1 : ((n - 8) * 3 + 6) / 7;  // the op placed after MFMA n, if any
      if (k < 0 || k >= 24 || 8 + (k * 7) / 3 != n) continue;
      const int t = k / 3, r = k % 3;
      if (r < 2) {
        const int f = 2 * t + r;
        if (f < 8) rb[f] = ob.frag(nxt + OPB32, f);
        else ra[f - 8] = oa.frag(nxt, f - 8);
      } else if (t < 4) {
        oa.piece(cur, w, t);
      } else {
        ob.piece(cur + OPB32, w, t - 4);
      }
    }
  }
  oa.advance();
  ob.advance();
}

// nb blocks of four steps (u = 4 b .. 4 b + 3 on slots S0..S3), ONE loop body for every block, the last included: its
// DMA re-reads the final step (the offsets saturate, Op32::limit) into slots nobody reads again, and its reads of
// "step 4 nb" are never used. No MFMA code after the loop, so the register allocator has no loop-exit block in which
// to move accumulators between AGPRs and VGPRs right behind an asm MFMA it cannot see the latency of (it did, in a
// separately compiled last body: wrong sums, profiles/r6_g4_interleave.md).
template <int LA, int LB>
__device__ __forceinline__ void mainloop(char* __restrict__ S0, char* __restrict__ S1, char* __restrict__ S2,
                                         char* __restrict__ S3, int nb, Op32<LA>& oa, Op32<LB>& ob, int w,
                                         f32x4 (&acc)[8][8]) {
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  auto issue = [&](char* __restrict__ s) {
#pragma unroll
    for (int j = 0; j < 4; ++j) oa.piece(s, w, j);
#pragma unroll
    for (int j = 0; j < 4; ++j) ob.piece(s + OPB32, w, j);
    oa.advance();
    ob.advance();
  };
  issue(S0);
  issue(S1);
  issue(S2);
  issue(S3);
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(24, 15));  // step 0 landed (steps 1..3 may fly)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) b0[i] = ob.frag(S0 + OPB32, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = oa.frag(S0, i);
  for (int b = 0; b < nb; ++b) {
    rstep<LA, LB>(acc, a0, b0, a1, b1, S1, S0, oa, ob, w);
    rstep<LA, LB>(acc, a1, b1, a0, b0, S2, S1, oa, ob, w);
    rstep<LA, LB>(acc, a0, b0, a1, b1, S3, S2, oa, ob, w);
    rstep<LA, LB>(acc, a1, b1, a0, b0, S0, S3, oa, ob, w);
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));  // the LDS-DMA past the end lands before the LDS is released
}

__device__ __forceinline__ void tile_origin(int tile, int nbm, int nbn, int group, int& m0, int& n0) {
  const int per_group = group * nbn;
  const int grp = tile / per_group, first = grp * group;
  const int gsz = min(nbm - first, group);
  const int in = tile - grp * per_group;
  m0 = (first + in % gsz) * 256;
  n0 = (in / gsz) * 256;
}

// One GEMM of a launch: operands, tile grid (nbm x nbn tiles of 256 x 256, GROUP-blocked order), epilogue; park =
// where this problem's whole tiles put their norm partials past P (a split launch's slabs), 0 = straight into P.
struct Prob {
  const u16* A;
  const u16* B;
  long lda, ldb;
  int nbm, nbn, group;
  long park;
  Epi ea;
};

// Up to four problems of one launch: problem i owns tiles [s_i, s_{i+1}) (s_0 = 0; unused starts = INT_MAX).
struct Probs {
  Prob q0, q1, q2, q3;
  int s1, s2, s3;
};

// A launch runs one to four problems with the same reduction length (e.g. the MLP's down and gate_up weight
// gradients as ONE grid: 344 + 688 = 1032 tiles = 4.03 rounds of 256 CUs instead of 1.34 + 2.69 — a partial last round
// costs most of a full one, profiles/r6_gemm_routing.md; with the next layer's o_proj + qkv: 1192 tiles = 4 rounds +
// 168 split tiles). splits > 1: the tiles past ndp are split into `splits` equal ranges of 128-deep blocks (pieces ->
// fp32 slabs of their problem's P, splitk_fixup_kernel per problem).
template <int LA, int LB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
g4_kernel(Probs ps, int kred, int ndp, int splits) {
  __shared__ __attribute__((aligned(16))) char smem[4 * SLOT32];
  // Blocks [0, ndp) own whole tiles, XCD-aware bijective remap among them (consecutive ids on one XCD: shared L2 for
  // the GROUP-blocked tile order); blocks >= ndp are the split pieces. Classes by BLOCK index, not by remapped id:
  // dispatch follows block order, so the whole tiles fill the first rounds and the short pieces the last one (a
  // remap over the whole grid put half of each round's blocks on pieces and stretched the whole tiles to 2 rounds).
  const int orig = blockIdx.x;
  int wgid = orig;
  if (orig < ndp) {
    const int xcd = orig & 7, q8 = ndp >> 3, r8 = ndp & 7;
    wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  }
  const int nb_all = kred / (4 * BK32);
  int tile = wgid, sk = 0, p0 = 0, p1 = nb_all;
  if (wgid >= ndp) {  // split piece sk of tile ndp + (wgid - ndp) / splits: blocks [p0, p1)
    const int j = wgid - ndp;
    sk = j % splits;
    tile = ndp + j / splits;
    p0 = (int)((long)sk * nb_all / splits);
    p1 = (int)((long)(sk + 1) * nb_all / splits);
  }
  // the problem this tile belongs to (wave-uniform selects of kernel arguments, no indexed copy of the struct)
  const int pi = (tile >= ps.s1) + (tile >= ps.s2) + (tile >= ps.s3);
#define G4SEL(f) (pi == 0 ? ps.q0.f : pi == 1 ? ps.q1.f : pi == 2 ? ps.q2.f : ps.q3.f)
  const int start = pi == 0 ? 0 : pi == 1 ? ps.s1 : pi == 2 ? ps.s2 : ps.s3;
  const int lt = tile - start;
  const u16* A = G4SEL(A);
  const u16* B = G4SEL(B);
  const long lda = G4SEL(lda), ldb = G4SEL(ldb), park = G4SEL(park);
  Epi ea;
  ea.C = G4SEL(ea.C);
  ea.P = G4SEL(ea.P);
  ea.ldc = G4SEL(ea.ldc);
  ea.flags = G4SEL(ea.flags);
  ea.O = G4SEL(ea.O);
  ea.Dl = G4SEL(ea.Dl);
  ea.ldO = G4SEL(ea.ldO);
  ea.dM = G4SEL(ea.dM);
  int m0, n0;
  tile_origin(lt, G4SEL(nbm), G4SEL(nbn), G4SEL(group), m0, n0);
#undef G4SEL
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const long k0 = (long)p0 * 4 * BK32;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  Op32<LA> oa;
  Op32<LB> ob;
  oa.init(A, lda, m0, k0, w, lane, wm);
  ob.init(B, ldb, n0, k0, w, lane, wn);
  oa.limit(4 * (p1 - p0));
  ob.limit(4 * (p1 - p0));
  mainloop<LA, LB>(smem, smem + SLOT32, smem + 2 * SLOT32, smem + 3 * SLOT32, p1 - p0, oa, ob, w, acc);
  // the epilogue's accumulator reads follow the last MFMAs: 20 wait states + a fence against hoisting
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (wgid >= ndp) {
    // slab of this problem's piece: its split tiles start at its first tile past ndp
    const int ndpl = max(ndp - start, 0);
    store_partial(acc, ea.P + ((long)(lt - ndpl) * splits + sk) * 65536, wm, wn, lane);
    return;
  }
  float* nrm = nullptr;
  if (ea.flags & 2)  // whole tiles of a split problem park theirs past the slabs (park > 0)
    nrm = ea.P + park + lt * 8 + w;
  store_tile(acc, ea, m0 + 128 * wm, n0 + 128 * wn, lane, nrm);
}

static int group_m() { return 8; }  // GROUP_M tile order

static Prob prob(const u16* A, long lda, const u16* B, long ldb, int M, int N, const Epi& ea, long park) {
  Prob p;
  p.A = A;
  p.B = B;
  p.lda = lda;
  p.ldb = ldb;
  p.nbm = M / 256;
  p.nbn = N / 256;
  p.group = std::min(group_m(), p.nbm);
  p.park = park;
  p.ea = ea;
  return p;
}

template <int LA, int LB>
static void launchn(const Probs& ps, int total, int kred, int ndp, int splits) {
  const int grid = ndp + (total - ndp) * splits;
  g4_kernel<LA, LB><<<grid, 256, 0, cur_stream()>>>(ps, kred, ndp, splits);
  SFT_LAUNCH_CHECK();
}

template <int LA, int LB>
static void launch2(const Prob& q0, const Prob& q1, int tiles0, int total, int kred, int ndp, int splits) {
  launchn<LA, LB>(Probs{q0, q1, q1, q1, tiles0, INT_MAX, INT_MAX}, total, kred, ndp, splits);
}

template <int LA, int LB>
static void launch(const u16* A, long lda, const u16* B, long ldb, int M, int N, int kred, int ndp, int splits,
                   const Epi& ea) {
  const int tiles = (M / 256) * (N / 256);
  const long park = splits > 1 ? (long)(tiles - ndp) * splits * 65536 : 0;
  const Prob q = prob(A, lda, B, ldb, M, N, ea, park);
  launch2<LA, LB>(q, q, tiles, tiles, kred, ndp, splits);
}

}  // namespace g4

// Weight gradient out[N, K] (+)= dy[T, N]^T x[T, K] on the 4-wave kernel. splits > 1: the tiles past the last whole
// round of 256 workgroups (hybrid) or all tiles are split over the token axis into fp32 slabs + ordered fixup.
// nrm: gradient-norm slots (8 per whole tile, waves 0..3 written; one per fixup block of a split tile).
void g4_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor& out, bool accumulate, int splits, bool hybrid,
              float* nrm, long nrm_cap) {
  const int T = dy.size(0), N = dy.size(1), K = x.size(1);
  SFT_CHECK(N % 256 == 0 && K % 256 == 0 && T % 128 == 0 && T > 0, "wgrad 4-wave: N, K % 256, T % 128");
  SFT_CHECK((uintptr_t)dy.data_ptr() % 16 == 0 && (uintptr_t)x.data_ptr() % 16 == 0 &&
                (uintptr_t)out.data_ptr() % 16 == 0, "wgrad 4-wave: 16-byte aligned operands");
  const int tiles = (N / 256) * (K / 256);
  if (splits < 1) splits = 1;
  splits = std::min(splits, T / 128);
  const int B = cu_budget();  // one round = B workgroups (csrc/cu_budget.h)
  const int ndp = splits <= 1 ? tiles : (hybrid ? tiles / B * B : 0);
  const int nsk = tiles - ndp;
  const long slots = (long)ndp * 8 + (long)nsk * 32;
  SFT_CHECK(nrm == nullptr || slots <= nrm_cap, "wgrad_gemm: norm slot buffer too small");
  at::Tensor part;
  if (nsk > 0)
    part = at::empty({(long)nsk * splits * 65536 + (nrm != nullptr ? (long)ndp * 8 : 0)}, dy.options().dtype(at::kFloat));
  g4::Epi ea{};
  ea.C = (u16*)out.data_ptr();
  ea.ldc = K;
  ea.P = nsk > 0 ? part.data_ptr<float>() : nrm;
  ea.flags = (accumulate ? 1 : 0) | (nrm != nullptr ? 2 : 0);
  g4::launch<g4::TR, g4::TR>((const u16*)dy.data_ptr(), N, (const u16*)x.data_ptr(), x.stride(0), N, K, T, ndp,
                             nsk > 0 ? splits : 1, ea);
  if (nsk > 0) {
    const long n8 = (long)nsk * 65536 / 8;
    splitk_fixup_kernel<256, 256><<<(unsigned)((n8 + 255) / 256), 256, 0, cur_stream()>>>(
        part.data_ptr<float>(), (u16*)out.data_ptr(), ndp, nsk, splits, K / 256, K, accumulate ? 1 : 0, nrm, N / 256,
        std::min(g4::group_m(), N / 256));
    SFT_LAUNCH_CHECK();
  }
}

// Up to four weight gradients over the same tokens as ONE grid (g4_kernel with several problems): out_i (+)= dy_i^T
// x_i. The whole rounds of B (cu_budget) tiles run across the problems in order; the partial last round (the tiles past
// them, which may span several problems: put the small ones last) is split over the tokens into fp32 slabs + the
// ordered fixup of each problem that has split tiles, split_left ways (0: min(8, B / leftover), the hybrid rule).
// split_all > 1: every tile split that many ways (small groups such as o_proj + qkv: 64 + 96 tiles x 3 = 480 pieces =
// 2 rounds of third-tiles, against one round of quarter-tiles + one of half-tiles apart).
void g4_wgrad_multi(const std::vector<WgradJob>& jobs, int split_all, int split_left) {
  const int np = (int)jobs.size();
  SFT_CHECK(np >= 1 && np <= 4, "wgrad multi: 1..4 problems");
  const int T = jobs[0].dy.size(0);
  int tiles[4] = {0, 0, 0, 0}, start[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < np; ++i) {
    const WgradJob& j = jobs[i];
    const int N = j.dy.size(1), K = j.x.size(1);
    SFT_CHECK(j.dy.size(0) == T && j.x.size(0) == T, "wgrad multi: the same tokens");
    SFT_CHECK(N % 256 == 0 && K % 256 == 0 && T % 128 == 0 && T > 0, "wgrad multi: N, K % 256, T % 128");
    SFT_CHECK((uintptr_t)j.dy.data_ptr() % 16 == 0 && (uintptr_t)j.x.data_ptr() % 16 == 0 &&
                  (uintptr_t)j.out.data_ptr() % 16 == 0,
              "wgrad multi: 16-byte aligned operands");
    tiles[i] = (N / 256) * (K / 256);
    start[i + 1] = start[i] + tiles[i];
  }
  const int total = start[np];
  const int B = cu_budget();
  int ndp = total / B * B, splits = 1;
  if (split_all > 1) {
    ndp = 0;
    splits = std::min(split_all, T / 128);
  } else if (total > ndp) {
    splits = split_left > 0 ? split_left : std::min(8, B / (total - ndp));
    splits = std::min(splits, T / 128);
  }
  if (splits < 2) {
    splits = 1;
    ndp = total;
  }
  // per problem: whole tiles [0, w) and split tiles [w, tiles)
  int w[4], sn[4];
  at::Tensor part[4];
  g4::Prob q[4];
  for (int i = 0; i < np; ++i) {
    const WgradJob& j = jobs[i];
    w[i] = std::min(std::max(ndp - start[i], 0), tiles[i]);
    sn[i] = tiles[i] - w[i];
    SFT_CHECK(j.nrm == nullptr || (long)w[i] * 8 + (long)sn[i] * 32 <= j.cap, "wgrad multi: norm slot buffer too small");
    if (sn[i] > 0)
      part[i] = at::empty({(long)sn[i] * splits * 65536 + (j.nrm != nullptr ? (long)w[i] * 8 : 0)},
                          j.dy.options().dtype(at::kFloat));
    const int N = j.dy.size(1), K = j.x.size(1);
    g4::Epi e{};
    e.C = (u16*)j.out.data_ptr();
    e.ldc = K;
    e.P = sn[i] > 0 ? part[i].data_ptr<float>() : j.nrm;
    e.flags = (j.acc ? 1 : 0) | (j.nrm != nullptr ? 2 : 0);
    q[i] = g4::prob((const u16*)j.dy.data_ptr(), N, (const u16*)j.x.data_ptr(), j.x.stride(0), N, K, e,
                sn[i] > 0 ? (long)sn[i] * splits * 65536 : 0);
  }
  for (int i = np; i < 4; ++i) q[i] = q[np - 1];
  g4::launchn<g4::TR, g4::TR>(g4::Probs{q[0], q[1], q[2], q[3], np > 1 ? start[1] : INT_MAX, np > 2 ? start[2] : INT_MAX,
                        np > 3 ? start[3] : INT_MAX},
                  total, T, ndp, splits);
  // the fixups of every problem with split tiles as one grid (32 blocks of 256 x 8 elements per tile)
  FixArgs fa[4];
  int nf = 0, bstart[4] = {0, 0, 0, 0}, nblocks = 0;
  for (int i = 0; i < np; ++i) {
    if (sn[i] <= 0) continue;
    const WgradJob& j = jobs[i];
    const int N = j.dy.size(1), K = j.x.size(1);
    fa[nf] = FixArgs{part[i].data_ptr<float>(), (u16*)j.out.data_ptr(), j.nrm, w[i], sn[i], K / 256, K,
                     j.acc ? 1 : 0, N / 256, std::min(g4::group_m(), N / 256)};
    bstart[nf++] = nblocks;
    nblocks += sn[i] * 32;
  }
  if (nf == 0) return;
  for (int i = nf; i < 4; ++i) fa[i] = fa[nf - 1];
  splitk_fixup_multi_kernel<256, 256><<<(unsigned)nblocks, 256, 0, cur_stream()>>>(
      fa[0], fa[1], fa[2], fa[3], nf > 1 ? bstart[1] : INT_MAX, nf > 2 ? bstart[2] : INT_MAX,
      nf > 3 ? bstart[3] : INT_MAX, splits);
  SFT_LAUNCH_CHECK();
}

// Two weight gradients as one grid (g4_wgrad_multi); without split_all the partial round must fall in problem 1.
void g4_wgrad_pair(const at::Tensor& dy0, const at::Tensor& x0, at::Tensor& out0, bool acc0, float* nrm0, long cap0,
                   const at::Tensor& dy1, const at::Tensor& x1, at::Tensor& out1, bool acc1, float* nrm1, long cap1,
                   int split_all) {
  const int tiles0 = (dy0.size(1) / 256) * (x0.size(1) / 256), tiles1 = (dy1.size(1) / 256) * (x1.size(1) / 256);
  const int B = cu_budget(), total = tiles0 + tiles1;
  SFT_CHECK(split_all > 1 || total - total / B * B <= tiles1, "wgrad pair: the partial round must fall in the second problem");
  g4_wgrad_multi({WgradJob{dy0, x0, out0, acc0, nrm0, cap0}, WgradJob{dy1, x1, out1, acc1, nrm1, cap1}}, split_all, 0);
}

// Input gradient dX[M, N] = dy[M, K] . w[K, N] into out (row stride ldo; w may be a column slice: row stride
// w.stride(0)). Wave quantisation: a grid that is not whole rounds of 256 workgroups runs its whole rounds as whole
// tiles and, for long reductions, the leftover tiles split over the reduction into fp32 slabs + the ordered fixup, e.g.
// the recipe's padding-free M = 10240: gate_up / lm_head dgrads are 40 x 8 = 320 tiles = 1.25 rounds -> 256 + 64 x 4
// pieces.
// attn_out / delta (optional): the attention output O [M, N] (row stride ld_attn) and delta [N / 128][M] fp32 =
// per-head rowsum(bf16(dX) . O), fused into the epilogue (flags bit 2; whole tiles only: no split-K).
void g4_dgrad(const at::Tensor& dy, const at::Tensor& w, u16* out, long ldo, const u16* attn_out, long ld_attn,
              float* delta) {
  const int M = dy.size(0), K = dy.size(1), N = w.size(1);
  SFT_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && K > 0, "dgrad 4-wave: M, N % 256, K % 128");
  g4::Epi ea{};
  ea.C = out;
  ea.ldc = ldo;
  if (delta != nullptr) {
    SFT_CHECK(attn_out != nullptr && ld_attn % 8 == 0 && (uintptr_t)attn_out % 16 == 0,
              "dgrad 4-wave delta: 16-byte aligned attention output rows");
    SFT_CHECK(K < 8192 || (M / 256) * (N / 256) % 256 == 0, "dgrad 4-wave delta: whole tiles only (no split-K)");
    // (and no budget split below: the delta epilogue needs whole tiles)
    ea.flags = 4;
    ea.O = attn_out;
    ea.Dl = delta;
    ea.ldO = ld_attn;
    ea.dM = M;
  }
  const int nbm = M / 256, nbn = N / 256, tiles = nbm * nbn;
  int ndp = tiles, splits = 1;
  // one round = B workgroups (csrc/cu_budget.h). Short reductions split their leftover round only under a reduced
  // budget (B < 256: the leftover tiles would otherwise wait a whole tile time on the CUs other work holds); with the
  // whole chip the fixup costs more than the partial round
  const int B = cu_budget();
  if (delta == nullptr && tiles % B != 0 && (K >= 8192 || (B < num_cus() && tiles > B))) {
    const int rest = tiles > B ? tiles % B : tiles;
    const int s = std::min(std::min(B / rest, 8), K / 128);
    if (s >= 2) {
      ndp = tiles - rest;
      splits = s;
    }
  }
  at::Tensor part;
  if (splits > 1) {
    part = at::empty({(long)(tiles - ndp) * splits * 65536}, dy.options().dtype(at::kFloat));
    ea.P = part.data_ptr<float>();
  }
  g4::launch<g4::ROW, g4::TR>((const u16*)dy.data_ptr(), dy.stride(0), (const u16*)w.data_ptr(), w.stride(0), M, N,
                              K, ndp, splits, ea);
  if (splits > 1) {
    SFT_TRACE("dgrad.splitk");
    const int nsk = tiles - ndp;
    const long n8 = (long)nsk * 65536 / 8;
    splitk_fixup_kernel<256, 256><<<(unsigned)((n8 + 255) / 256), 256, 0, cur_stream()>>>(
        part.data_ptr<float>(), out, ndp, nsk, splits, nbn, (int)ldo, 0, nullptr, nbm, std::min(g4::group_m(), nbm));
    SFT_LAUNCH_CHECK();
  }
}

}  // namespace sftamd
