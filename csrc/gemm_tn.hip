// Forward-layout GEMM for gfx950 with fused epilogues: C[M, N] = A[M, K] . B[N, K]^T, bf16 in, fp32
// accumulate (the projection forward y = x W^T: both operands K-contiguous, "TN" in BLAS terms).
//
// Why a hand-written kernel next to hipBLASLt: the elementwise op that follows each projection can
// ride in the epilogue instead of re-reading the GEMM output from HBM:
//   EPI_SWIGLU  gate_up projection: writes gu = [gate | up] (saved for backward) AND act = silu(gate)*up
//               (the down projection's input) — the separate SwiGLU kernel's 540 MB/layer re-read is gone;
//   EPI_ROPE    qkv projection: rotary embedding of the q and k heads applied before the store.
// The pairing trick: the B tile's LDS image is filled from permuted WEIGHT ROWS (no weight copy —
// the stager just points its pieces at other rows) so that MFMA fragments j = 2q and 2q + 1 of a
// wave hold the two columns the epilogue must combine: (gate c, up c) for SwiGLU, (d, d + 64) of a
// head for RoPE (rotate_half). Weights keep their HF layout ([gate; up], [q; k; v]).
//
// Main loop = the ring structure of gemm_wgrad.hip (measured there): 256 x 256 (or 256 x 128) tile
// per 512-thread workgroup (8 waves, 2x4 / 4x2), BK = 32 per stage, NS stages of global_load_lds
// in flight (up to all 160 KB of LDS), counted vmcnt + raw s_barrier (one per stage), next-stage
// fragments read during the current stage's MFMAs, LDS-DMA pieces interleaved with MFMA rows.
// Operands are K-contiguous, so fragments are plain 16-byte ds_read_b128 rows (no transposed read):
// LDS image rows are 64 B (32 bf16 of k) with a chunk swizzle (swz below) applied on the GLOBAL
// source address (glds writes lane-linear) that makes every ds_read_b128 lane group conflict-free.
// Tile order: XCD-aware bijective remap, then GROUP_M-blocked (8 M-tiles per group) so the ~32
// tiles an XCD runs at once share A and B slabs in its L2.
#include "common.h"

namespace sftamd {
namespace tn {

constexpr int NT = 512;
constexpr int BK = 32;     // k per stage
constexpr int ROWB = 64;   // bytes per LDS image row
static int group_m() { return 8; }  // GROUP_M tile order: 8 row blocks share each weight panel

enum { EPI_PLAIN = 0, EPI_SWIGLU = 1, EPI_ROPE = 2 };

// ds_read_b128 is serviced in four NON-contiguous 16-lane groups (/opt/skills/guides/MI355X_MICROARCH.md §LDS:
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...). A fragment read has lane (g = lane>>4, ii = lane&15) at
// image row R + ii, chunk g: its 16-B slot in the 256-B bank row is 4 (ii & 3) + (g ^ S(ii >> 2)).
// S = {0, 2, 3, 1} makes the 16 slots of every group distinct (the plain S(q) = q is 2-way).
__device__ __forceinline__ int swz_sel(int q) { return (0x78 >> (2 * q)) & 3; }
__device__ __forceinline__ int swz(int row, int ch) { return ch ^ swz_sel((row >> 2) & 3); }

__device__ __forceinline__ void glds16(const u16* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_row(const char* base, int off) { return *(const bf16x8*)(base + off); }

constexpr unsigned waitcnt_imm(int vm, int lgkm) {  // gfx9: vmcnt[3:0] expcnt[6:4] lgkmcnt[11:8] vmcnt[5:4]<<14
  return (unsigned)((vm & 15) | (7 << 4) | ((lgkm & 15) << 8) | ((vm >> 4) << 14));
}

template <int BM, int BN, int WM, int WN, int NS_>
struct Cfg {
  static constexpr int NS = NS_;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int APIECES = BM / 16, PIECES = (BM + BN) / 16;  // 1 KB = 16 image rows per piece
  static constexpr int PPW = PIECES / 8;
  static constexpr int STAGE = (BM + BN) * ROWB;
  static constexpr int EPI_ROWS = 64, EPI_LD = TN + 4;
  static constexpr int EPI = 8 * EPI_ROWS * EPI_LD * 4;
  static constexpr int LDS = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  static_assert(WM * WN == 8 && PIECES % 8 == 0 && FM >= PPW, "config");
  static_assert(TN == 64, "epilogue pairing assumes 64-column wave tiles");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// Global row of the B operand that lands in LDS image rows [16 pb, 16 pb + 16) of a tile.
template <int EPI, int BN>
__device__ __forceinline__ int b_piece_row(int pb, int n0, int I) {
  if constexpr (EPI == EPI_SWIGLU) {
    // image rows 32q + 16h + r <- gate (h=0) / up (h=1) row c0 + 16q + r; c0 = n0 / 2 (act columns)
    return (pb & 1) * I + (n0 >> 1) + 16 * (pb >> 1);
  } else if constexpr (EPI == EPI_ROPE) {
    // per 128-row head: image rows 32q + 16h + r <- head dim d = 16q + 64h + r
    const int head = pb >> 3, u = pb & 7;
    return n0 + 128 * head + 16 * (u >> 1) + 64 * (u & 1);
  } else {
    return n0 + 16 * pb;
  }
}

// Piece j of wave w is global piece P = w + 8 j (A pieces first). Every piece of a wave is a fixed
// number of rows away from the wave's first A / first B piece (also for the permuted B rows of the
// SWIGLU / ROPE tiles), so the stager keeps two lane pointers and compile-time row strides.
template <int EPI>
constexpr int b_piece_stride() { return EPI == EPI_SWIGLU ? 64 : 128; }  // rows between B pieces w + 8k

template <class G, int EPI>
struct Stager {
  static constexpr int JA = G::APIECES / 8;  // pieces j < JA are A pieces
  const u16* pa;
  const u16* pb;
  long lda, ldb;
  int left;
  __device__ __forceinline__ void piece(char* buf, int w, int j) {
    const u16* src = j < JA ? pa + (long)(128 * j) * lda : pb + (long)(b_piece_stride<EPI>() * (j - JA)) * ldb;
    glds16(src, buf + (w + 8 * j) * 1024);  // image = A rows then B rows, 1 KB (16 rows) per piece
  }
  __device__ __forceinline__ void advance() {
    if (--left > 0) {
      pa += BK;
      pb += BK;
    }
  }
  __device__ __forceinline__ void issue(char* buf, int w) {
#pragma unroll
    for (int j = 0; j < G::PPW; ++j) piece(buf, w, j);
    advance();
  }
};

__device__ __forceinline__ char* pick(int i, char* b0, char* b1, char* b2, char* b3, char* b4, char* b5) {
  switch (i) {
    case 0: return b0;
    case 1: return b1;
    case 2: return b2;
    case 3: return b3;
    case 4: return b4;
    default: return b5;
  }
}

template <class G, int EPI>
__device__ __forceinline__ void ring_loop(char* __restrict__ b0, char* __restrict__ b1, char* __restrict__ b2,
                                          char* __restrict__ b3, char* __restrict__ b4, char* __restrict__ b5,
                                          int nsteps, Stager<G, EPI>& st, int w, int offA, int offB,
                                          f32x4 (&acc)[G::FM][G::FN]) {
  constexpr int NS = G::NS, PPW = G::PPW;
  constexpr int U = (NS % 2) ? 2 * NS : NS;  // stage slot and B register set both compile-time
  bf16x8 fa[G::FM], fb[2][G::FN];
#pragma unroll
  for (int i = 0; i < NS; ++i) st.issue(pick(i, b0, b1, b2, b3, b4, b5), w);
  __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 1) * PPW, 0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < G::FN; ++j) fb[0][j] = lds_row(b0, offB + 1024 * j);
#pragma unroll
  for (int i = 0; i < G::FM; ++i) fa[i] = lds_row(b0, offA + 1024 * i);
  for (int t0 = 0; t0 < nsteps; t0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t0 + u < nsteps) {
        __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 2) * PPW, 0));
        __builtin_amdgcn_s_barrier();
        char* dst = pick(u % NS, b0, b1, b2, b3, b4, b5);
        const char* nxt = pick((u + 1) % NS, b0, b1, b2, b3, b4, b5);
        const int cb = u & 1;
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb[cb ^ 1][j] = lds_row(nxt, offB + 1024 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[cb][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_row(nxt, offA + 1024 * i);
          if (i < PPW) st.piece(dst, w, i);
          __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);      // DS read (one fragment)
          if (i < PPW) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (the DMA)
        }
        st.advance();
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));  // drain the tail DMAs before LDS is reused
}

struct EpiArgs {
  u16* C;        // PLAIN / ROPE: C[M, ldc];  SWIGLU: gu[M, 2I]
  u16* act;      // SWIGLU: act[M, I]
  const float* cosb;  // ROPE: [M, 64] fp32
  const float* sinb;
  long ldc;
  int I;          // SWIGLU: intermediate size
  int rope_cols;  // ROPE: columns [0, rope_cols) are rotated (q and k heads)
};

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }
__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

// fp32 wave tile -> wave-private LDS rows (TN + 4 floats, conflict-free) -> 16-byte stores.
template <class G, int EPI>
__device__ __forceinline__ void epilogue(char* smem, f32x4 (&acc)[G::FM][G::FN], const EpiArgs& ea, int m0, int n0,
                                         int wm, int wn, int w, int lane) {
  const int g = lane >> 4, ii = lane & 15;
  float* ep = reinterpret_cast<float*>(smem) + w * G::EPI_ROWS * G::EPI_LD;
  constexpr int FPP = G::EPI_ROWS / 16 < G::FM ? G::EPI_ROWS / 16 : G::FM;  // fragment rows per pass
  constexpr int ROWS = FPP * 16;
#pragma unroll
  for (int pass = 0; pass < G::FM / FPP; ++pass) {
#pragma unroll
    for (int i = 0; i < FPP; ++i)
#pragma unroll
      for (int j = 0; j < G::FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) ep[(16 * i + 4 * g + e) * G::EPI_LD + 16 * j + ii] = acc[pass * FPP + i][j][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region: writes before reads
    const int rbase = m0 + wm * G::TM + pass * ROWS;
    if constexpr (EPI == EPI_PLAIN) {
      constexpr int SEGS = G::TN / 8;
#pragma unroll
      for (int it = 0; it < ROWS * SEGS / 64; ++it) {
        const int seg = it * 64 + lane, row = seg / SEGS, cs = seg - row * SEGS;
        const float* pr = ep + row * G::EPI_LD + cs * 8;
        float v[8];
        *(float4*)&v[0] = *(const float4*)pr;
        *(float4*)&v[4] = *(const float4*)(pr + 4);
        *(uint4*)(ea.C + (long)(rbase + row) * ea.ldc + n0 + wn * G::TN + cs * 8) = pack8(v);
      }
    } else {
      // unit = (row, pair p, half): segment a = cols 32p + 8h (fragment 2p), b = cols 32p + 16 + 8h (2p + 1)
      constexpr int UPR = G::TN / 16;  // units per row
#pragma unroll
      for (int it = 0; it < ROWS * UPR / 64; ++it) {
        const int un = it * 64 + lane, row = un / UPR, r = un - row * UPR, p = r >> 1, hh = r & 1;
        const float* pa = ep + row * G::EPI_LD + 32 * p + 8 * hh;
        float a[8], b[8];
        *(float4*)&a[0] = *(const float4*)pa;
        *(float4*)&a[4] = *(const float4*)(pa + 4);
        *(float4*)&b[0] = *(const float4*)(pa + 16);
        *(float4*)&b[4] = *(const float4*)(pa + 20);
        const long grow = rbase + row;
        const int t = wn * G::TN + 32 * p + 8 * hh;  // image column of segment a
        if constexpr (EPI == EPI_SWIGLU) {
          const int c = (n0 >> 1) + 16 * (t >> 5) + 8 * hh;  // act column
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            a[e] = rbf(a[e]);  // act from the bf16 gate/up the backward will see
            b[e] = rbf(b[e]);
            o[e] = silu(a[e]) * b[e];
          }
          u16* gp = ea.C + grow * ea.ldc + c;
          *(uint4*)gp = pack8(a);
          *(uint4*)(gp + ea.I) = pack8(b);
          *(uint4*)(ea.act + grow * ea.I + c) = pack8(o);
        } else {  // ROPE
          const int head = t >> 7, u = t & 127, d = 16 * (u >> 5) + 8 * hh;
          const int col = n0 + 128 * head + d;
          u16* op = ea.C + grow * ea.ldc + col;
          if (col < ea.rope_cols) {
            float cs[8], sn[8], lo[8], hi[8];
            const float* cp = ea.cosb + grow * 64 + d;
            const float* sp = ea.sinb + grow * 64 + d;
            *(float4*)&cs[0] = *(const float4*)cp;
            *(float4*)&cs[4] = *(const float4*)(cp + 4);
            *(float4*)&sn[0] = *(const float4*)sp;
            *(float4*)&sn[4] = *(const float4*)(sp + 4);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x1 = rbf(a[e]), x2 = rbf(b[e]);  // rope of the bf16 projection (unfused twin)
              lo[e] = x1 * cs[e] - x2 * sn[e];
              hi[e] = x2 * cs[e] + x1 * sn[e];
            }
            *(uint4*)op = pack8(lo);
            *(uint4*)(op + 64) = pack8(hi);
          } else {
            *(uint4*)op = pack8(a);
            *(uint4*)(op + 64) = pack8(b);
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

template <int BM, int BN, int WM, int WN, int NS, int EPI>
__global__ void __launch_bounds__(NT) tn_kernel(const u16* __restrict__ A, const u16* __restrict__ B, int K, long lda,
                                                long ldb, int nbm, int nbn, int group, EpiArgs ea) {
  using G = Cfg<BM, BN, WM, WN, NS>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  // XCD-aware bijective remap (consecutive ids share an XCD), then GROUP_M-blocked tile order
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_group = group * nbn;
  const int grp = wgid / per_group, first = grp * group;
  const int gsz = min(nbm - first, group);
  const int in = wgid - grp * per_group;
  const int bm = first + in % gsz, bn = in / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w - wm * WN;

  Stager<G, EPI> st;
  st.lda = lda;
  st.ldb = ldb;
  st.left = K / BK;
  {
    const int lr = lane >> 2, ch = swz(lr, lane & 3);  // row in piece, pre-swizzled chunk
    st.pa = A + (long)(m0 + 16 * w + lr) * lda + 8 * ch;
    st.pb = B + (long)(b_piece_row<EPI, BN>(w, n0, ea.I) + lr) * ldb + 8 * ch;
  }
  // fragment rows 16 i + ii all share the swizzle of ii (bits 2-3 of the row): fragment i of a wave
  // is 1 KB after fragment i - 1, an immediate offset of the ds_read
  const int g = lane >> 4, ii = lane & 15;
  const int offA = (wm * G::TM + ii) * ROWB + 16 * swz(ii, g);
  const int offB = (BM + wn * G::TN + ii) * ROWB + 16 * swz(ii, g);
  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* b[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) b[i] = smem + (i < NS ? i : 0) * G::STAGE;
  ring_loop<G, EPI>(b[0], b[1], b[2], b[3], b[4], b[5], K / BK, st, w, offA, offB, acc);
  __syncthreads();
  epilogue<G, EPI>(smem, acc, ea, m0, n0, wm, wn, w, lane);
}

// ============================================================================================
// BK = 64 variant: 128-byte LDS image rows = whole cache lines per glds row (the BK = 32 ring above
// fetches every line in two 64-byte halves, one per stage, which costs L2 request bandwidth).
// Stage = (BM + BN) x 128 B (64 KB at 256 x 256), NS = 2 stages; each stage is consumed in two
// 32-deep MFMA sub-steps; the only barrier is before the first read of the next stage, after which
// the DMA of stage t + NS goes into the slot just drained.
// Swizzle for 128-B rows: chunk ^ ((row >> 1) & 7) — conflict-free for the ds_read_b128 lane groups.
// ============================================================================================
constexpr int BK2 = 64, ROWB2 = 128;
__device__ __forceinline__ int swz2(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <int BM, int BN, int WM, int WN, int NS_>
struct Cfg2 {
  static constexpr int NS = NS_;
  static constexpr int NW = WM * WN;  // 8 waves (2x4: 128x64 wave tiles) or 4 waves (2x2: 128x128, acc in AGPRs)
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int APIECES = BM / 8, PIECES = (BM + BN) / 8;  // 1 KB = 8 image rows per piece
  static constexpr int PPW = PIECES / NW;
  static constexpr int STAGE = (BM + BN) * ROWB2;
  static constexpr int EPI_ROWS = 64, EPI_LD = TN + 4;
  static constexpr int EPI = NW * EPI_ROWS * EPI_LD * 4;
  static constexpr int LDS = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  static_assert((NW == 8 || NW == 4) && PIECES % NW == 0 && APIECES % NW == 0 && FM * 2 >= PPW, "config");
  static_assert(TN % 32 == 0, "epilogue pairing needs 32-column multiples per wave");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// Row offset (in B rows) of B piece pb = w + 8 k relative to piece w, and the base row of piece w.
// 8-row pieces of the permuted images: SWIGLU image row 32q + 16h + r, ROPE (per 128-row head) 32q + 16h + r.
template <int EPI>
__device__ __forceinline__ int b2_row(int pb, int n0, int I) {
  if constexpr (EPI == EPI_SWIGLU) {
    return ((pb >> 1) & 1) * I + (n0 >> 1) + 16 * (pb >> 2) + 8 * (pb & 1);
  } else if constexpr (EPI == EPI_ROPE) {
    const int head = pb >> 4, v = pb & 15;
    return n0 + 128 * head + 16 * (v >> 2) + 64 * ((v >> 1) & 1) + 8 * (v & 1);
  } else {
    return n0 + 8 * pb;
  }
}
template <int EPI, int NW>
constexpr int b2_koff(int k) {  // b2_row(w + NW k) - b2_row(w), independent of w < NW (NW = 4 or 8)
  return EPI == EPI_SWIGLU ? 4 * NW * k
                           : (EPI == EPI_ROPE ? 128 * ((NW * k) >> 4) + 16 * (((NW * k) & 15) >> 2) : 8 * NW * k);
}

template <class G, int EPI>
struct Stager2 {
  static constexpr int JA = G::APIECES / G::NW;
  const u16* pa;
  const u16* pb;
  long lda, ldb;
  int left;
  __device__ __forceinline__ void piece(char* buf, int w, int j) {
    const u16* src = j < JA ? pa + (long)(8 * G::NW * j) * lda : pb + (long)b2_koff<EPI, G::NW>(j - JA) * ldb;
    glds16(src, buf + (w + G::NW * j) * 1024);
  }
  __device__ __forceinline__ void advance() {
    if (--left > 0) {
      pa += BK2;
      pb += BK2;
    }
  }
};

template <class G, int EPI, bool SCHED = true, bool TRC = false>
__device__ __forceinline__ void ring2_loop(char* __restrict__ b0, char* __restrict__ b1, char* __restrict__ b2,
                                           int nsteps, Stager2<G, EPI>& st, int w, int offA0, int offA1, int offB0,
                                           int offB1, f32x4 (&acc)[G::FM][G::FN]) {
  constexpr int NS = G::NS, PPW = G::PPW;
  bf16x8 fa[G::FM], fb[2][G::FN];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    char* d = i == 0 ? b0 : (i == 1 ? b1 : b2);
#pragma unroll
    for (int j = 0; j < PPW; ++j) st.piece(d, w, j);
    st.advance();
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 1) * PPW, 0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < G::FN; ++j) fb[0][j] = lds_row(b0, offB0 + 2048 * j);
#pragma unroll
  for (int i = 0; i < G::FM; ++i) fa[i] = lds_row(b0, offA0 + 2048 * i);
  for (int t0 = 0; t0 < nsteps; t0 += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      if (t0 + u < nsteps) {
        char* cur = u == 0 ? b0 : (u == 1 ? b1 : b2);
        const int un = (u + 1) % NS;
        char* nxt = un == 0 ? b0 : (un == 1 ? b1 : b2);
        // sub-step 0: MFMA on (t, k 0..31) while reading (t, k 32..63) from the same slot
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb[1][j] = lds_row(cur, offB1 + 2048 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = TRC ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[0][j], fa[i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[0][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_row(cur, offA1 + 2048 * i);
          if (SCHED) {
            __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
        }
        __builtin_amdgcn_s_setprio(0);
        // sub-step 1: stage t+1 landed (own DMAs) and every wave is done reading slot t -> barrier,
        // then refill slot t with stage t + NS while MFMA-ing (t, k 32..63) and reading (t+1, k 0..31)
        __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 2) * PPW, 0));
        __builtin_amdgcn_s_barrier();
        // (after the last stage these read a slot nobody uses: harmless, and branch-free)
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb[0][j] = lds_row(nxt, offB0 + 2048 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = TRC ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[1][j], fa[i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[1][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_row(nxt, offA0 + 2048 * i);
          // DMA pieces of stage t + NS spread over the fragment rows (PPW <= 2 FM)
          if (2 * i < PPW) st.piece(cur, w, 2 * i);
          if (2 * i + 1 < PPW) st.piece(cur, w, 2 * i + 1);
          if (SCHED) {
            __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if (2 * i + 1 < PPW) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
            else if (2 * i < PPW) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          }
        }
        st.advance();
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
}

// Early-release variant of ring2_loop (NS = 2): all fragments of a stage's second k-half are read
// at the start of the stage (32 more VGPRs), so the slot is released — and the DMA of stage t + 2
// issued into it — half a stage earlier: ~1.5 stages of lead time per DMA instead of 1.
template <class G, int EPI>
__device__ __forceinline__ void ring2e_loop(char* __restrict__ b0, char* __restrict__ b1, int nsteps,
                                            Stager2<G, EPI>& st, int w, int offA0, int offA1, int offB0, int offB1,
                                            f32x4 (&acc)[G::FM][G::FN]) {
  constexpr int PPW = G::PPW, H = G::FM / 2;
  static_assert(G::NS == 2 && PPW <= 2 * H, "early-release ring: 2 stages");
  bf16x8 fa[G::FM], fa2[G::FM], fb0[G::FN], fb1[G::FN];
#pragma unroll
  for (int j = 0; j < PPW; ++j) st.piece(b0, w, j);
  st.advance();
#pragma unroll
  for (int j = 0; j < PPW; ++j) st.piece(b1, w, j);
  st.advance();
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(PPW, 0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < G::FN; ++j) fb0[j] = lds_row(b0, offB0 + 2048 * j);
#pragma unroll
  for (int i = 0; i < G::FM; ++i) fa[i] = lds_row(b0, offA0 + 2048 * i);
  for (int t0 = 0; t0 < nsteps; t0 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (t0 + u < nsteps) {
        char* cur = u == 0 ? b0 : b1;
        char* nxt = u == 0 ? b1 : b0;
        // A: read (t, k 32..63); MFMA the first half of (t, k 0..31) while they land
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb1[j] = lds_row(cur, offB1 + 2048 * j);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) fa2[i] = lds_row(cur, offA1 + 2048 * i);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < H; ++i)
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb0[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(PPW, 0));  // own reads of slot cur done (stage t+1 may fly)
        __builtin_amdgcn_s_barrier();                     // every wave's reads of slot cur done
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = H; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb0[j], acc[i][j], 0, 0, 0);
          const int q = i - H;
          if (2 * q < PPW) st.piece(cur, w, 2 * q);
          if (2 * q + 1 < PPW) st.piece(cur, w, 2 * q + 1);
          __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);
          if (2 * q + 1 < PPW) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          else if (2 * q < PPW) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        st.advance();
        __builtin_amdgcn_s_setprio(0);
        // B: stage t+1 landed (leave stage t+2 in flight); read (t+1, k 0..31) under (t, k 32..63)
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(PPW, 0));
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb0[j] = lds_row(nxt, offB0 + 2048 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa2[i], fb1[j], acc[i][j], 0, 0, 0);
          fa[i] = lds_row(nxt, offA0 + 2048 * i);
          __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
}

// Epilogue of the TRC (transposed-C) build: with the B fragment as the MFMA's first operand, lane
// (g, ii) of fragment (i, j) holds output row 16 i + ii, columns 16 j + 4 g .. + 3 — four consecutive
// columns, so the tile goes to LDS as packed bf16x4 (one ds_write_b64 per fragment instead of four
// ds_write_b32 of fp32) and back as 16-byte rows for the global stores; the paired fragments (2q,
// 2q + 1) of SWIGLU / ROPE meet in one lane and are combined in registers before staging.
__device__ __forceinline__ uint2 pack4(const float* f) {
  return make_uint2(pk2bf(f[0], f[1]), pk2bf(f[2], f[3]));
}

template <class G, int EPI>
__device__ __forceinline__ void epilogue_t(char* smem, f32x4 (&acc)[G::FM][G::FN], const EpiArgs& ea, int m0, int n0,
                                           int wm, int wn, int w, int lane) {
  // per-wave LDS region: EROWS rows x LDW bf16 (rows 16-byte multiples, +16 B pad against write conflicts)
  static_assert(G::NW == 8 && G::TN == 64, "transposed-C epilogue: 8 waves of 128x64");
  constexpr int NCOL = EPI == EPI_SWIGLU ? G::TN + G::TN / 2 : G::TN;  // SWIGLU stages gate | up | act
  constexpr int LDW = NCOL + 8;
  constexpr int EROWS = (G::TM * LDW * 2 * 8 <= G::LDS) ? G::TM : G::TM / 2;  // within the kernel's LDS
  constexpr int PASSES = G::TM / EROWS, FPP = EROWS / 16;
  static_assert(EROWS * LDW * 2 * 8 <= G::LDS, "epilogue LDS");
  const int g = lane >> 4, ii = lane & 15;
  u16* ep = reinterpret_cast<u16*>(smem) + w * EROWS * LDW;
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    const int rbase = m0 + wm * G::TM + pass * EROWS;
#pragma unroll
    for (int fi = 0; fi < FPP; ++fi) {
      const int i = pass * FPP + fi;
      u16* er = ep + (16 * fi + ii) * LDW;
      if constexpr (EPI == EPI_PLAIN) {
#pragma unroll
        for (int j = 0; j < G::FN; ++j) {
          const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          *(uint2*)(er + 16 * j + 4 * g) = pack4(v);
        }
      } else {
#pragma unroll
        for (int q = 0; q < G::FN / 2; ++q) {
          float a[4], b[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = rbf(acc[i][2 * q][e]);  // the bf16 projection values the unfused path would see
            b[e] = rbf(acc[i][2 * q + 1][e]);
          }
          if constexpr (EPI == EPI_SWIGLU) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = silu(a[e]) * b[e];
            *(uint2*)(er + 16 * q + 4 * g) = pack4(a);                       // gate  [0, TN/2)
            *(uint2*)(er + G::TN / 2 + 16 * q + 4 * g) = pack4(b);           // up    [TN/2, TN)
            *(uint2*)(er + G::TN + 16 * q + 4 * g) = pack4(o);               // act   [TN, 3TN/2)
          } else {  // ROPE: lo = head dim d, hi = d + 64
            const int t = wn * G::TN + 32 * q + 4 * g;
            const int head = t >> 7, u = t & 127, d = 16 * (u >> 5) + (u & 15);
            if (n0 + 128 * head + d < ea.rope_cols) {
              const long row = rbase + 16 * fi + ii;
              const float4 c4 = *(const float4*)(ea.cosb + row * 64 + d);
              const float4 s4 = *(const float4*)(ea.sinb + row * 64 + d);
              const float cs[4] = {c4.x, c4.y, c4.z, c4.w}, sn[4] = {s4.x, s4.y, s4.z, s4.w};
              float lo[4], hi[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                lo[e] = a[e] * cs[e] - b[e] * sn[e];
                hi[e] = b[e] * cs[e] + a[e] * sn[e];
              }
              *(uint2*)(er + 16 * q + 4 * g) = pack4(lo);
              *(uint2*)(er + G::TN / 2 + 16 * q + 4 * g) = pack4(hi);
            } else {
              *(uint2*)(er + 16 * q + 4 * g) = pack4(a);
              *(uint2*)(er + G::TN / 2 + 16 * q + 4 * g) = pack4(b);
            }
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region: writes before reads
    constexpr int SEGS = NCOL / 8;                       // 16-byte segments per staged row
#pragma unroll
    for (int it = 0; it < EROWS * SEGS / 64; ++it) {
      const int sg = it * 64 + lane, row = sg / SEGS, cs = sg - row * SEGS;
      const uint4 v = *(const uint4*)(ep + row * LDW + cs * 8);
      const long grow = rbase + row;
      if constexpr (EPI == EPI_PLAIN) {
        *(uint4*)(ea.C + grow * ea.ldc + n0 + wn * G::TN + cs * 8) = v;
      } else if constexpr (EPI == EPI_SWIGLU) {
        const int part = cs / (G::TN / 16), k = cs - part * (G::TN / 16);  // 0 gate, 1 up, 2 act
        const int c = (n0 >> 1) + (G::TN / 2) * wn + 8 * k;
        if (part == 0) *(uint4*)(ea.C + grow * ea.ldc + c) = v;
        else if (part == 1) *(uint4*)(ea.C + grow * ea.ldc + ea.I + c) = v;
        else *(uint4*)(ea.act + grow * ea.I + c) = v;
      } else {  // ROPE: staged [lo 32 | hi 32]
        const int part = cs / (G::TN / 16), k = cs - part * (G::TN / 16);
        const int head = wn >> 1, dbase = 32 * (wn & 1);
        *(uint4*)(ea.C + grow * ea.ldc + n0 + 128 * head + dbase + 64 * part + 8 * k) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

template <int BM, int BN, int WM, int WN, int NS, int EPI, int VAR = 0>
__global__ void __launch_bounds__(WM * WN * 64) tn2_kernel(const u16* __restrict__ A, const u16* __restrict__ B, int K, long lda,
                                                 long ldb, int nbm, int nbn, int group, EpiArgs ea) {
  using G = Cfg2<BM, BN, WM, WN, NS>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_group = group * nbn;
  const int grp = wgid / per_group, first = grp * group;
  const int gsz = min(nbm - first, group);
  const int in = wgid - grp * per_group;
  const int bm = first + in % gsz, bn = in / gsz;
  const int m0 = bm * BM, n0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w - wm * WN;

  Stager2<G, EPI> st;
  st.lda = lda;
  st.ldb = ldb;
  st.left = K / BK2;
  {
    // piece P = w + NW j holds image rows 8P + lr (lr = lane >> 3), slot lane & 7; (row >> 1) & 7 =
    // 4 (P & 1) + (lr >> 1) and P & 1 = w & 1 for every piece of the wave (NW even)
    const int lr = lane >> 3, ch = (lane & 7) ^ (4 * (w & 1) + (lr >> 1));
    st.pa = A + (long)(m0 + 8 * w + lr) * lda + 8 * ch;
    st.pb = B + (long)(b2_row<EPI>(w, n0, ea.I) + lr) * ldb + 8 * ch;
  }
  const int g = lane >> 4, ii = lane & 15;
  const int ra = wm * G::TM + ii, rb = BM + wn * G::TN + ii;
  const int offA0 = ra * ROWB2 + 16 * swz2(ra, g), offA1 = ra * ROWB2 + 16 * swz2(ra, 4 + g);
  const int offB0 = rb * ROWB2 + 16 * swz2(rb, g), offB1 = rb * ROWB2 + 16 * swz2(rb, 4 + g);
  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (VAR == 1)
    ring2e_loop<G, EPI>(smem, smem + G::STAGE, K / BK2, st, w, offA0, offA1, offB0, offB1, acc);
  else
    ring2_loop<G, EPI, VAR == 2, VAR == 3>(smem, smem + G::STAGE, smem + (NS > 2 ? 2 : 0) * G::STAGE, K / BK2, st,
                                           w, offA0, offA1, offB0, offB1, acc);
  __syncthreads();
  if constexpr (VAR == 3)
    epilogue_t<G, EPI>(smem, acc, ea, m0, n0, wm, wn, w, lane);
  else
    epilogue<G, EPI>(smem, acc, ea, m0, n0, wm, wn, w, lane);
}

// ============================================================================================
// Ping-pong 8-phase schedule (cfg 8 / 9), /opt/skills/guides/cdna_hip_programming.md §5 "The 256² 8-phase template".
// Same tile (256 x 256, BK = 64, 8 waves of 128 x 64) and the same two 64 KB LDS stages as the BK = 64
// ring above, but each K-tile runs as FOUR phases, one output quadrant (64 x 32 per wave, 16 MFMAs)
// each, and the two wave rows run ONE BARRIER APART: while wave row 0 is in a phase's MFMA segment,
// wave row 1 (its partner on the same SIMD) issues the next phase's LDS reads and DMA, and vice versa
// — matrix beside memory on every SIMD (/opt/skills/guides/MI355X_MICROARCH.md §Two waves per SIMD). Every phase is
//   [L: ds_reads of this phase's fragments | DMA of one class of tile t + 2 | counted vmcnt]
//   lgkmcnt(0); s_barrier; setprio 1; 16 MFMA; setprio 0; s_barrier
// The stage is laid out in four 16 KB CLASS images, one per group of fragments read together:
//   A_lo: tile rows {0..63, 128..191} (fragments i = 0..3 of both wave rows), A_hi: rows +64 (i = 4..7),
//   B_lo: tile columns 64 q + {0..31} (j = 0, 1 of every wave column), B_hi: columns +32 (j = 2, 3),
// so each class is released right after the phase that reads it and refilled with tile t + 2 at once:
//   ph1 reads A_lo + B_lo -> quadrant (A_lo, B_lo);  ph2 reads B_hi, DMA A_lo + B_lo -> (A_lo, B_hi)
//   ph3 reads A_hi, DMA B_hi -> (A_hi, B_hi);        ph4 DMA A_hi                   -> (A_hi, B_lo)
// A DMA therefore has ~6-7 phases to land. The class images are separate __restrict__ pointers, so the
// compiler's waitcnt pass does not drain the DMA of one class before reading another. Each wave issues
// 2 DMAs per class in a fixed order, so the vmcnt that retires a class is a compile-time count:
//   ph1 waits for B_hi(t) (10 younger DMAs), ph2 for A_hi(t) (8), ph4 for A_lo/B_lo(t + 1) (10),
// always one barrier pair before the read (LDS-DMA data is ordered for other waves only by the
// issuer's vmcnt followed by a barrier the reader has passed); lgkmcnt(0) BEFORE each phase's first
// barrier retires the phase's reads, which is what lets the next phase refill that class.
// ============================================================================================
constexpr int CLS = 16 * 1024;  // class image: 128 rows x 128 B
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {  // immediates must be literal; n is wave-uniform and even
    case 0: __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 15)); break;
    case 2: __builtin_amdgcn_s_waitcnt(waitcnt_imm(2, 15)); break;
    case 4: __builtin_amdgcn_s_waitcnt(waitcnt_imm(4, 15)); break;
    case 6: __builtin_amdgcn_s_waitcnt(waitcnt_imm(6, 15)); break;
    case 8: __builtin_amdgcn_s_waitcnt(waitcnt_imm(8, 15)); break;
    case 10: __builtin_amdgcn_s_waitcnt(waitcnt_imm(10, 15)); break;
    case 12: __builtin_amdgcn_s_waitcnt(waitcnt_imm(12, 15)); break;
    default: __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 15)); break;
  }
}
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void lgkm0() { __builtin_amdgcn_s_waitcnt(waitcnt_imm(63, 0)); }

struct Stager3 {
  const u16* pa;  // this lane's source in the wave's first A_lo piece (tile row 8 w + lr)
  const u16* pb;  // ... first B_lo piece
  long a64, a128, a192, b1, b2, b3;  // element offsets of the wave's other pieces
  // the wave's two 8-row pieces of class C (0 A_lo, 1 A_hi, 2 B_lo, 3 B_hi) into class image ``img``;
  // KOFF = K-tile offset from the stager's current tile
  template <int C, int KOFF = 0>
  __device__ __forceinline__ void cls(char* img, int w) {
    const u16* a = pa + KOFF * BK2;
    const u16* b = pb + KOFF * BK2;
    const u16* s0 = C == 0 ? a : (C == 1 ? a + a64 : (C == 2 ? b : b + b2));
    const u16* s1 = C == 0 ? a + a128 : (C == 1 ? a + a192 : (C == 2 ? b + b1 : b + b3));
    glds16(s0, img + w * 1024);
    glds16(s1, img + (8 + w) * 1024);
  }
  __device__ __forceinline__ void advance() {
    pa += BK2;
    pb += BK2;
  }
};

template <bool TRC, int I0, int J0>
__device__ __forceinline__ void pp_mma(f32x4 (&acc)[8][4], const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[I0 + i][J0 + j] = TRC ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], acc[I0 + i][J0 + j], 0, 0, 0)
                                  : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[I0 + i][J0 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

// fragment reads: offA / offB = this lane's (row, k-chunk g) byte offset in a class image; +2048 per
// 16-row fragment, k-sub-step 1 = chunk 4 + g (offX1)
__device__ __forceinline__ void pp_read_a(const char* img, int offA0, int offA1, bf16x8 (&fa)[4][2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    fa[i][0] = lds_row(img, offA0 + 2048 * i);
    fa[i][1] = lds_row(img, offA1 + 2048 * i);
  }
}
__device__ __forceinline__ void pp_read_b(const char* img, int offB0, int offB1, bf16x8 (&fb)[2][2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    fb[j][0] = lds_row(img, offB0 + 2048 * j);
    fb[j][1] = lds_row(img, offB1 + 2048 * j);
  }
}

// End of a phase's load segment, then its MFMA segment. D = 1: lgkmcnt(0) before the first barrier
// (a class may be refilled ONE phase after it is read); D = 2: lgkmcnt(0) after it (refilled two
// phases after: /opt/skills/guides/cdna_hip_programming.md §5, "Read a staged buffer ... WAR").
template <int D, bool TRC, int I0, int J0>
__device__ __forceinline__ void pp_phase(f32x4 (&acc)[8][4], const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[2][2]) {
  if (D == 1) lgkm0();
  bar();
  if (D == 2) lgkm0();  // also retires phase 4's read of the NEXT tile's B_lo, used only by its phase 1
  pp_mma<TRC, I0, J0>(acc, fa, fb);
  bar();
}

// One K-tile t on stage X (class images xAl, xAh, xBl, xBh); Y = the other stage (tile t + 1).
// Reads: A_lo(t) in phase 1, B_hi(t) in 2, A_hi(t) in 3, B_lo(t + 1) in 4 (into the other B_lo register
// set), 8 / 4 / 8 / 4 ds_read_b128 per phase. Each wait retires the class read in the NEXT phase.
// D = 1 DMA slots: ph1 B_lo(t+2), ph2 A_lo(t+2), ph3 B_hi(t+2), ph4 A_hi(t+2) -> X.
// D = 2 DMA slots: ph1 A_hi(t+1) -> Y, ph2 B_lo(t+2), ph3 A_lo(t+2), ph4 B_hi(t+2) -> X.
// e1 = tile t+1 exists (so tile t-1 issued its slots for t+1), e0 = tile t+2 exists; a wait's count
// is 2 x the number of this wave's DMA slots issued after the awaited one.
template <bool TRC, int D>
__device__ __forceinline__ void pp_tile(char* __restrict__ xAl, char* __restrict__ xAh, char* __restrict__ xBl,
                                        char* __restrict__ xBh, char* __restrict__ yAh, const char* __restrict__ yBl,
                                        int t, int nk, Stager3& st, int w, int offA0, int offA1, int offB0,
                                        int offB1, f32x4 (&acc)[8][4], bf16x8 (&blc)[2][2], bf16x8 (&bln)[2][2]) {
  const int e1 = t + 1 < nk, e0 = t + 2 < nk;
  bf16x8 fa[4][2], fbh[2][2];
  // phase 1: retire B_hi(t); read A_lo(t)
  wait_vm(D == 1 ? 2 + 8 * e1 : 2 + 6 * e1);
  pp_read_a(xAl, offA0, offA1, fa);
  if (D == 1) {
    if (e0) st.cls<2>(xBl, w);
  } else {
    if (e1) st.cls<1, -1>(yAh, w);
  }
  pp_phase<D, TRC, 0, 0>(acc, fa, blc);
  // phase 2: retire A_hi(t); read B_hi(t)
  wait_vm(D == 1 ? 8 * e1 + 2 * e0 : 8 * e1);
  pp_read_b(xBh, offB0, offB1, fbh);
  if (e0) {
    if (D == 1) st.cls<0>(xAl, w);
    else st.cls<2>(xBl, w);
  }
  pp_phase<D, TRC, 0, 2>(acc, fa, fbh);
  // phase 3: retire B_lo(t+1); read A_hi(t)
  if (e1) wait_vm(D == 1 ? 6 + 4 * e0 : 6 + 2 * e0);
  pp_read_a(xAh, offA0, offA1, fa);
  if (e0) {
    if (D == 1) st.cls<3>(xBh, w);
    else st.cls<0>(xAl, w);
  }
  pp_phase<D, TRC, 4, 2>(acc, fa, fbh);
  // phase 4: retire A_lo(t+1); read B_lo(t+1)
  if (e1) {
    wait_vm(D == 1 ? 4 + 6 * e0 : 4 + 4 * e0);
    pp_read_b(yBl, offB0, offB1, bln);
  }
  if (e0) {
    if (D == 1) st.cls<1>(xAh, w);
    else st.cls<3>(xBh, w);
    st.advance();
  }
  pp_phase<D, TRC, 4, 0>(acc, fa, blc);
}

template <int EPI, bool TRC, int D>
__global__ void __launch_bounds__(512) tn3_kernel(const u16* __restrict__ A, const u16* __restrict__ B, int K, long lda,
                                                  long ldb, int nbm, int nbn, int group, EpiArgs ea) {
  using G = Cfg2<256, 256, 2, 4, 2>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_group = group * nbn;
  const int grp = wgid / per_group, first = grp * group;
  const int gsz = min(nbm - first, group);
  const int in = wgid - grp * per_group;
  const int bm = first + in % gsz, bn = in / gsz;
  const int m0 = bm * 256, n0 = bn * 256;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int nk = K / BK2;

  Stager3 st;
  {
    // class piece c (8 image rows 8c + lr) of wave w: c = w and c = w + 8 -> (row >> 1) & 7 = 4 (w & 1) + (lr >> 1)
    const int lr = lane >> 3, ch = (lane & 7) ^ (4 * (w & 1) + (lr >> 1));
    st.pa = A + (long)(m0 + 8 * w + lr) * lda + 8 * ch;
    st.a64 = 64 * lda;
    st.a128 = 128 * lda;
    st.a192 = 192 * lda;
    // B_lo piece c covers tile columns 64 (c >> 2) + 8 (c & 3) + lr = 8-column piece P = 8 (c >> 2) + (c & 3);
    // B_hi adds 32 columns (4 pieces); the EPI permutation maps pieces to weight rows (b2_row)
    const int P0 = 8 * (w >> 2) + (w & 3);
    const int r0 = b2_row<EPI>(P0, n0, ea.I);
    st.pb = B + (long)(r0 + lr) * ldb + 8 * ch;
    st.b1 = (long)(b2_row<EPI>(P0 + 16, n0, ea.I) - r0) * ldb;
    st.b2 = (long)(b2_row<EPI>(P0 + 4, n0, ea.I) - r0) * ldb;
    st.b3 = (long)(b2_row<EPI>(P0 + 20, n0, ea.I) - r0) * ldb;
  }
  const int g = lane >> 4, ii = lane & 15;
  const int ra = wm * 64 + ii, rb = wn * 32 + ii;  // class-image rows of this lane's first A / B fragment
  const int offA0 = ra * ROWB2 + 16 * swz2(ra, g), offA1 = ra * ROWB2 + 16 * swz2(ra, 4 + g);
  const int offB0 = rb * ROWB2 + 16 * swz2(rb, g), offB1 = rb * ROWB2 + 16 * swz2(rb, 4 + g);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* x0 = smem;
  char* y0 = smem + 4 * CLS;
  // prologue: the DMA slots tiles -2 and -1 would have issued (class order B_lo, A_lo, B_hi, A_hi; with
  // D = 2, A_hi(1) is left to phase 1 of tile 0), then B_lo(0) into the first B_lo register set
  st.cls<2>(x0 + 2 * CLS, w);
  st.cls<0>(x0, w);
  st.cls<3>(x0 + 3 * CLS, w);
  st.cls<1>(x0 + CLS, w);
  st.advance();
  if (nk > 1) {
    st.cls<2>(y0 + 2 * CLS, w);
    st.cls<0>(y0, w);
    st.cls<3>(y0 + 3 * CLS, w);
    if (D == 1) st.cls<1>(y0 + CLS, w);
  }
  st.advance();
  wait_vm(nk > 1 ? (D == 1 ? 12 : 10) : 4);  // B_lo(0), A_lo(0)
  bar();
  bf16x8 bl0[2][2], bl1[2][2];
  pp_read_b(x0 + 2 * CLS, offB0, offB1, bl0);
  lgkm0();
  if (D == 1) bar();   // phase 1 of tile 0 refills B_lo (D = 1): every wave's read of B_lo(0) retired first
  if (wm == 1) bar();  // wave row 1 runs one barrier behind wave row 0
  for (int t = 0; t < nk; t += 2) {
    pp_tile<TRC, D>(x0, x0 + CLS, x0 + 2 * CLS, x0 + 3 * CLS, y0 + CLS, y0 + 2 * CLS, t, nk, st, w, offA0, offA1,
                    offB0, offB1, acc, bl0, bl1);
    if (t + 1 < nk)
      pp_tile<TRC, D>(y0, y0 + CLS, y0 + 2 * CLS, y0 + 3 * CLS, x0 + CLS, x0 + 2 * CLS, t + 1, nk, st, w, offA0,
                      offA1, offB0, offB1, acc, bl1, bl0);
  }
  if (wm == 0) bar();
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
  __syncthreads();
  if constexpr (TRC)
    epilogue_t<G, EPI>(smem, acc, ea, m0, n0, wm, wn, w, lane);
  else
    epilogue<G, EPI>(smem, acc, ea, m0, n0, wm, wn, w, lane);
}

// ============================================================================================
// Persistent 4-wave GEMM (the main loop of tn6 below): 4 waves of 128 x 128 (one wave per SIMD, 256 fp32 accumulators
// pinned in AGPRs by tied inline-asm MFMAs, csrc/gemm_4w.hip) with the per-tile fixed cost taken off the critical path.
// A K = 2048 tile round of the non-persistent kernels costs ~16 us besides its K loop (K sweep: 0.228 ms per 1024 of
// K + 0.18 ms fixed on gate_up, profiles/r3_gemm_4wave.md): the prologue's 128 KB burst of every CU at once and the
// LDS-staged epilogue's store burst. Here one workgroup per CU walks its XCD's tiles (per-XCD contiguous ranges of
// the GROUP_M order, so the XCD's 32 CUs share A / B panels in its L2), and per tile:
//   * the NEXT tile's first K-tile is DMA'd into stage X during the last sub-step (both stages are free after the
//     last barrier: that sub-step's MFMAs need only registers), its second K-tile into Y right after the epilogue;
//   * the epilogue stores straight from registers: TRC MFMAs (B fragment first) leave each lane 4 consecutive columns
//     of a row per fragment; v_permlane16_swap between fragment pairs makes that 8 (16 bytes), so a tile is 32
//     16-byte stores per lane, issued and not waited for (the next tile's MFMAs run while they drain);
//   * the first sub-step's MFMAs take srcC = 0 (no accumulator zeroing pass).
// vmcnt bookkeeping (loads and stores share the counter): next K0 (16) < stores (32) < next K1 (16), so "K0 landed"
// is vmcnt(48) — within the counter's 63.
// ============================================================================================
// LDS-DMA of the persistent kernel through buffer descriptors (csrc/gemm_4w.hip, profiles/r3_bwd_gemm_4wave.md): the
// A tile's rows in a per-tile descriptor, the whole weight in another, each lane's byte offset in a VGPR set once per
// tile, the piece / K offsets in SGPRs — no per-piece 64-bit VALU address arithmetic in the loop.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
__device__ __forceinline__ rsrc_t tile_rsrc(const u16* p) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, 0xFFFFFFFFu, 0x00020000);
}

template <int EPI>
struct Stager5 {
  rsrc_t ra, rb;
  unsigned va, vb;       // lane byte offsets (A: within the tile's rows; B: within the weight)
  unsigned a32;          // bytes between A pieces j, j + 1 (32 rows)
  unsigned boff[8];      // B piece q relative to piece 0 (EPI row permutation), bytes
  unsigned kb;           // K progress, bytes
  __device__ __forceinline__ void adv(int k) { kb += 2 * k; }
  __device__ __forceinline__ void piece(char* stage, int w, int j, int koff = 0) {
    char* dst = stage + (w + 4 * j) * 1024;
    if (j < 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)dst, 16, va,
                                               kb + 2 * koff + j * a32, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)dst, 16, vb,
                                               kb + 2 * koff + boff[j - 8], 0, 0);
  }
};

template <bool INIT>
__device__ __forceinline__ void mfma_t(f32x4& c, const bf16x8& b, const bf16x8& a) {
  if constexpr (INIT)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}

// one sub-step: 8 MFMA groups (fragment row i x 8 B fragments, TRC); READ: the next sub-step's 16 fragments from img;
// NP DMA pieces spread over the first DG groups; BAR: the K-tile barrier after group 0
template <int EPI, bool INIT, bool READ, int NP, bool BAR, int DG = 4, bool ROWC = false>
__device__ __forceinline__ void tn5_sub(f32x4 (&acc)[8][8], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8],
                                        bf16x8 (&ra)[8], bf16x8 (&rb)[8], const char* img, int offA, int offB,
                                        Stager5<EPI>& st, char* dst, int w, char* dst2 = nullptr) {
  static_assert(NP % DG == 0 && NP <= 32, "DMA pieces per group");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (ROWC) mfma_t<INIT>(acc[i][j], fa[i], fb[j]);  // A first: rows on the register index
      else mfma_t<INIT>(acc[i][j], fb[j], fa[i]);                  // TRC: columns on the register index
    }
    if (BAR && i == 0) __builtin_amdgcn_s_barrier();
    if (READ) {
      ra[i] = lds_row(img, offA + 2048 * i);
      rb[i] = lds_row(img, offB + 2048 * i);
    }
    if (i < DG) {
#pragma unroll
      for (int k = 0; k < NP / DG; ++k) {
        const int pc = i * (NP / DG) + k;  // pieces 16..31: the following K-tile into dst2
        if (pc < 16) st.piece(dst, w, pc);
        else st.piece(dst2, w, pc - 16, BK2);
      }
    }
  }
}

__device__ __forceinline__ void tn5_coords(int tile, int nbm, int nbn, int group, int& m0, int& n0) {
  const int per_group = group * nbn;
  const int grp = tile / per_group, first = grp * group;
  const int gsz = min(nbm - first, group);
  const int in = tile - grp * per_group;
  m0 = (first + in % gsz) * 256;
  n0 = (in / gsz) * 256;
}

__device__ __forceinline__ unsigned pack2(float a, float b) { return pk2bf(a, b); }

// Launched with one workgroup per CU (persistent): each walks its XCD's contiguous share of the tile order.
__device__ __forceinline__ int tn5_range_start(int x, int tiles) {
  const int q8 = tiles >> 3, r8 = tiles & 7;
  return x * q8 + min(x, r8);
}

// ============================================================================================
// Row-contiguous store epilogue (cfg 60 / 61 = plain / nt stores): the persistent main loop above with the MFMA operands
// in natural order (A fragment first: lane (g, ii) of fragment (i, j) holds rows 16 i + 4 g + e, column 16 j + ii of
// the wave tile) and the B image rows PERMUTED in the LDS-DMA (each lane of a piece just points at another weight
// row) so that image row 16 j + ii of a wave's 128 columns is output column 8 ii + j. A lane's 8 fragments then hold 8
// CONSECUTIVE columns of each of its rows: one 16-byte store per (fragment row i, register e), 4 rows x 256 contiguous
// bytes per wave instruction = 8 whole cache lines (hipBLASLt's pattern, profiles/r4_gemm_fwd.md; the TRC kernel's
// stores cover 16 rows x 64 bytes = 16 half lines), no lane shuffles, 32 stores per lane and tile.
// Paired epilogues put the two columns an output combines into fragments j and j + 4 of ONE lane: image row 16 j + ii
// <- column 4 ii + j of the "lo" half (SWIGLU: gate, ROPE: head dim d), 16 (j + 4) + ii <- the same column of the "hi"
// half (up, d + 64). A lane then holds 4 consecutive columns of each output per row; one DPP exchange with the
// neighbour lane (ii ^ 1) turns two rows x 8 bytes into one row x 16 bytes per lane (8 rows x 128 bytes = 8 whole
// lines per instruction). SWIGLU: 48 stores per lane and tile (gate, up, act), ROPE: 32.
// B piece q (= image piece w + 4 q) of wave w holds weight rows r6_base + r6_off(q) + {8 or 4} x (lane >> 3).
// ============================================================================================
template <int EPI>
__device__ __forceinline__ int r6_base(int n0, int w, int lr) {
  if constexpr (EPI == EPI_PLAIN) return n0 + 64 * (w & 1) + (w >> 1) + 8 * lr;
  else if constexpr (EPI == EPI_SWIGLU) return (n0 >> 1) + 32 * (w & 1) + (w >> 1) + 4 * lr;
  else return n0 + 32 * (w & 1) + (w >> 1) + 4 * lr;
}
template <int EPI>
__device__ __forceinline__ int r6_off(int q, int I) {
  if constexpr (EPI == EPI_PLAIN) return 128 * (q >> 2) + 2 * (q & 3);
  const int S = EPI == EPI_SWIGLU ? 64 : 128, H = EPI == EPI_SWIGLU ? I : 64;
  return S * (q >> 2) + 2 * (q & 1) + ((q & 2) ? H : 0);
}

template <int EPI>
__device__ __forceinline__ void tn6_stager(Stager5<EPI>& st, const u16* A, long lda, long ldb, int m0, int n0, int w,
                                           int lane) {
  const int lr = lane >> 3, ch = (lane & 7) ^ (4 * (w & 1) + (lr >> 1));
  st.ra = tile_rsrc(A + (long)m0 * lda);
  st.va = (unsigned)(((8 * w + lr) * lda + 8 * ch) * 2);
  st.vb = (unsigned)(((long)r6_base<EPI>(n0, w, lr) * ldb + 8 * ch) * 2);
  st.kb = 0;
}

__device__ __forceinline__ unsigned dpp_swap1(unsigned v) {  // value of lane ii ^ 1 (quad_perm [1, 0, 3, 2])
  return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

// Two rows (registers e, e + 1) x 4 columns per lane -> one row x 8 columns: the even lane of a pair keeps row e and
// takes its neighbour's 4 columns of it, the odd lane keeps row e + 1 (columns 4 (ii - 1) ..).
__device__ __forceinline__ u32x4 pair_rows(uint2 x0, uint2 x1, bool odd) {
  const unsigned sx = odd ? x0.x : x1.x, sy = odd ? x0.y : x1.y;
  const unsigned rx = dpp_swap1(sx), ry = dpp_swap1(sy);
  return odd ? u32x4{rx, ry, x1.x, x1.y} : u32x4{x0.x, x0.y, rx, ry};
}

template <int EPI, int AUX>
__device__ __forceinline__ void tn6_store(f32x4 (&acc)[8][8], const EpiArgs& ea, int m0, int n0, int wm, int wn,
                                          int lane) {
  const int g = lane >> 4, ii = lane & 15;
  const int r0 = m0 + wm * 128;  // the wave's first row
  if constexpr (EPI == EPI_PLAIN) {
    const rsrc_t rc = tile_rsrc(ea.C + (long)r0 * ea.ldc);
    const unsigned v = (unsigned)(((long)(4 * g) * ea.ldc + n0 + 128 * wn + 8 * ii) * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const u32x4 d = {pack2(acc[i][0][e], acc[i][1][e]), pack2(acc[i][2][e], acc[i][3][e]),
                         pack2(acc[i][4][e], acc[i][5][e]), pack2(acc[i][6][e], acc[i][7][e])};
        __builtin_amdgcn_raw_buffer_store_b128(d, rc, v, (int)((16 * i + e) * ea.ldc * 2), AUX);
      }
  } else {
    const bool odd = ii & 1;
    const int cpair = 4 * (ii & ~1);  // first column of the lane pair's 8
    if constexpr (EPI == EPI_SWIGLU) {
      const int c0 = (n0 >> 1) + 64 * wn;  // first act column of the wave
      const rsrc_t rg = tile_rsrc(ea.C + (long)r0 * ea.ldc), rat = tile_rsrc(ea.act + (long)r0 * ea.I);
      const unsigned vg = (unsigned)(((long)(4 * g + odd) * ea.ldc + c0 + cpair) * 2);
      const unsigned vu = vg + (unsigned)(ea.I * 2);
      const unsigned va = (unsigned)(((long)(4 * g + odd) * ea.I + c0 + cpair) * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int ep = 0; ep < 2; ++ep) {
          uint2 G[2], U[2], Ac[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = 2 * ep + h;
            float ga[4], up[4], o[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              ga[jj] = rbf(acc[i][jj][e]);  // act from the bf16 gate / up the backward will see
              up[jj] = rbf(acc[i][4 + jj][e]);
              o[jj] = silu(ga[jj]) * up[jj];
            }
            G[h] = make_uint2(pack2(ga[0], ga[1]), pack2(ga[2], ga[3]));
            U[h] = make_uint2(pack2(up[0], up[1]), pack2(up[2], up[3]));
            Ac[h] = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
          }
          const int so = (16 * i + 2 * ep);
          __builtin_amdgcn_raw_buffer_store_b128(pair_rows(G[0], G[1], odd), rg, vg, (int)(so * ea.ldc * 2), AUX);
          __builtin_amdgcn_raw_buffer_store_b128(pair_rows(U[0], U[1], odd), rg, vu, (int)(so * ea.ldc * 2), AUX);
          __builtin_amdgcn_raw_buffer_store_b128(pair_rows(Ac[0], Ac[1], odd), rat, va, (int)(so * ea.I * 2), AUX);
        }
    } else {  // ROPE: the wave's 128 columns are one head; lo = dims 4 ii + jj, hi = + 64
      const int hc = n0 + 128 * wn;
      const bool rot = hc < ea.rope_cols;  // a q / k head (wave-uniform)
      const rsrc_t rc = tile_rsrc(ea.C + (long)r0 * ea.ldc);
      const unsigned vl = (unsigned)(((long)(4 * g + odd) * ea.ldc + hc + cpair) * 2);
      const unsigned vh = vl + 128;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int ep = 0; ep < 2; ++ep) {
          uint2 L[2], H[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = 2 * ep + h;
            float lo[4], hi[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              lo[jj] = acc[i][jj][e];
              hi[jj] = acc[i][4 + jj][e];
            }
            if (rot) {
              const long row = r0 + 16 * i + 4 * g + e;
              const float4 c4 = *(const float4*)(ea.cosb + row * 64 + 4 * ii);
              const float4 s4 = *(const float4*)(ea.sinb + row * 64 + 4 * ii);
              const float cs[4] = {c4.x, c4.y, c4.z, c4.w}, sn[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                const float x1 = rbf(lo[jj]), x2 = rbf(hi[jj]);  // rope of the bf16 projection (unfused twin)
                lo[jj] = x1 * cs[jj] - x2 * sn[jj];
                hi[jj] = x2 * cs[jj] + x1 * sn[jj];
              }
            }
            L[h] = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
            H[h] = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
          }
          const int so = (16 * i + 2 * ep) * ea.ldc * 2;
          __builtin_amdgcn_raw_buffer_store_b128(pair_rows(L[0], L[1], odd), rc, vl, so, AUX);
          __builtin_amdgcn_raw_buffer_store_b128(pair_rows(H[0], H[1], odd), rc, vh, so, AUX);
        }
    }
  }
}

template <int EPI, bool NK2, int AUX>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
tn6_kernel(const u16* __restrict__ A, const u16* __restrict__ B, int K, long lda, long ldb, int nbm, int nbn,
           int group, EpiArgs ea) {
  using G = Cfg2<256, 256, 2, 2, 2>;
  constexpr int NST = EPI == EPI_SWIGLU ? 48 : 32;  // stores per lane and tile
  __shared__ __attribute__((aligned(16))) char smem[2 * G::STAGE];
  const int tiles = nbm * nbn, nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, l = orig >> 3, nx = (nwg - xcd + 7) >> 3;
  const int t_end = tn5_range_start(xcd + 1, tiles);
  int tile = tn5_range_start(xcd, tiles) + l;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tile >= t_end) return;
  const int wm = w >> 1, wn = w & 1;
  const int nk = K / BK2;
  const int g = lane >> 4, ii = lane & 15;
  const int ra = wm * 128 + ii, rb = 256 + wn * 128 + ii;
  const int offA0 = ra * ROWB2 + 16 * swz2(ra, g), offA1 = ra * ROWB2 + 16 * swz2(ra, 4 + g);
  const int offB0 = rb * ROWB2 + 16 * swz2(rb, g), offB1 = rb * ROWB2 + 16 * swz2(rb, 4 + g);
  char* X = smem;
  char* Y = smem + G::STAGE;
  Stager5<EPI> st;
  st.rb = tile_rsrc(B);
  st.a32 = (unsigned)(64 * lda);
#pragma unroll
  for (int q = 0; q < 8; ++q) st.boff[q] = (unsigned)((long)r6_off<EPI>(q, ea.I) * ldb * 2);
  int m0, n0;
  tn5_coords(tile, nbm, nbn, group, m0, n0);
  tn6_stager(st, A, lda, ldb, m0, n0, w, lane);
#pragma unroll
  for (int j = 0; j < 16; ++j) st.piece(X, w, j);
  st.adv(BK2);
#pragma unroll
  for (int j = 0; j < 16; ++j) st.piece(Y, w, j);
  st.adv(BK2);
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(16, 15));  // K0 of the first tile (its K1 may fly)
  f32x4 acc[8][8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  bool first = true;
  for (;;) {
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a0[i] = lds_row(X, offA0 + 2048 * i);
      b0[i] = lds_row(X, offB0 + 2048 * i);
    }
    const int next = tile + nx;
    const bool has_next = next < t_end;
    int m1 = m0, n1 = n0;
    if (has_next) tn5_coords(next, nbm, nbn, group, m1, n1);
    // the K-tile pairs of the persistent main loop (tn5_sub: boundaries, DMA placement and vmcnt accounting)
    auto pair = [&](auto init, auto dma, auto last) {
      constexpr bool IN = decltype(init)::value, DM = decltype(dma)::value, LA = decltype(last)::value;
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(63, 0));
      tn5_sub<EPI, IN, true, 0, false, 4, true>(acc, a0, b0, a1, b1, X, offA1, offB1, st, X, w);
      if (IN && !first) {
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(NST, 0));  // K1 landed; the previous tile's stores may still drain
      } else {
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
      }
      tn5_sub<EPI, false, true, DM ? 16 : 0, true, 4, true>(acc, a1, b1, a0, b0, Y, offA0, offB0, st, X, w);
      if (DM) st.adv(BK2);
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(63, 0));
      tn5_sub<EPI, false, true, 0, false, 4, true>(acc, a0, b0, a1, b1, Y, offA1, offB1, st, Y, w);
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
      if constexpr (LA) {
        tn6_stager(st, A, lda, ldb, m1, n1, w, lane);
        tn5_sub<EPI, false, false, 32, true, 4, true>(acc, a1, b1, a0, b0, X, offA0, offB0, st, X, w, Y);
      } else {
        tn5_sub<EPI, false, true, 16, true, 4, true>(acc, a1, b1, a0, b0, X, offA0, offB0, st, Y, w);
        st.adv(BK2);
      }
    };
    if constexpr (NK2) {
      pair(std::true_type(), std::false_type(), std::true_type());
    } else {
      pair(std::true_type(), std::true_type(), std::false_type());
      for (int t = 2; t < nk - 2; t += 2) pair(std::false_type(), std::true_type(), std::false_type());
      pair(std::false_type(), std::false_type(), std::true_type());
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    tn6_store<EPI, AUX>(acc, ea, m0, n0, wm, wn, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (!has_next) break;
    st.adv(2 * BK2);
    if constexpr (EPI == EPI_SWIGLU)
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(NST, 15));  // K0 and K1 landed (the 48 stores may fly)
    else
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(NST + 16, 15));  // K0 landed (K1 and the 32 stores may fly)
    first = false;
    tile = next;
    m0 = m1;
    n0 = n1;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 15));
}

template <int EPI>
void launch6(const at::Tensor& a, const at::Tensor& w, int N, const EpiArgs& ea, bool nt) {
  const int M = a.size(0), K = a.size(1);
  SFT_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0, "gemm_tn row-contiguous: M, N % 256, K % 128");
  SFT_CHECK(ea.ldc % 8 == 0 && ((uintptr_t)ea.C) % 16 == 0, "gemm_tn row-contiguous: 16-byte aligned output rows");
  const int nbm = M / 256, nbn = N / 256, tiles = nbm * nbn;
  const int grid = std::min(tiles, num_cus());
  const int grp = std::min(group_m(), nbm);
  auto A = (const u16*)a.data_ptr();
  auto B = (const u16*)w.data_ptr();
  const long lda = a.stride(0), ldb = w.stride(0);
  if (K == 128) {
    if (nt) tn6_kernel<EPI, true, 2><<<grid, 256, 0, cur_stream()>>>(A, B, K, lda, ldb, nbm, nbn, grp, ea);
    else tn6_kernel<EPI, true, 0><<<grid, 256, 0, cur_stream()>>>(A, B, K, lda, ldb, nbm, nbn, grp, ea);
  } else {
    if (nt) tn6_kernel<EPI, false, 2><<<grid, 256, 0, cur_stream()>>>(A, B, K, lda, ldb, nbm, nbn, grp, ea);
    else tn6_kernel<EPI, false, 0><<<grid, 256, 0, cur_stream()>>>(A, B, K, lda, ldb, nbm, nbn, grp, ea);
  }
  SFT_LAUNCH_CHECK();
}

template <int EPI, bool TRC, int D = 1>
void launch3(const at::Tensor& a, const at::Tensor& w, int N, const EpiArgs& ea) {
  const int M = a.size(0), K = a.size(1);
  const int nbm = M / 256, nbn = N / 256;
  tn3_kernel<EPI, TRC, D><<<nbm * nbn, 512, 0, cur_stream()>>>((const u16*)a.data_ptr(), (const u16*)w.data_ptr(), K,
                                                            a.stride(0), w.stride(0), nbm, nbn,
                                                            std::min(group_m(), nbm), ea);
  SFT_LAUNCH_CHECK();
}

template <int BM, int BN, int WM, int WN, int NS, int EPI, int VAR = 0>
void launch2(const at::Tensor& a, const at::Tensor& w, int N, const EpiArgs& ea) {
  const int M = a.size(0), K = a.size(1);
  const int nbm = M / BM, nbn = N / BN;
  tn2_kernel<BM, BN, WM, WN, NS, EPI, VAR><<<nbm * nbn, WM * WN * 64, 0, cur_stream()>>>(
      (const u16*)a.data_ptr(), (const u16*)w.data_ptr(), K, a.stride(0), w.stride(0), nbm, nbn,
      std::min(group_m(), nbm), ea);
  SFT_LAUNCH_CHECK();
}

template <int BM, int BN, int WM, int WN, int NS, int EPI>
void launch(const at::Tensor& a, const at::Tensor& w, int N, const EpiArgs& ea) {
  const int M = a.size(0), K = a.size(1);
  const int nbm = M / BM, nbn = N / BN;
  tn_kernel<BM, BN, WM, WN, NS, EPI><<<nbm * nbn, NT, 0, cur_stream()>>>(
      (const u16*)a.data_ptr(), (const u16*)w.data_ptr(), K, a.stride(0), w.stride(0), nbm, nbn,
      std::min(group_m(), nbm), ea);
  SFT_LAUNCH_CHECK();
}

}  // namespace tn

static void check_tn(const at::Tensor& a, const at::Tensor& w) {
  SFT_CHECK_CUDA(a);
  SFT_CHECK_BF16(a);
  SFT_CHECK_BF16(w);
  SFT_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1), "gemm_tn: a [M, K], w [N, K]");
  SFT_CHECK(a.stride(1) == 1 && w.stride(1) == 1, "gemm_tn: K-contiguous operands");
  SFT_CHECK(a.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_tn: 16-byte aligned rows");
  SFT_CHECK(a.size(0) % 256 == 0 && a.size(1) % tn::BK == 0 && a.size(1) > 0, "gemm_tn: M % 256, K % 32");
}

// cfg: 0 = 256x256 BK32 ring (NS 5; any K % 32), 2 = 256x256 BK64 (NS 2), 5 = BK64 transposed-C epilogue, 11 = the
// ping-pong 8-phase schedule (transposed-C, D = 2; the default for qkv + RoPE, with a 256 x 128 tail launch), 60 / 61 =
// the persistent 4-wave kernel with the row-contiguous store epilogue (plain / nt stores: the plain forwards without a
// TunableOp selection, the LoRA wide GEMM). Measurements: profiles/r1_gemm_tn.md, r2_gemm_pingpong.md,
// r4_gemm_fwd.md, r5_gemm_fwd.md.
at::Tensor gemm_tn(const at::Tensor& a, const at::Tensor& w, int64_t cfg) {
  check_tn(a, w);
  SFT_TRACE(trace_name("tn.c", cfg));
  const int M = a.size(0), N = w.size(0);
  auto c = at::empty({M, N}, a.options());
  tn::EpiArgs ea{(u16*)c.data_ptr(), nullptr, nullptr, nullptr, (long)N, 0, 0};
  const bool k64 = a.size(1) % 64 == 0;
  if (cfg == 2 || cfg == 5 || cfg == 11) {
    SFT_CHECK(N % 256 == 0 && k64, "gemm_tn BK64: N % 256, K % 64");
    if (cfg == 2) tn::launch2<256, 256, 2, 4, 2, tn::EPI_PLAIN>(a, w, N, ea);
    else if (cfg == 5) tn::launch2<256, 256, 2, 4, 2, tn::EPI_PLAIN, 3>(a, w, N, ea);
    else tn::launch3<tn::EPI_PLAIN, true, 2>(a, w, N, ea);
  } else if (cfg == 60 || cfg == 61) {
    tn::launch6<tn::EPI_PLAIN>(a, w, N, ea, cfg == 61);
  } else {
    SFT_CHECK(cfg == 0, "gemm_tn: cfg ", cfg, " not built (0, 2, 5, 11, 60, 61)");
    SFT_CHECK(N % 256 == 0, "gemm_tn 256x256: N % 256");
    tn::launch<256, 256, 2, 4, 5, tn::EPI_PLAIN>(a, w, N, ea);
  }
  return c;
}

// x [M, K], w_gu [2I, K] = [gate; up]  ->  (gu [M, 2I], act [M, I] = silu(gate) * up)
std::tuple<at::Tensor, at::Tensor> gemm_tn_swiglu(const at::Tensor& x, const at::Tensor& w_gu, int64_t cfg) {
  check_tn(x, w_gu);
  SFT_TRACE(trace_name("tn.swiglu.c", cfg));
  const int M = x.size(0), N = w_gu.size(0), I = N / 2;
  SFT_CHECK(N % 2 == 0 && I % 128 == 0, "gemm_tn_swiglu: intermediate size % 128");
  auto gu = at::empty({M, N}, x.options());
  auto act = at::empty({M, I}, x.options());
  tn::EpiArgs ea{(u16*)gu.data_ptr(), (u16*)act.data_ptr(), nullptr, nullptr, (long)N, I, 0};
  SFT_CHECK(cfg == 0 || cfg == 2 || cfg == 5 || cfg == 11 || cfg == 60 || cfg == 61,
            "gemm_tn_swiglu: cfg ", cfg, " not built (0, 2, 5, 11, 60, 61)");
  if (cfg == 60 || cfg == 61) tn::launch6<tn::EPI_SWIGLU>(x, w_gu, N, ea, cfg == 61);
  else if (x.size(1) % 64 == 0 && N % 256 == 0 && cfg == 11) tn::launch3<tn::EPI_SWIGLU, true, 2>(x, w_gu, N, ea);
  else if (x.size(1) % 64 == 0) tn::launch2<256, 256, 2, 4, 2, tn::EPI_SWIGLU, 3>(x, w_gu, N, ea);
  else tn::launch<256, 256, 2, 4, 5, tn::EPI_SWIGLU>(x, w_gu, N, ea);
  return {gu, act};
}

// x [M, K], w [N, K] (N = (nq + 2 nkv) * 128), cos/sin [M, 64] fp32: C = x w^T with rotate_half RoPE
// applied to columns [0, rope_cols).
at::Tensor gemm_tn_rope(const at::Tensor& x, const at::Tensor& w, const at::Tensor& cosb, const at::Tensor& sinb,
                        int64_t rope_cols, int64_t cfg) {
  check_tn(x, w);
  SFT_TRACE(trace_name("tn.rope.c", cfg));
  const int M = x.size(0), N = w.size(0);
  SFT_CHECK(N % 256 == 0 && rope_cols % 128 == 0, "gemm_tn_rope: N % 256, head_dim 128");
  SFT_CHECK(cosb.scalar_type() == at::kFloat && sinb.scalar_type() == at::kFloat && cosb.is_contiguous() &&
                sinb.is_contiguous() && cosb.numel() == (long)M * 64 && sinb.numel() == (long)M * 64,
            "gemm_tn_rope: cos/sin [M, 64] fp32");
  auto c = at::empty({M, N}, x.options());
  tn::EpiArgs ea{(u16*)c.data_ptr(), nullptr, cosb.data_ptr<float>(), sinb.data_ptr<float>(), (long)N, 0,
                 (int)rope_cols};
  SFT_CHECK(cfg == 0 || cfg == 2 || cfg == 5 || cfg == 11 || cfg == 60 || cfg == 61,
            "gemm_tn_rope: cfg ", cfg, " not built (0, 2, 5, 11, 60, 61)");
  if (cfg == 60 || cfg == 61) tn::launch6<tn::EPI_ROPE>(x, w, N, ea, cfg == 61);
  else if (cfg == 2 && x.size(1) % 64 == 0) tn::launch2<256, 256, 2, 4, 2, tn::EPI_ROPE>(x, w, N, ea);
  else if (cfg == 5 && x.size(1) % 64 == 0) tn::launch2<256, 256, 2, 4, 2, tn::EPI_ROPE, 3>(x, w, N, ea);
  else if (cfg == 11 && x.size(1) % 64 == 0) {
    // Wave-quantisation tail (gemm_dgrad.hip does the same): the SmolLM3 qkv grid is 32 x 12 = 384 tiles of
    // 256 x 256 = 1.5 rounds of 256 CUs. The whole round runs as one launch over the leading columns and the
    // leftover columns as 256 x 128 tiles (one round at about half a tile's time) in a second launch; heads never
    // straddle the cut (a multiple of 256), the tail's rope boundary is shifted with its pointers.
    // SFTAMD_TN_TAIL=0: one launch.
    const char* e = std::getenv("SFTAMD_TN_TAIL");
    const bool tail_on = !(e && e[0] == '0');
    const int nbm = M / 256, nbn = N / 256, tiles = nbm * nbn;
    int main_n = 0;
    if (tail_on && tiles % 256 != 0 && 256 % nbm == 0) {
      main_n = tiles / 256 * (256 / nbm);
      if ((nbn - main_n) * 2 * nbm > 256) main_n = 0;  // the 256 x 128 tail must fit one round
    }
    if (main_n <= 0) {
      tn::launch3<tn::EPI_ROPE, true, 2>(x, w, N, ea);
    } else {
      const int ncut = main_n * 256;
      SFT_TRACE("tn.rope.tail");
      tn::launch3<tn::EPI_ROPE, true, 2>(x, w.narrow(0, 0, ncut), ncut, ea);
      tn::EpiArgs et = ea;
      et.C = ea.C + ncut;
      et.rope_cols = std::max(0, ea.rope_cols - ncut);
      tn::launch2<256, 128, 4, 2, 3, tn::EPI_ROPE>(x, w.narrow(0, ncut, N - ncut), N - ncut, et);
    }
  } else tn::launch<256, 256, 2, 4, 5, tn::EPI_ROPE>(x, w, N, ea);
  return c;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("gemm_tn", &gemm_tn);
  m.impl("gemm_tn_swiglu", &gemm_tn_swiglu);
  m.impl("gemm_tn_rope", &gemm_tn_rope);
}

}  // namespace sftamd
