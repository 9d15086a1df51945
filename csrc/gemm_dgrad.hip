// Input-gradient ("dgrad") GEMM for gfx950: dX[M, N] = dY[M, K] . W[K, N], bf16 in, fp32 accumulate — the
// backward of y = x W^T for a weight stored [K = out features][N = in features] (NN in BLAS terms), with an
// optional fused SwiGLU-backward epilogue for the MLP down projection:
//
//   EPI_PLAIN       dX[m][n] = bf16(acc)
//   EPI_SWIGLU_BWD  with gu = [gate | up] saved by the forward ([M, 2N]) and dact = acc (fp32, never stored):
//                   dgu[m][n]     = dact * up * s * (1 + gate * (1 - s)),   s = sigmoid(gate)
//                   dgu[m][N + n] = dact * gate * s
//                   — the [M, N] bf16 dact round trip (write + re-read, 360 MB per SmolLM3 layer at 16 x 512
//                   tokens) and the separate swiglu_bwd launch disappear.
//
// Layout: computed transposed, C'[n][m] = sum_k W[k][n] dY[m][k], so the W tile (reduction-major, rows k) is
// the MFMA A operand read with the gfx950 transposed LDS read ds_read_b64_tr_b16 exactly as the weight-gradient
// kernel reads its operands (gemm_wgrad.hip: [32 k][128 n] images, 256-B rows, chunk XOR swizzle applied on the
// global source address because global_load_lds writes lane-linear), and the dY tile (K-contiguous rows m) is
// the B operand read along its rows like the forward kernel's weight tile (gemm_tn.hip: [m][32 k] images,
// 64-B rows). The transposed reads hand lane group g the reduction indices 8 g .. 8 g + 7 of each 32-deep step (rows
// 8 g + qq and 8 g + 4 + qq, each with its own chunk swizzle), the natural order, so the B fragment is ONE 16-byte
// read per lane (conflict-free under the B swizzle; the permuted order used before took two 8-byte reads, 2-way
// bank-conflicted).
//
// Main loop = the ring of gemm_wgrad.hip: 256 x 256 tile (n x m) per 512-thread workgroup (8 waves 2 x 4),
// BK = 32 per stage, NS stages of global_load_lds in flight, counted vmcnt + raw s_barrier once per stage,
// the next stage's fragments read while the current stage's MFMAs run, the DMA pieces spread between MFMA
// rows. Tile order: XCD-aware bijective remap, then GROUP-blocked along n.
// Epilogue: per 16-row slice of m, the fp32 wave tile is transposed through wave-private LDS ([m][n] rows of
// TM + 4 floats) so every output / gate / up access is a 16-byte vector along n.
#include "common.h"

#include <type_traits>

namespace sftamd {
namespace dgrad {

constexpr int NT = 512;
constexpr int BK = 32;
constexpr int AROWB = 256;          // A image row: 128 n x bf16
constexpr int AIMG = BK * AROWB;    // [32 k][128 n] = 8 KB
constexpr int BROWB = 64;           // B image row: 32 k x bf16

enum { EPI_PLAIN = 0, EPI_SWIGLU_BWD = 1 };

__device__ __forceinline__ int swz_a(int row, int ch) { return ch ^ (((row & 3) << 2) | ((row >> 2) & 3)); }
__device__ __forceinline__ int img_a(int row, int ch) { return row * AROWB + 16 * swz_a(row, ch); }
__device__ __forceinline__ int swz_b(int row, int ch) { return ch ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3); }

__device__ __forceinline__ void glds16(const u16* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
}

typedef __attribute__((address_space(3))) s16x4 lds_s4;

// The transposed weight read in the natural k order: lane group g holds k = 8 g .. 8 g + 7 of a 32-deep step (lo at
// row 8 g + qq, hi 4 rows below), so the dY fragment is ONE 16-byte read (bank-conflict-free under swz_b / swz_b2)
// instead of two 8-byte halves of two chunks in a permuted k order (2-way conflicted: 31 % of cfg 7's LDS cycles,
// profiles/r6_gemm_routing.md)
// (rows r and r + 4 carry different swz_a chunk swizzles: the hi half has its own offset)
__device__ __forceinline__ bf16x8 lds_tr4(const char* base, int off, int offh) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + off));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + offh));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}


constexpr unsigned waitcnt_imm(int vm, int lgkm) {  // gfx9: vmcnt[3:0] expcnt[6:4] lgkmcnt[11:8] vmcnt[5:4]<<14
  return (unsigned)((vm & 15) | (7 << 4) | ((lgkm & 15) << 8) | ((vm >> 4) << 14));
}

template <int BM, int BN, int WM, int WN, int NS_>
struct Cfg {
  static constexpr int NS = NS_;
  static constexpr int NW = WM * WN;                // 8 waves, or 4 (two workgroups per CU: cfg 8)
  static constexpr int TM = BM / WM, TN = BN / WN;  // wave tile: TM n x TN m
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int IA = BM / 128;               // A images per stage
  static constexpr int QA = 8 / NW;                 // A pieces (4 rows x 256 B) per image and wave
  static constexpr int STAGE_A = IA * AIMG, STAGE = STAGE_A + BN * BROWB;
  static constexpr int PB = BN / (16 * NW);         // B pieces (16 rows x 64 B) per wave per stage
  static constexpr int PPW = IA * QA + PB;          // DMA pieces per wave per stage
  static constexpr int EPI_LD = TM + 4;
  static constexpr int EPI = NW * 16 * EPI_LD * 4;
  static constexpr int LDS = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  static_assert((NW == 8 || NW == 4) && BM % 128 == 0 && BN % (16 * NW) == 0 && FM >= PPW, "config");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <class G>
struct Stager {
  const u16* pa;
  const u16* pb;
  long lda, ldb;
  int w, left;
  __device__ __forceinline__ void init(const u16* W, const u16* dY, long ldw, long ldd, int n0, int m0, int wave,
                                       int lane, int nsteps) {
    w = wave;
    lda = ldw;
    ldb = ldd;
    left = nsteps;
    const int ra = 4 * wave + (lane >> 4), ca = lane & 15;  // A: rows k 4w..4w+3, 16 lanes per 256-B row
    pa = W + (long)ra * ldw + n0 + 8 * swz_a(ra, ca);
    const int rb = lane >> 2;                                // B: 16 rows m per piece, 4 lanes per 64-B row
    pb = dY + (long)(m0 + 16 * wave + rb) * ldd + 8 * swz_b(rb, lane & 3);
  }
  // Past the last step the same rows are fetched again into a slot nobody reads, so every step issues
  // exactly PPW DMAs and the counted waits stay compile-time constants (see gemm_wgrad.hip).
  __device__ __forceinline__ void piece(char* buf, int j) {
    if (j < G::IA * G::QA) {  // A image j % IA, rows 4 (w + NW q) .. (the swizzle depends on row & 15 only)
      const int img = j % G::IA, q = j / G::IA;
      glds16(pa + img * 128 + (long)(4 * G::NW * q) * lda, buf + img * AIMG + (w + G::NW * q) * 1024);
    } else {
      const int jj = j - G::IA * G::QA;  // B piece w + NW jj: rows 16 (w + NW jj) ..
      glds16(pb + (long)(16 * G::NW * jj) * ldb, buf + G::STAGE_A + (w + G::NW * jj) * 1024);
    }
  }
  __device__ __forceinline__ void advance() {
    if (--left > 0) {
      pa += BK * lda;
      pb += BK;
    }
  }
  __device__ __forceinline__ void issue(char* buf) {
#pragma unroll
    for (int j = 0; j < G::PPW; ++j) piece(buf, j);
    advance();
  }
};

__device__ __forceinline__ char* pick(int i, char* b0, char* b1, char* b2, char* b3, char* b4) {
  switch (i) {
    case 0: return b0;
    case 1: return b1;
    case 2: return b2;
    case 3: return b3;
    default: return b4;
  }
}

template <class G, bool SCHED>
__device__ __forceinline__ void ring_loop(char* __restrict__ b0, char* __restrict__ b1, char* __restrict__ b2,
                                          char* __restrict__ b3, char* __restrict__ b4, int nsteps, Stager<G>& st,
                                          const int (&offA)[G::FM], const int (&offH)[G::FM], int offB,
                                          f32x4 (&acc)[G::FM][G::FN]) {
  constexpr int NS = G::NS, PPW = G::PPW;
  constexpr int U = (NS % 2) ? 2 * NS : NS;  // unroll: stage slot and B register set both compile-time
  bf16x8 fa[G::FM], fb[2][G::FN];
#pragma unroll
  for (int i = 0; i < NS; ++i) st.issue(pick(i, b0, b1, b2, b3, b4));
  __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 1) * PPW, 0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < G::FN; ++j) fb[0][j] = *(const bf16x8*)(b0 + offB + 1024 * j);
#pragma unroll
  for (int i = 0; i < G::FM; ++i) fa[i] = lds_tr4(b0, offA[i], offH[i]);
  for (int t0 = 0; t0 < nsteps; t0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t0 + u < nsteps) {
        __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 2) * PPW, 0));
        __builtin_amdgcn_s_barrier();
        char* dst = pick(u % NS, b0, b1, b2, b3, b4);
        const char* nxt = pick((u + 1) % NS, b0, b1, b2, b3, b4);
        const int cb = u & 1;
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb[cb ^ 1][j] = *(const bf16x8*)(nxt + offB + 1024 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[cb][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_tr4(nxt, offA[i], offH[i]);
          if (i < PPW) st.piece(dst, i);
          if (SCHED) {
            __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);      // DS read (one fragment)
            if (i < PPW) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (the DMA)
          }
        }
        st.advance();
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));  // drain the tail DMAs before LDS is reused
}

struct EpiArgs {
  u16* out;        // PLAIN: dX [M, ldo];  SWIGLU_BWD: dgu [M, 2N]
  const u16* gu;   // SWIGLU_BWD: gate | up [M, 2N]
  long ldo;
  int N;
};

template <class G, int EPI>
__device__ __forceinline__ void epilogue(char* smem, f32x4 (&acc)[G::FM][G::FN], const EpiArgs& ea, int n0, int m0,
                                         int wm, int wn, int w, int lane) {
  const int g = lane >> 4, c = lane & 15;
  float* ep = reinterpret_cast<float*>(smem) + w * 16 * G::EPI_LD;
  constexpr int SEGS = G::TM / 8;  // 16-byte output segments per m row
  if constexpr (EPI == EPI_SWIGLU_BWD) {
    // gate / up are streamed through a PD-deep register ring: unit u's loads are issued PD units ahead, so each
    // 16-row slice no longer waits out an HBM round trip per 64-segment step (the straight version issued the two
    // loads, waited vmcnt(0), computed and stored, 16 times per wave per tile)
    constexpr int IT = 16 * SEGS / 64, U = G::FN * IT, PD = U < 4 ? U : 4;  // 8 measured no better (r3_run44)
    static_assert(U >= PD, "ring deeper than the epilogue");
    auto base_of = [&](int u) -> long {
      const int jf = u / IT, seg = (u - jf * IT) * 64 + lane, row = seg / SEGS, cs = seg - row * SEGS;
      const long m = m0 + wn * G::TN + 16 * jf + row;
      return m * 2L * ea.N + n0 + wm * G::TM + cs * 8;
    };
    uint4 rg[PD][2];
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const long b = base_of(u);
      rg[u][0] = *(const uint4*)(ea.gu + b);
      rg[u][1] = *(const uint4*)(ea.gu + b + ea.N);
    }
#pragma unroll
    for (int jf = 0; jf < G::FN; ++jf) {
#pragma unroll
      for (int i = 0; i < G::FM; ++i) *(f32x4*)(ep + c * G::EPI_LD + 16 * i + 4 * g) = acc[i][jf];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region: writes before reads
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int u = jf * IT + it;
        const int seg = it * 64 + lane, row = seg / SEGS, cs = seg - row * SEGS;
        const float* pr = ep + row * G::EPI_LD + cs * 8;
        float v[8], gt[8], up[8], dg[8], du[8];
        *(float4*)&v[0] = *(const float4*)pr;
        *(float4*)&v[4] = *(const float4*)(pr + 4);
        unpack8(rg[u % PD][0], gt);
        unpack8(rg[u % PD][1], up);
        if (u + PD < U) {
          const long b = base_of(u + PD);
          rg[u % PD][0] = *(const uint4*)(ea.gu + b);
          rg[u % PD][1] = *(const uint4*)(ea.gu + b + ea.N);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // explicit fma, no contraction: every tile config rounds identically
#pragma clang fp contract(off)
          const float sg = 1.f / (1.f + __expf(-gt[e]));
          const float t = v[e] * sg;
          du[e] = t * gt[e];
          dg[e] = (t * up[e]) * __builtin_fmaf(gt[e], 1.f - sg, 1.f);
        }
        const long b = base_of(u);
        *(uint4*)(ea.out + b) = pack8(dg);
        *(uint4*)(ea.out + b + ea.N) = pack8(du);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next slice overwrites
    }
    return;
  }
#pragma unroll
  for (int jf = 0; jf < G::FN; ++jf) {
#pragma unroll
    for (int i = 0; i < G::FM; ++i) *(f32x4*)(ep + c * G::EPI_LD + 16 * i + 4 * g) = acc[i][jf];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region: writes before reads
#pragma unroll
    for (int it = 0; it < 16 * SEGS / 64; ++it) {
      const int seg = it * 64 + lane, row = seg / SEGS, cs = seg - row * SEGS;
      const float* pr = ep + row * G::EPI_LD + cs * 8;
      float v[8];
      *(float4*)&v[0] = *(const float4*)pr;
      *(float4*)&v[4] = *(const float4*)(pr + 4);
      const long m = m0 + wn * G::TN + 16 * jf + row;
      const int n = n0 + wm * G::TM + cs * 8;
      if constexpr (EPI == EPI_PLAIN) {
        *(uint4*)(ea.out + m * ea.ldo + n) = pack8(v);
      } else {
        const long base = m * 2L * ea.N + n;
        float gt[8], up[8], dg[8], du[8];
        unpack8(*(const uint4*)(ea.gu + base), gt);
        unpack8(*(const uint4*)(ea.gu + base + ea.N), up);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          swiglu_grad(v[e], gt[e], up[e], dg[e], du[e]);
        }
        *(uint4*)(ea.out + base) = pack8(dg);
        *(uint4*)(ea.out + base + ea.N) = pack8(du);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next slice overwrites
  }
}

template <int BM, int BN, int WM, int WN, int NS, int EPI, int OCC = 1, bool SCHED = true>
__global__ void __launch_bounds__(WM * WN * 64, OCC) dgrad_kernel(const u16* __restrict__ dY, const u16* __restrict__ W, int K,
                                                        long ldd, long ldw, int nbn, int nbm, int group, EpiArgs ea) {
  using G = Cfg<BM, BN, WM, WN, NS>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_group = group * nbm;
  const int grp = wgid / per_group, first = grp * group;
  const int gsz = min(nbn - first, group);
  const int in = wgid - grp * per_group;
  const int bn = first + in % gsz, bm = in / gsz;
  const int n0 = bn * BM, m0 = bm * BN;
  SFT_DASSERT(bn < nbn && bm < nbm);

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w - wm * WN;

  Stager<G> st;
  st.init(W, dY, ldw, ldd, n0, m0, w, lane, K / BK);
  const int g = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
  const int r0 = 8 * g + qq;  // natural k order (lds_tr4): lane group g holds k 8 g .. 8 g + 7
  int offA[G::FM], offH[G::FM];
#pragma unroll
  for (int i = 0; i < G::FM; ++i) {
    const int nl = wm * G::TM + 16 * i;
    offA[i] = (nl >> 7) * AIMG + img_a(r0, 2 * ((nl & 127) >> 4) + (pp >> 1)) + 8 * (pp & 1);
    offH[i] = (nl >> 7) * AIMG + img_a(r0 + 4, 2 * ((nl & 127) >> 4) + (pp >> 1)) + 8 * (pp & 1);
  }
  // B fragment: the 16-byte chunk g of row wn*TN + 16 j + ii (rows share the swizzle of ii: fragment j is 1 KB
  // after j - 1); conflict-free for ds_read_b128's 16-lane groups under swz_b
  const int rowb = wn * G::TN + ii;
  const int offB = G::STAGE_A + rowb * BROWB + 16 * swz_b(ii, g);
  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* b[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) b[i] = smem + (i < NS ? i : 0) * G::STAGE;
  ring_loop<G, SCHED>(b[0], b[1], b[2], b[3], b[4], K / BK, st, offA, offH, offB, acc);
  __syncthreads();
  epilogue<G, EPI>(smem, acc, ea, n0, m0, wm, wn, w, lane);
}

// ============================================================================================
// BK = 64 variant (cfg 7): a stage holds 64 k — A' images [64 k][128 n] (16 KB), B' rows of 128 B (whole
// cache lines: the BK = 32 ring fetches every dY line in two halves) — in NS = 2 slots (128 KB). Each stage is
// consumed in two 32-deep sub-steps (the pipeline of gemm_tn.hip ring2_loop): sub-step 0 computes k 0..31 from
// registers while reading k 32..63 of the same slot; then one barrier (stage t+1 landed, slot t drained), and
// sub-step 1 computes k 32..63 while reading stage t+1's k 0..31 and refilling slot t with stage t+2.
// B' swizzle for 128-B rows: chunk ^ ((row >> 1) & 7).
constexpr int BK2 = 64;
constexpr int AIMG2 = BK2 * AROWB;  // [64 k][128 n] = 16 KB
constexpr int BROWB2 = 128;
__device__ __forceinline__ int swz_b2(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <int BM, int BN, int WM, int WN>
struct Cfg2 {
  static constexpr int NS = 2;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int IA = BM / 128;
  static constexpr int STAGE_A = IA * AIMG2, STAGE = STAGE_A + BN * BROWB2;
  static constexpr int PA = IA * 2;                 // A pieces per wave: 2 row groups (of 32 k) per image
  static constexpr int PB = BN / 64;                // B pieces (8 rows x 128 B) per wave
  static constexpr int PPW = PA + PB;
  static constexpr int EPI_LD = TM + 4;
  static constexpr int EPI = 8 * 16 * EPI_LD * 4;
  static constexpr int LDS = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  static_assert(WM * WN == 8 && BM % 128 == 0 && BN % 64 == 0 && 2 * FM >= PPW, "config");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <class G>
struct Stager2 {
  const u16* pa;
  const u16* pb;
  long lda, ldb;
  int w, left;
  __device__ __forceinline__ void init(const u16* W, const u16* dY, long ldw, long ldd, int n0, int m0, int wave,
                                       int lane, int nsteps) {
    w = wave;
    lda = ldw;
    ldb = ldd;
    left = nsteps;
    const int ra = 4 * wave + (lane >> 4);  // + 32 jj: the swizzle depends on row & 15 only through wave / lane
    pa = W + (long)ra * ldw + n0 + 8 * swz_a(ra, lane & 15);
    const int rb = 8 * wave + (lane >> 3);  // B piece w + 8 j: rows 8 (w + 8 j) + lane / 8
    pb = dY + (long)(m0 + rb) * ldd + 8 * swz_b2(rb, lane & 7);
  }
  __device__ __forceinline__ void piece(char* buf, int j) {
    if (j < G::PA) {  // image j >> 1, row group j & 1
      glds16(pa + (long)(32 * (j & 1)) * lda + 128 * (j >> 1), buf + (j >> 1) * AIMG2 + (w + 8 * (j & 1)) * 1024);
    } else {
      const int jb = j - G::PA;
      glds16(pb + (long)(64 * jb) * ldb, buf + G::STAGE_A + (w + 8 * jb) * 1024);
    }
  }
  __device__ __forceinline__ void advance() {
    if (--left > 0) {
      pa += BK2 * lda;
      pb += BK2;
    }
  }
};

template <class G>
__device__ __forceinline__ void ring2_loop(char* __restrict__ b0, char* __restrict__ b1, int nsteps, Stager2<G>& st,
                                           const int (&offA)[G::FM], const int (&offH)[G::FM], int ob0, int ob1,
                                           f32x4 (&acc)[G::FM][G::FN]) {
  constexpr int PPW = G::PPW;
  bf16x8 fa[G::FM], fb[2][G::FN];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) st.piece(i == 0 ? b0 : b1, j);
    st.advance();
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(PPW, 0));
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < G::FN; ++j) fb[0][j] = *(const bf16x8*)(b0 + ob0 + 2048 * j);
#pragma unroll
  for (int i = 0; i < G::FM; ++i) fa[i] = lds_tr4(b0, offA[i], offH[i]);
  for (int t0 = 0; t0 < nsteps; t0 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (t0 + u < nsteps) {
        char* cur = u == 0 ? b0 : b1;
        char* nxt = u == 0 ? b1 : b0;
        // sub-step 0: k 0..31 of stage t from registers; read k 32..63 of the same slot
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb[1][j] = *(const bf16x8*)(cur + ob1 + 2048 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[0][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_tr4(cur, offA[i] + 32 * AROWB, offH[i] + 32 * AROWB);
        }
        __builtin_amdgcn_s_setprio(0);
        // stage t + 1 landed (this wave's DMAs) and every wave is done reading slot t
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int j = 0; j < G::FN; ++j) fb[0][j] = *(const bf16x8*)(nxt + ob0 + 2048 * j);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[1][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_tr4(nxt, offA[i], offH[i]);
          if (2 * i < PPW) st.piece(cur, 2 * i);          // refill slot t with stage t + 2
          if (2 * i + 1 < PPW) st.piece(cur, 2 * i + 1);
        }
        st.advance();
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));
}

template <int BM, int BN, int WM, int WN, int EPI>
__global__ void __launch_bounds__(NT) dgrad2_kernel(const u16* __restrict__ dY, const u16* __restrict__ W, int K,
                                                    long ldd, long ldw, int nbn, int nbm, int group, EpiArgs ea) {
  using G = Cfg2<BM, BN, WM, WN>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_group = group * nbm;
  const int grp = wgid / per_group, first = grp * group;
  const int gsz = min(nbn - first, group);
  const int in = wgid - grp * per_group;
  const int bn = first + in % gsz, bm = in / gsz;
  const int n0 = bn * BM, m0 = bm * BN;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w - wm * WN;
  Stager2<G> st;
  st.init(W, dY, ldw, ldd, n0, m0, w, lane, K / BK2);
  const int g = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
  const int r0 = 8 * g + qq;  // natural k order (lds_tr4): lane group g holds k 8 g .. 8 g + 7 of each sub-step
  int offA[G::FM], offH[G::FM];
#pragma unroll
  for (int i = 0; i < G::FM; ++i) {
    const int nl = wm * G::TM + 16 * i;
    offA[i] = (nl >> 7) * AIMG2 + img_a(r0, 2 * ((nl & 127) >> 4) + (pp >> 1)) + 8 * (pp & 1);
    offH[i] = (nl >> 7) * AIMG2 + img_a(r0 + 4, 2 * ((nl & 127) >> 4) + (pp >> 1)) + 8 * (pp & 1);
  }
  // B fragment of sub-step s: the 16-byte chunk 4 s + g of row wn*TN + 16 j + ii (swizzle of ii)
  const int rowb = wn * G::TN + ii;
  const int bbase = G::STAGE_A + rowb * BROWB2;
  const int ob0 = bbase + 16 * swz_b2(ii, g), ob1 = bbase + 16 * swz_b2(ii, 4 + g);
  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  ring2_loop<G>(smem, smem + G::STAGE, K / BK2, st, offA, offH, ob0, ob1, acc);
  __syncthreads();
  epilogue<Cfg<BM, BN, WM, WN, 2>, EPI>(smem, acc, ea, n0, m0, wm, wn, w, lane);
}

template <int BM, int BN, int WM, int WN, int EPI>
void launch2(const at::Tensor& dy, const at::Tensor& w, const EpiArgs& ea);

static int group_n() { return 8; }  // GROUP tile order over the output columns

template <int BM, int BN, int WM, int WN, int NS, int EPI, int OCC = 1, bool SCHED = true>
void launch(const at::Tensor& dy, const at::Tensor& w, const EpiArgs& ea) {
  const int M = dy.size(0), K = dy.size(1), N = w.size(1);
  const int nbn = N / BM, nbm = M / BN;
  dgrad_kernel<BM, BN, WM, WN, NS, EPI, OCC, SCHED><<<nbn * nbm, WM * WN * 64, 0, cur_stream()>>>(
      (const u16*)dy.data_ptr(), (const u16*)w.data_ptr(), K, dy.stride(0), w.stride(0), nbn, nbm,
      std::min(group_n(), nbn), ea);
  SFT_LAUNCH_CHECK();
}

template <int BM, int BN, int WM, int WN, int EPI>
void launch2(const at::Tensor& dy, const at::Tensor& w, const EpiArgs& ea) {
  const int M = dy.size(0), K = dy.size(1), N = w.size(1);
  const int nbn = N / BM, nbm = M / BN;
  dgrad2_kernel<BM, BN, WM, WN, EPI><<<nbn * nbm, NT, 0, cur_stream()>>>(
      (const u16*)dy.data_ptr(), (const u16*)w.data_ptr(), K, dy.stride(0), w.stride(0), nbn, nbm,
      std::min(group_n(), nbn), ea);
  SFT_LAUNCH_CHECK();
}

}  // namespace dgrad

void g4_dgrad(const at::Tensor& dy, const at::Tensor& w, u16* out, long ldo, const u16* attn_out = nullptr,
              long ld_attn = 0, float* delta = nullptr);

// dO = dy @ w_o on the 4-wave kernel with flash attention's delta fused into the epilogue: returns (dO [M, N],
// delta [N / 128, M] fp32 = per-head rowsum(dO . attn_out)), the layout flash_bwd takes (its `delta` argument).
std::tuple<at::Tensor, at::Tensor> dgrad_gemm_delta(const at::Tensor& dy, const at::Tensor& w,
                                                    const at::Tensor& attn_out) {
  SFT_CHECK_CUDA(dy);
  SFT_CHECK_BF16(dy);
  SFT_CHECK_BF16(w);
  SFT_CHECK_BF16(attn_out);
  SFT_CHECK(dy.dim() == 2 && w.dim() == 2 && attn_out.dim() == 2, "dgrad_gemm_delta: 2-D operands");
  SFT_CHECK(dy.stride(1) == 1 && w.stride(1) == 1 && attn_out.stride(1) == 1, "dgrad_gemm_delta: contiguous rows");
  const int64_t M = dy.size(0), K = dy.size(1), N = w.size(1);
  SFT_CHECK(w.size(0) == K && attn_out.size(0) == M && attn_out.size(1) == N,
            "dgrad_gemm_delta: dy [M, K] . w [K, N], attn_out [M, N]");
  SFT_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && K > 0 && K < 8192,
            "dgrad_gemm_delta: M, N % 256, K % 128, K < 8192 (whole tiles)");
  SFT_CHECK(dy.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && (uintptr_t)dy.data_ptr() % 16 == 0 &&
                (uintptr_t)w.data_ptr() % 16 == 0,
            "dgrad_gemm_delta: 16-byte aligned rows");
  auto out = at::empty({M, N}, dy.options());
  auto delta = at::empty({N / 128, M}, dy.options().dtype(at::kFloat));
  SFT_TRACE("dgrad.c14.delta");
  g4_dgrad(dy, w, (u16*)out.data_ptr(), N, (const u16*)attn_out.data_ptr(), attn_out.stride(0),
           delta.data_ptr<float>());
  return {out, delta};
}

// dX = dy @ w (w [K, N]); with gate_up ([M, 2N], the SwiGLU input saved by the forward) the SwiGLU backward
// is fused: returns dgu [M, 2N] instead of dX. cfg: 14 = the 4-wave ring (csrc/gemm_4w.hip; every plain SmolLM3 /
// Llama dgrad), 7 = 256 x 256 tiles with 64-deep stages (the SwiGLU-backward epilogue: 0.425 vs 0.483 ms for the
// 4-wave kernel's register epilogue, profiles/r6_gemm_routing.md), 5 = the 32-deep ring (K % 64 != 0), 2 = 256 x 128
// tiles (the wave-tail launch below).
at::Tensor dgrad_gemm(const at::Tensor& dy, const at::Tensor& w, const c10::optional<at::Tensor>& gate_up,
                      int64_t cfg) {
  SFT_CHECK_CUDA(dy);
  SFT_CHECK_BF16(dy);
  SFT_CHECK_BF16(w);
  SFT_CHECK(dy.dim() == 2 && w.dim() == 2, "dgrad_gemm: 2-D operands");
  SFT_CHECK(dy.stride(1) == 1 && w.stride(1) == 1, "dgrad_gemm: rows must be contiguous");
  const int64_t M = dy.size(0), K = dy.size(1), N = w.size(1);
  SFT_CHECK(w.size(0) == K, "dgrad_gemm: dy [M, K] . w [K, N]");
  SFT_CHECK(cfg != 7 || K % 64 == 0, "dgrad_gemm cfg 7 (BK 64): K multiple of 64");
  SFT_CHECK(cfg != 14 || K % 128 == 0, "dgrad_gemm cfg 14 (4-wave): K multiple of 128");
  SFT_CHECK(M % 128 == 0 && N % 256 == 0 && K % 32 == 0 && K >= 32, "dgrad_gemm: M multiple of 128 (256 for cfg 0/1), N of 256, K of 32");
  SFT_CHECK(cfg == 2 || M % 256 == 0, "dgrad_gemm: 256 x 256 tiles need M % 256 == 0");
  SFT_CHECK(dy.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && (uintptr_t)dy.data_ptr() % 16 == 0 &&
                (uintptr_t)w.data_ptr() % 16 == 0,
            "dgrad_gemm: 16-byte aligned rows");
  dgrad::EpiArgs ea{};
  ea.N = (int)N;
  at::Tensor out;
  const bool swiglu = gate_up.has_value() && gate_up->defined();
  if (swiglu) {
    const at::Tensor& gu = *gate_up;
    SFT_CHECK_BF16(gu);
    SFT_CHECK_CONTIG(gu);
    SFT_CHECK(gu.dim() == 2 && gu.size(0) == M && gu.size(1) == 2 * N, "dgrad_gemm: gate_up must be [M, 2N]");
    out = at::empty({M, 2 * N}, dy.options());
    ea.gu = (const u16*)gu.data_ptr();
    ea.ldo = 2 * N;
  } else {
    out = at::empty({M, N}, dy.options());
    ea.ldo = N;
  }
  ea.out = (u16*)out.data_ptr();
  if (M == 0 || N == 0) return out;
  // Wave-quantisation tail (256 x 256 configs): with nbn x nbm tiles over 256 CUs the last round is partial —
  // the SmolLM3 down projection has 43 x 32 = 1376 tiles = 5.375 rounds, run as 6. When the leftover n-tiles fit
  // one round as 256 x 128 half tiles, the whole rounds run as one launch over the leading columns and the leftover
  // columns as a second launch of half tiles (5 + 0.5 rounds). Column sub-ranges are plain pointer offsets: the
  // W columns (stride stays N), the output / gate / up columns (ea.N keeps the full width for the up half).
  // SFTAMD_DGRAD_TAIL: 0 = off, 2 = the half-tile config (default).
  auto run1 = [&](auto epi, int c, const at::Tensor& wv, const dgrad::EpiArgs& e) {
    constexpr int E = decltype(epi)::value;
    SFT_TRACE(trace_name(E == dgrad::EPI_SWIGLU_BWD ? "dgrad.swiglu.c" : "dgrad.c", c));
    switch (c) {
      case 2: dgrad::launch<256, 128, 4, 2, 3, E>(dy, wv, e); break;   // 256 x 128 tiles (the wave-tail launch)
      case 5: dgrad::launch<256, 256, 2, 4, 3, E, 1, false>(dy, wv, e); break;  // 32-deep ring: K % 64 != 0
      case 7: dgrad::launch2<256, 256, 2, 4, E>(dy, wv, e); break;      // 64-deep stages: the SwiGLU-backward epilogue
      case 14:  // the 4-wave ring with interleaved issue (csrc/gemm_4w.hip), plain epilogue
        SFT_CHECK(E == dgrad::EPI_PLAIN, "dgrad_gemm cfg 14: plain epilogue only");
        g4_dgrad(dy, wv, e.out, e.ldo);
        break;
      default: SFT_CHECK(false, "dgrad_gemm: cfg ", c, " not built (2, 5, 7, 14)");
    }
  };
  const int tail_cfg = [] {
    const char* e = std::getenv("SFTAMD_DGRAD_TAIL");
    return e && e[0] ? atoi(e) : 2;
  }();
  auto run = [&](auto epi) {
    const long nbn = N / 256, nbm = M / 256, tiles = nbn * nbm;
    const bool full = cfg != 2;
    long main_n = 0;
    if (full && tail_cfg == 2 && tiles % 256 != 0 && 256 % nbm == 0) {
      main_n = tiles / 256 * (256 / nbm);                  // n-tiles of the whole rounds
      if ((nbn - main_n) * (M / 128) > 256) main_n = 0;      // the half tiles must fit one round
    }
    if (main_n <= 0) {
      run1(epi, (int)cfg, w, ea);
      return;
    }
    const long n_split = main_n * 256;
    SFT_TRACE("dgrad.tail");
    run1(epi, (int)cfg, w.narrow(1, 0, n_split), ea);
    dgrad::EpiArgs et = ea;
    et.out = ea.out + n_split;
    if (et.gu != nullptr) et.gu = ea.gu + n_split;
    run1(epi, tail_cfg, w.narrow(1, n_split, N - n_split), et);
  };
  if (swiglu) run(std::integral_constant<int, dgrad::EPI_SWIGLU_BWD>());
  else run(std::integral_constant<int, dgrad::EPI_PLAIN>());
  return out;
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("dgrad_gemm", &dgrad_gemm);
  m.impl("dgrad_gemm_delta", &dgrad_gemm_delta);
}

}  // namespace sftamd
