// Weight-gradient GEMMs for gfx950: dW[N, K] (+)= dy[T, N]^T @ x[T, K], bf16 in, fp32 accumulate, written (or
// accumulated, beta = 1) straight into the bf16 flat gradient buffer, with optional gradient-norm partials of the
// stored values.
//
// Why hand-written kernels: both operands of a weight gradient are stored "reduction-major" (the token index T is the
// ROW index of dy and of x), the layout that hipBLASLt/rocBLAS run at ~1.0 PF/s on MI355X for the SmolLM3 shapes (NT
// in BLAS terms, profiles/), against ~1.4 PF/s for the forward (TN) GEMMs. On CDNA4 that layout costs nothing extra:
// the tiles are staged row-major into LDS exactly as they sit in HBM (LDS-DMA, 16 B per lane, no register round
// trip) and BOTH MFMA operands are read with the gfx950 transposed LDS read ds_read_b64_tr_b16.
//
// Variants (wgrad_gemm cfg = 1000 H + 100 S + c):
//   c = 14  the 4-wave 256 x 256 ring of csrc/gemm_4w.hip — every SmolLM3 / Llama shape with N, K % 256, T % 128;
//   c = 9   the 8-wave ring below, 256 x 128 tiles (K % 128 only, or T % 128 != 0);
//   c = 10  the 8-wave ring below, 256 x 256 tiles;
//   S >= 2  tiles split S ways over the token axis into fp32 slabs + the ordered fixup (deterministic): every tile
//           (H = 0; small grids such as o_proj's 64 tiles) or only the tiles past the last whole round of 256
//           workgroups (H = 1, hybrid).
//
// The 8-wave ring: BM x BN output tile per 512-thread workgroup (8 waves), 32 tokens per stage, NS stages of LDS-DMA
// in flight; LDS images are [32 tokens][128 columns] bf16 (256-byte rows) with the chunk XOR swizzle
// ch ^ ((row&3)<<2 | (row>>2)&3), applied on the GLOBAL source address (the DMA writes lane-linear), which keeps the
// transposed reads bank-conflict free; v_mfma_f32_16x16x32_bf16; XCD-aware workgroup remap; epilogue through LDS
// (fp32, padded rows) so the beta-accumulate read-modify-write of the bf16 gradient is 16-byte vectorised.
#include "common.h"
#include "g4_api.h"
#include "splitk_fixup.h"

#include <type_traits>

namespace sftamd {
namespace wgrad {

constexpr int ROWB = 256;             // bytes per LDS image row (128 bf16)
constexpr int NT = 512;

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ (((row & 3) << 2) | ((row >> 2) & 3)); }
__device__ __forceinline__ int img_off(int row, int ch) { return row * ROWB + 16 * swz(row, ch); }

typedef __attribute__((address_space(3))) s16x4 lds_s4;

__device__ __forceinline__ bf16x8 lds_tr(const char* base, int off) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + off));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + off + 16 * ROWB));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void glds16(const u16* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
}

// Epilogue: fp32 wave tile -> LDS (rows padded to TN + 4 floats: conflict-free) -> 16-byte
// read-modify-write of the bf16 gradient (beta = 1 when accumulating, else plain store).
// ``nrm`` (optional): this wave's slot of the gradient-norm partials — the fp32 sum of squares of the values
// it stores (before bf16 rounding; the FINAL gradient when this is the last contribution of the step), so the
// clip norm needs no separate pass over the gradient.
template <class G>
__device__ __forceinline__ void epilogue(char* smem, f32x4 (&acc)[G::FM][G::FN], u16* __restrict__ C, int K, int n0,
                                         int k0, int wm, int wk, int w, int lane, int accumulate,
                                         float* __restrict__ nrm = nullptr) {
  const int g = lane >> 4, ii = lane & 15;
  float ss = 0.f;
  float* ep = reinterpret_cast<float*>(smem) + w * G::EPI_ROWS * G::EPI_LD;
  constexpr int FPP = G::EPI_ROWS / 16 < G::FM ? G::EPI_ROWS / 16 : G::FM;  // fragments per pass
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
    constexpr int SEGS = G::TN / 8;                      // 16-byte output segments per row
#pragma unroll
    for (int it = 0; it < ROWS * SEGS / 64; ++it) {
      const int seg = it * 64 + lane, row = seg / SEGS, cs = seg - row * SEGS;
      const float* pr = ep + row * G::EPI_LD + cs * 8;
      float v[8];
      *(float4*)&v[0] = *(const float4*)pr;
      *(float4*)&v[4] = *(const float4*)(pr + 4);
      u16* out = C + (long)(n0 + wm * G::TM + pass * ROWS + row) * K + k0 + wk * G::TN + cs * 8;
      if (accumulate) {
        float o[8];
        unpack8(*(const uint4*)out, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += o[e];
      }
      if (nrm != nullptr) {  // fp32 values before the bf16 store: no extra registers (the 256x256 ring kernel
#pragma unroll             // sits at 256 VGPRs; unpacking the stored bf16 made it spill inside its main loop)
        for (int e = 0; e < 8; ++e) ss += v[e] * v[e];
      }
      *(uint4*)out = pack8(v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (nrm != nullptr) {
    ss = wave_sum(ss);
    if (lane == 0) *nrm = ss;
  }
}

// ============================================================================================
// The 8-wave ring: BK = 32 tokens per stage, NS stages (up to all 160 KB of LDS), the LDS-DMA of a
// stage issued NS-1 steps before it is read (a 64-token two-stage loop kept only one 64 KB K-tile in
// flight per CU and measured load-latency bound: 1.46x faster without its loads). Per 32-token step:
//   wait vmcnt((NS-2) x pieces) -> step t+1 landed; lgkmcnt(0) -> this wave's reads of slot t done
//   barrier; glds step t+NS -> slot t % NS; ds_read fragments of step t+1; MFMA on step t (regs).
// ============================================================================================
constexpr int BKR = 32;
constexpr int IMGR = BKR * ROWB;  // 8 KB per [32][128] image

template <int BM, int BN, int WM, int WN, int NS_>
struct RCfg {
  static constexpr int NS = NS_;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int IA = BM / 128, IB = BN / 128, NIMG = IA + IB;
  static constexpr int STAGE = NIMG * IMGR;
  static constexpr int PPW = NIMG;  // one 1 KB piece (rows 4w..4w+3) per image per wave
  static constexpr int EPI_ROWS = 64, EPI_LD = TN + 4;
  static constexpr int EPI = 8 * EPI_ROWS * EPI_LD * 4;
  static constexpr int LDS = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  static_assert(WM * WN == 8 && NS >= 3 && NS <= 6, "ring config");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <class G>
struct RStager {
  const u16* pa;
  const u16* pb;
  long lda, ldb;
  int w, left;
  __device__ __forceinline__ void init(const u16* A, const u16* B, int N, int K, int n0, int k0, int wave, int lane,
                                       int nsteps, int t0 = 0) {
    w = wave;
    lda = N;
    ldb = K;
    left = nsteps;
    const int r = 4 * wave + (lane >> 4), c = lane & 15;
    pa = A + (long)(t0 + r) * N + n0 + 8 * swz(r, c);
    pb = B + (long)(t0 + r) * K + k0 + 8 * swz(r, c);
  }
  // Past the last step the same (valid) rows are fetched again into a slot nobody reads: every
  // step then issues exactly PPW DMAs, so the counted waits are compile-time constants with no
  // tail branches (a branch around a wait makes the compiler's own waitcnt pass assume the
  // no-wait path and drain lgkmcnt before the next MFMA block).
  __device__ __forceinline__ void piece(char* buf, int j) {
    const u16* p = j < G::IA ? pa + j * 128 : pb + (j - G::IA) * 128;
    glds16(p, buf + j * IMGR + w * 1024);
  }
  __device__ __forceinline__ void advance() {
    if (--left > 0) {
      pa += BKR * lda;
      pb += BKR * ldb;
    }
  }
  __device__ __forceinline__ void issue(char* buf) {
#pragma unroll
    for (int j = 0; j < G::NIMG; ++j) piece(buf, j);
    advance();
  }
};

template <class G>
__device__ __forceinline__ void rread(const char* base, const int (&offA)[G::FM], const int (&offB)[G::FN],
                                      bf16x8 (&af)[G::FM], bf16x8 (&bf)[G::FN]) {
#pragma unroll
  for (int j = 0; j < G::FN; ++j) bf[j] = lds_tr(base, offB[j]);
#pragma unroll
  for (int i = 0; i < G::FM; ++i) af[i] = lds_tr(base, offA[i]);
}

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

constexpr unsigned waitcnt_imm(int vm, int lgkm) {  // gfx9: vmcnt[3:0] expcnt[6:4] lgkmcnt[11:8] vmcnt[5:4]<<14
  return (unsigned)((vm & 15) | (7 << 4) | ((lgkm & 15) << 8) | ((vm >> 4) << 14));
}

// The stage pointers are separate __restrict__ parameters: once inlined, every ds_read and every
// LDS-DMA write carries the alias scope of its stage, so the compiler's waitcnt pass only waits for
// DMA into the slot being read (which the explicit counted wait already retired).
//
// Registers: the B fragments of the next step are double-buffered (read at the start of a step),
// the A fragments are refilled in place — fragment row i of step t+1 is read right after the four
// MFMAs of row i of step t, so it still has a whole step of MFMAs to land — which keeps the kernel
// at ~216 VGPRs (2 waves per SIMD) with every MFMA operand already resident.
template <class G, bool SCHED>
__device__ __forceinline__ void ring_loop(char* __restrict__ b0, char* __restrict__ b1, char* __restrict__ b2,
                                          char* __restrict__ b3, char* __restrict__ b4, char* __restrict__ b5,
                                          int nsteps, RStager<G>& st, const int (&offA)[G::FM],
                                          const int (&offB)[G::FN], f32x4 (&acc)[G::FM][G::FN]) {
  constexpr int NS = G::NS, PPW = G::PPW;
  constexpr int U = (NS % 2) ? 2 * NS : NS;  // unroll: stage slot and B register set both compile-time
  bf16x8 fa[G::FM], fb[2][G::FN];
#pragma unroll
  for (int i = 0; i < NS; ++i) st.issue(pick(i, b0, b1, b2, b3, b4, b5));
  __builtin_amdgcn_s_waitcnt(waitcnt_imm((NS - 1) * PPW, 0));
  __builtin_amdgcn_s_barrier();
  rread<G>(b0, offA, offB, fa, fb[0]);
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
        for (int j = 0; j < G::FN; ++j) fb[cb ^ 1][j] = lds_tr(nxt, offB[j]);
        __builtin_amdgcn_s_setprio(1);
        // one LDS-DMA piece after each of the first NIMG fragment rows: the DMA issue cost is
        // spread between MFMA groups instead of stalling every wave right after the barrier
#pragma unroll
        for (int i = 0; i < G::FM; ++i) {
#pragma unroll
          for (int j = 0; j < G::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[cb][j], acc[i][j], 0, 0, 0);
          fa[i] = lds_tr(nxt, offA[i]);
          if (i < G::NIMG) st.piece(dst, i);
          if (SCHED) {
            __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);      // DS read (one fragment)
            if (i < G::NIMG) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (the DMA)
          }
        }
        st.advance();
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 0));  // drain the tail DMAs before LDS is reused
}

// Split-K epilogue: the fp32 wave tile goes straight to this piece's tile-local slab P[BM][BN] (no bf16
// rounding, no read of C); splitk_fixup_kernel sums a tile's slabs in a fixed order (deterministic).
template <class G, int BN>
__device__ __forceinline__ void epilogue_partial(f32x4 (&acc)[G::FM][G::FN], float* __restrict__ P, int wm, int wk,
                                                 int lane) {
  const int g = lane >> 4, ii = lane & 15;
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        P[(wm * G::TM + 16 * i + 4 * g + e) * BN + wk * G::TN + 16 * j + ii] = acc[i][j][e];
}

template <int BM, int BN, int WM, int WN, int NS, bool SCHED, bool NORM = false>
__global__ void __launch_bounds__(NT) ring_kernel(const u16* __restrict__ A, const u16* __restrict__ B,
                                                  u16* __restrict__ C, int T, int N, int K, int nbk, int flags,
                                                  float* __restrict__ P, int ndp, int splits, int tile0 = 0) {
  // flags: bit 0 = accumulate into C, bit 1 = write gradient-norm partials of the whole tiles (8 per tile) to
  // P (no split) or past the split slabs (no extra kernel argument: one more pointer costs this 256-VGPR kernel
  // spills inside its main loop)
  using G = RCfg<BM, BN, WM, WN, NS>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  // whole tiles = blocks [0, ndp) (XCD-aware remap among them), split pieces = the blocks after them: by block index,
  // so the whole tiles fill the first dispatch rounds and the short pieces the last (csrc/gemm_4w.hip)
  const int orig = blockIdx.x;
  int wgid = orig;
  if (orig < ndp) {
    const int nd = min(ndp, (int)gridDim.x), xcd = orig & 7, q8 = nd >> 3, r8 = nd & 7;
    wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  }
  // Hybrid data-parallel + split-K: workgroups [0, ndp) own whole tiles (direct epilogue); the remaining
  // tiles (the partial last wave) are each split `splits` ways over the token axis — consecutive workgroups,
  // uneven step ranges allowed — into fp32 slabs reduced by splitk_fixup_kernel.
  const int nall = T / BKR;
  int tile = tile0 + wgid, sk = 0, s0 = 0, s1 = nall;  // tile0: a tail launch's first tile (DP only)
  if (wgid >= ndp) {
    const int j = wgid - ndp;
    sk = j % splits;
    tile = ndp + j / splits;
    s0 = (int)((long)sk * nall / splits);
    s1 = (int)((long)(sk + 1) * nall / splits);
  }
  const int bn = tile / nbk, bk = tile - bn * nbk;
  const int n0 = bn * BM, k0 = bk * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wk = w - wm * WN;
  const int nsteps = s1 - s0;

  RStager<G> st;
  st.init(A, B, N, K, n0, k0, w, lane, nsteps, s0 * BKR);
  const int g = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
  const int r0 = 4 * (((g & 1) << 1) | (g >> 1)) + qq;  // conflict-free block order (see wgrad_kernel)
  int offA[G::FM], offB[G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i) {
    const int nl = wm * G::TM + 16 * i;
    offA[i] = (nl >> 7) * IMGR + img_off(r0, 2 * ((nl & 127) >> 4) + (pp >> 1)) + 8 * (pp & 1);
  }
#pragma unroll
  for (int j = 0; j < G::FN; ++j) {
    const int kl = wk * G::TN + 16 * j;
    offB[j] = (G::IA + (kl >> 7)) * IMGR + img_off(r0, 2 * ((kl & 127) >> 4) + (pp >> 1)) + 8 * (pp & 1);
  }
  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* b[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) b[i] = smem + (i < NS ? i : 0) * G::STAGE;
  ring_loop<G, SCHED>(b[0], b[1], b[2], b[3], b[4], b[5], nsteps, st, offA, offB, acc);
  if (wgid >= ndp) {
    epilogue_partial<G, BN>(acc, P + ((long)(tile - ndp) * splits + sk) * BM * BN, wm, wk, lane);
    return;
  }
  __syncthreads();
  float* nrm = nullptr;  // wave-uniform (scalar) pointer: no VGPRs
  if (NORM && (flags & 2))
    nrm = (splits <= 1 ? P : P + (long)(gridDim.x - ndp) * BM * BN) + tile * 8 + __builtin_amdgcn_readfirstlane(w);
  epilogue<G>(smem, acc, C, K, n0, k0, wm, wk, w, lane, flags & 1, nrm);
}

// Gradient-norm slots a ring launch writes (norm partials): 8 per whole tile, one per fixup block of a split tile.
static long ring_norm_slots(int tiles, int ndp, int BM, int BN) { return (long)ndp * 8 + (long)(tiles - ndp) * BM * BN / 2048; }

// splits > 1: tiles beyond the first `full_waves` x 256 (or all of them when full_waves == 0) are split over the
// token axis; full_waves < 0 = split every tile.
template <int BM, int BN, int WM, int WN, int NS, bool SCHED = false>
void launch_ring(const at::Tensor& dy, const at::Tensor& x, at::Tensor& out, bool accumulate, int splits = 1,
                 bool hybrid = false, float* nrm = nullptr, long nrm_cap = 0) {
  const int T = dy.size(0), N = dy.size(1), K = x.size(1);
  const int nbn = N / BM, nbk = K / BN, tiles = nbn * nbk;
  const int ndp = splits <= 1 ? tiles : (hybrid ? tiles / 256 * 256 : 0);
  const int nsk = tiles - ndp;
  SFT_CHECK(nrm == nullptr || ring_norm_slots(tiles, ndp, BM, BN) <= nrm_cap, "wgrad_gemm: norm slot buffer too small");
  at::Tensor part;
  if (nsk > 0)  // tile-local fp32 slabs, one per split piece (stream-ordered caching allocation) [+ whole-tile norms]
    part = at::empty({(long)nsk * splits * BM * BN + (nrm != nullptr ? (long)ndp * 8 : 0)}, dy.options().dtype(at::kFloat));
  float* P = nsk > 0 ? part.data_ptr<float>() : nrm;
  const int flags = (accumulate ? 1 : 0) | (nrm != nullptr ? 2 : 0);
  // NORM: separate instantiation, so the plain kernel keeps its register allocation; at 256 x 256 without the
  // pinned MFMA / DMA interleave (with it the allocator spills inside the main loop: 14 reloads vs 1)
  constexpr bool SCHED_N = BN == 256 ? false : SCHED;
  if (nrm != nullptr)
    ring_kernel<BM, BN, WM, WN, NS, SCHED_N, true><<<ndp + nsk * splits, NT, 0, cur_stream()>>>(
        (const u16*)dy.data_ptr(), (const u16*)x.data_ptr(), (u16*)out.data_ptr(), T, N, K, nbk, flags, P, ndp, splits);
  else
    ring_kernel<BM, BN, WM, WN, NS, SCHED><<<ndp + nsk * splits, NT, 0, cur_stream()>>>(
        (const u16*)dy.data_ptr(), (const u16*)x.data_ptr(), (u16*)out.data_ptr(), T, N, K, nbk, flags, P, ndp, splits);
  SFT_LAUNCH_CHECK();
  if (nsk > 0) {
    const long n8 = (long)nsk * BM * BN / 8;
    splitk_fixup_kernel<BM, BN><<<(unsigned)((n8 + 255) / 256), 256, 0, cur_stream()>>>(
        part.data_ptr<float>(), (u16*)out.data_ptr(), ndp, nsk, splits, nbk, K, accumulate ? 1 : 0, nrm);
    SFT_LAUNCH_CHECK();
  }
}

}  // namespace wgrad

void g4_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor& out, bool accumulate, int splits, bool hybrid,
              float* nrm, long nrm_cap);

// cfg: see the header. norm (optional, fp32, contiguous): gradient-norm partial slots — every slot the launch owns is
// written, the rest are left untouched (the caller zeroes the buffer once per step).
void wgrad_gemm(at::Tensor out, at::Tensor dy, at::Tensor x, bool accumulate, int64_t cfg,
                const c10::optional<at::Tensor>& norm) {
  SFT_CHECK_CUDA(dy);
  SFT_CHECK_BF16(dy);
  SFT_CHECK_BF16(x);
  SFT_CHECK_BF16(out);
  SFT_CHECK_CONTIG(dy);
  SFT_CHECK_CONTIG(out);
  SFT_CHECK(dy.dim() == 2 && x.dim() == 2 && out.dim() == 2, "wgrad_gemm: 2-D operands");
  // x may have a padded row pitch (a [T, K] view into a wider buffer) on the 4-wave kernel
  SFT_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.stride(0) >= x.size(1), "wgrad_gemm: x rows contiguous");
  SFT_CHECK(x.stride(0) == x.size(1) || cfg % 100 == 14, "wgrad_gemm: a padded x pitch needs cfg 14");
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  SFT_CHECK(x.size(0) == T && out.size(0) == N && out.size(1) == K, "wgrad_gemm: shape mismatch");
  SFT_CHECK(T % 32 == 0 && T > 0, "wgrad_gemm: T must be a positive multiple of 32");
  SFT_TRACE(trace_name("wgrad.c", cfg));
  if (norm.has_value() && norm->defined()) SFT_TRACE("wgrad.norm_slots");
  const bool hybrid = cfg >= 1000;
  const int splits = (int)((cfg % 1000) / 100);
  SFT_CHECK(cfg < 2000, "wgrad_gemm: cfg ", cfg, " not built");
  cfg %= 100;
  SFT_CHECK(cfg == 9 || cfg == 10 || cfg == 14, "wgrad_gemm: cfg ", cfg, " not built (9, 10, 14)");
  SFT_CHECK(splits <= 1 || T / 32 >= splits, "wgrad_gemm split-K: at least one 32-token step per split");
  float* nrm = nullptr;
  long nrm_cap = 0;
  if (norm.has_value() && norm->defined()) {
    SFT_CHECK(norm->scalar_type() == at::kFloat && norm->is_contiguous() && norm->is_cuda(), "wgrad_gemm: fp32 norm slots");
    nrm = norm->data_ptr<float>();
    nrm_cap = norm->numel();
  }
  if (cfg == 14) {  // 4 waves of 128 x 128, AGPR accumulators (csrc/gemm_4w.hip)
    g4_wgrad(dy, x, out, accumulate, splits, hybrid, nrm, nrm_cap);
    return;
  }
  if (cfg == 10) {
    SFT_CHECK(N % 256 == 0 && K % 256 == 0, "wgrad_gemm ring 256x256: N, K multiples of 256");
    wgrad::launch_ring<256, 256, 2, 4, 5, true>(dy, x, out, accumulate, splits, hybrid, nrm, nrm_cap);
  } else {
    SFT_CHECK(N % 256 == 0 && K % 128 == 0, "wgrad_gemm ring 256x128: N multiple of 256, K of 128");
    if (splits > 1) wgrad::launch_ring<256, 128, 4, 2, 6, true>(dy, x, out, accumulate, splits, hybrid, nrm, nrm_cap);
    else wgrad::launch_ring<256, 128, 4, 2, 6>(dy, x, out, accumulate, 1, false, nrm, nrm_cap);
  }
}

void g4_wgrad_pair(const at::Tensor& dy0, const at::Tensor& x0, at::Tensor& out0, bool acc0, float* nrm0, long cap0,
                   const at::Tensor& dy1, const at::Tensor& x1, at::Tensor& out1, bool acc1, float* nrm1, long cap1,
                   int split_all);

// Two weight gradients over the same tokens in ONE 4-wave launch (e.g. the MLP's down and gate_up: 344 + 688 tiles =
// 4.03 rounds instead of 1.34 + 2.69 with a partial last round each; csrc/gemm_4w.hip g4_wgrad_pair).
void wgrad_gemm_pair(at::Tensor out0, at::Tensor dy0, at::Tensor x0, bool acc0, const c10::optional<at::Tensor>& norm0,
                     at::Tensor out1, at::Tensor dy1, at::Tensor x1, bool acc1,
                     const c10::optional<at::Tensor>& norm1, int64_t split_all) {
  SFT_CHECK_CUDA(dy0);
  SFT_CHECK_BF16(out0);
  SFT_CHECK_BF16(dy0);
  SFT_CHECK_BF16(x0);
  SFT_CHECK_BF16(out1);
  SFT_CHECK_BF16(dy1);
  SFT_CHECK_BF16(x1);
  SFT_CHECK_CONTIG(dy0);
  SFT_CHECK_CONTIG(dy1);
  SFT_CHECK_CONTIG(out0);
  SFT_CHECK_CONTIG(out1);
  SFT_CHECK(x0.dim() == 2 && x0.stride(1) == 1 && x0.stride(0) % 8 == 0 && x0.stride(0) >= x0.size(1) &&
                x1.dim() == 2 && x1.stride(1) == 1 && x1.stride(0) % 8 == 0 && x1.stride(0) >= x1.size(1),
            "wgrad_gemm_pair: x rows contiguous");
  SFT_CHECK(out0.size(0) == dy0.size(1) && out0.size(1) == x0.size(1) && out1.size(0) == dy1.size(1) &&
                out1.size(1) == x1.size(1), "wgrad_gemm_pair: shape mismatch");
  auto slots = [](const c10::optional<at::Tensor>& n, float*& p, long& cap) {
    p = nullptr;
    cap = 0;
    if (n.has_value() && n->defined()) {
      SFT_CHECK(n->scalar_type() == at::kFloat && n->is_contiguous() && n->is_cuda(), "wgrad_gemm_pair: fp32 norm slots");
      p = n->data_ptr<float>();
      cap = n->numel();
    }
  };
  float *n0, *n1;
  long c0, c1;
  slots(norm0, n0, c0);
  slots(norm1, n1, c1);
  SFT_TRACE("wgrad.pair");
  if (n0 != nullptr || n1 != nullptr) SFT_TRACE("wgrad.norm_slots");
  SFT_CHECK(split_all >= 0 && split_all <= 8, "wgrad_gemm_pair: split_all 0..8");
  g4_wgrad_pair(dy0, x0, out0, acc0, n0, c0, dy1, x1, out1, acc1, n1, c1, (int)split_all);
}

// Up to four weight gradients over the same tokens in ONE 4-wave launch (csrc/gemm_4w.hip g4_wgrad_multi), e.g. a
// layer's down + gate_up with the next layer's o_proj + qkv: 1192 tiles = 4 whole rounds + 168 tiles split
// split_left ways (0: the hybrid rule), against 4 rounds + 8 split tiles and a separate 2-round grid of third-tiles.
// norms[i] with numel 0 = no norm slots for problem i.
void wgrad_gemm_multi(at::TensorList outs, at::TensorList dys, at::TensorList xs, at::IntArrayRef accs,
                      at::TensorList norms, int64_t split_all, int64_t split_left) {
  const size_t n = outs.size();
  SFT_CHECK(n >= 1 && n <= 4 && dys.size() == n && xs.size() == n && accs.size() == n && norms.size() == n,
            "wgrad_gemm_multi: 1..4 problems, one of each argument per problem");
  SFT_CHECK(split_all >= 0 && split_all <= 8 && split_left >= 0 && split_left <= 8, "wgrad_gemm_multi: splits 0..8");
  std::vector<WgradJob> jobs;
  bool any_norm = false;
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor &out = outs[i], &dy = dys[i], &x = xs[i], &nr = norms[i];
    SFT_CHECK_CUDA(dy);
    SFT_CHECK_BF16(out);
    SFT_CHECK_BF16(dy);
    SFT_CHECK_BF16(x);
    SFT_CHECK_CONTIG(dy);
    SFT_CHECK_CONTIG(out);
    SFT_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.stride(0) >= x.size(1),
              "wgrad_gemm_multi: x rows contiguous");
    SFT_CHECK(out.size(0) == dy.size(1) && out.size(1) == x.size(1), "wgrad_gemm_multi: shape mismatch");
    float* np = nullptr;
    long cap = 0;
    if (nr.defined() && nr.numel() > 0) {
      SFT_CHECK(nr.scalar_type() == at::kFloat && nr.is_contiguous() && nr.is_cuda(), "wgrad_gemm_multi: fp32 norm slots");
      np = nr.data_ptr<float>();
      cap = nr.numel();
      any_norm = true;
    }
    jobs.push_back(WgradJob{dy, x, out, accs[i] != 0, np, cap});
  }
  SFT_TRACE(trace_name("wgrad.multi", (int)n));
  if (any_norm) SFT_TRACE("wgrad.norm_slots");
  g4_wgrad_multi(jobs, (int)split_all, (int)split_left);
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) {
  m.impl("wgrad_gemm", &wgrad_gemm);
  m.impl("wgrad_gemm_pair", &wgrad_gemm_pair);
  m.impl("wgrad_gemm_multi", &wgrad_gemm_multi);
}

}  // namespace sftamd
