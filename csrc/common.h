// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of the sftamd extension.
// Wave64 everywhere: lane = threadIdx.x & 63; bf16 is handled as raw u16 storage with
// fp32 math; 16-byte vector accesses (8 x bf16) for every streaming kernel (CDNA guide G13).
#pragma once

#include <ATen/ATen.h>
#include <c10/hip/HIPException.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include "cu_budget.h"

#include <cstdint>
#include <string>

namespace sftamd {

typedef unsigned short u16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(u16 u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

// two floats -> two round-to-nearest-even bf16 in one word (low = a): one v_cvt_pk_bf16_f32. Two scalar (__bf16)
// conversions compile to two half-used cvt_pk plus a shift and an or.
__device__ __forceinline__ unsigned pk2bf(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f32x2_t;
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// SwiGLU backward of one element, the rounding pinned (explicit fma, no contraction): dact d, gate g, up u ->
// dgate = d u sg (1 + g (1 - sg)), dup = d g sg with sg = sigmoid(g). Shared by the standalone kernel and the fused
// epilogues that promise bitwise-equal results.
__device__ __forceinline__ void swiglu_grad(float d, float g, float u, float& dg, float& du) {
#pragma clang fp contract(off)
  const float sg = 1.f / (1.f + __expf(-g));
  du = (d * g) * sg;
  dg = ((d * u) * sg) * __builtin_fmaf(g, 1.f - sg, 1.f);
}

// 8 x bf16 in a uint4 <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pk2bf(f[0], f[1]), pk2bf(f[2], f[3]), pk2bf(f[4], f[5]), pk2bf(f[6], f[7]));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based 32-bit hash (murmur3-style finaliser) of a 64-bit element index and a seed: the
// random stream of stochastic rounding and LoRA dropout. Regenerable anywhere (no RNG state).
__device__ __forceinline__ unsigned hash_u32(unsigned long long i, unsigned seed) {
  unsigned x = (unsigned)i * 0x9E3779B9u ^ (unsigned)(i >> 32) * 0x85EBCA6Bu ^ seed * 0xC2B2AE35u;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// Dropout keep bit of element i (LoRA dropout, dropout_add): the even / odd element of each pair shares ONE hash, its
// low / high 16 bits compared against a 16-bit threshold p * 65536 (half the hashing of one hash per element; p is
// resolved to 1 / 65536). Regenerated in backward from (seed, index); twin: ops/reference.py dropout_keep.
__device__ __forceinline__ bool drop_keep(unsigned long long i, unsigned seed, unsigned thresh16) {
  const unsigned h = hash_u32(i >> 1, seed);
  return ((i & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thresh16;
}

// (16-bit keep threshold, 1 / (1 - p)) of a dropout probability (clamped to [0, 0.999])
inline unsigned drop_thresh16(double p, float* scale) {
  const double pc = p < 0 ? 0 : (p > 0.999 ? 0.999 : p);
  *scale = (float)(1.0 / (1.0 - pc));
  return (unsigned)(pc * 65536.0);
}

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline int num_cus() { return kNumCUs; }

#define SFT_CHECK(cond, ...) TORCH_CHECK(cond, "sftamd: ", __VA_ARGS__)
#define SFT_CHECK_CUDA(t) SFT_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define SFT_CHECK_BF16(t) SFT_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define SFT_CHECK_CONTIG(t) SFT_CHECK((t).is_contiguous(), #t " must be contiguous")
#define SFT_LAUNCH_CHECK() C10_HIP_KERNEL_LAUNCH_CHECK()

// dispatch trace (csrc/dispatch_trace.cpp): SFT_TRACE("attn.fwd3") / SFT_TRACE(trace_name("tn.c", cfg))
bool trace_on();
void trace_hit(const std::string& name);
inline std::string trace_name(const char* base, long v) { return std::string(base) + std::to_string(v); }
#define SFT_TRACE(name)                                 \
  do {                                                  \
    if (::sftamd::trace_on()) ::sftamd::trace_hit(name); \
  } while (0)

// Device-side invariant checks, compiled in only by `python build_ext.py --debug` (-DSFTAMD_DEBUG,
// separate _C_debug.so loaded when SFTAMD_DEBUG=1). The release kernels clamp or skip bad inputs
// instead; the debug build names the kernel, block and thread of the first violation and aborts.
// Triage recipe: SFTAMD_DEBUG=1 AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 python ...
#ifdef SFTAMD_DEBUG
#define SFT_DASSERT(cond)                                                                                   \
  do {                                                                                                      \
    if (!(cond)) {                                                                                          \
      printf("sftamd device assert failed: %s at %s:%d (block %d,%d,%d thread %d)\n", #cond, __FILE__,      \
             __LINE__, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x);                \
      __builtin_trap();                                                                                     \
    }                                                                                                       \
  } while (0)
#else
#define SFT_DASSERT(cond) \
  do {                    \
  } while (0)
#endif

}  // namespace sftamd
