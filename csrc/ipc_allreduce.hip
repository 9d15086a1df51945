// One-shot intra-node all-reduce over peer-mapped device memory: the optional
// custom collective for small, latency-bound messages (token counts, the clip norm, small buckets), next to RCCL.
//
// Every rank owns one registered region [data: cap bytes][flags]; the regions are exchanged as HIP IPC handles
// (dmabuf) and opened by every peer, so a kernel on rank r can read rank p's data over xGMI (or, for ranks sharing a
// device, from the same HBM). One call, per workgroup b (its own chunk of the message):
//   1. copy the chunk of x into this rank's region;
//   2. release (system scope) and raise flag[r][b] = round in EVERY rank's region;
//   3. wait (acquire, system scope) until flag[p][b] >= round in this rank's region for all p;
//   4. x = sum over p = 0..N-1 of rank p's chunk, in rank order (every rank computes the identical sum);
//   5. raise / wait a second flag set ("done reading") so the next call cannot overwrite a chunk a peer still reads.
// Waits are bounded (s_memrealtime, 100 MHz): a peer that never arrives sets the region's error word instead of
// hanging the device AND poisons this call's output with NaN (a silently wrong sum — e.g. a clip norm that differs
// across ranks — is the failure to avoid); ipc_ar_check() (synchronising) or ipc_ar_poll() (a pinned copy of the
// error word behind each call, read without waiting) report it. Flags and data use vector memory operations only.
// The region is allocated uncached (hipDeviceMallocUncached) so peers polling it over xGMI never hit a stale cached
// line; hipMalloc memory is the fallback when the driver refuses an IPC handle for it.
#include "common.h"

#include <cstring>
#include <vector>

namespace sftamd {
namespace ipcar {

constexpr int MAXW = 8;      // ranks
constexpr int MAXB = 64;     // workgroups (flag slots per rank)
constexpr int NT = 256;
constexpr unsigned long long TIMEOUT_TICKS = 200000000ull;  // 2 s of the 100 MHz real-time counter

struct Peers {
  char* base[MAXW];
};

struct Ctx {
  char* local = nullptr;      // this rank's region
  long cap = 0;               // data bytes
  int world = 0, rank = 0;
  int* err = nullptr;         // device error word
  int* err_host = nullptr;    // pinned copy of it, refreshed behind every call (ipc_ar_poll)
  hipEvent_t ev = nullptr;    // recorded after that copy
  bool uncached = false;
  std::vector<void*> opened;  // peer mappings to close
  Peers peers{};
  bool ready = false;
};

static std::vector<Ctx>& contexts() {
  static std::vector<Ctx> v;
  return v;
}

__device__ __forceinline__ unsigned* flag_ptr(char* base, long cap, int set, int rank, int blk) {
  return (unsigned*)(base + cap) + ((long)set * MAXW + rank) * MAXB + blk;
}

// returns false on timeout
__device__ __forceinline__ bool wait_flags(char* local, long cap, int set, int world, int blk, unsigned round,
                                           int* err) {
  bool ok = true;
  if ((int)threadIdx.x < world) {
    unsigned* f = flag_ptr(local, cap, set, threadIdx.x, blk);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - round) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > TIMEOUT_TICKS) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  return __syncthreads_and(ok);
}

__device__ __forceinline__ void raise_flags(const Peers& peers, long cap, int set, int world, int rank, int blk,
                                            unsigned round) {
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world)
    __hip_atomic_store(flag_ptr(peers.base[threadIdx.x], cap, set, rank, blk), round, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__device__ __forceinline__ void add_vec(float* acc, const uint4& v);
template <>
__device__ __forceinline__ void add_vec<u16>(float* acc, const uint4& v) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] += f[i];
}
template <>
__device__ __forceinline__ void add_vec<float>(float* acc, const uint4& v) {
  acc[0] += __uint_as_float(v.x);
  acc[1] += __uint_as_float(v.y);
  acc[2] += __uint_as_float(v.z);
  acc[3] += __uint_as_float(v.w);
}
template <typename T>
__device__ __forceinline__ uint4 pack_vec(const float* acc);
template <>
__device__ __forceinline__ uint4 pack_vec<u16>(const float* acc) { return pack8(acc); }
template <>
__device__ __forceinline__ uint4 pack_vec<float>(const float* acc) {
  return make_uint4(__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3]));
}

// x: nvec 16-byte vectors (the host pads nothing: numel * esz is a multiple of 16, checked)
template <typename T>
__global__ __launch_bounds__(NT) void allreduce_kernel(uint4* __restrict__ x, long nvec, Peers peers, long cap,
                                                       int world, int rank, unsigned round, int* err) {
  constexpr int E = 16 / sizeof(T);
  const int blk = blockIdx.x, nb = gridDim.x;
  const long per = (nvec + nb - 1) / nb, v0 = blk * per, v1 = min(nvec, v0 + per);
  char* local = peers.base[rank];
  uint4* mine = (uint4*)local;
  for (long i = v0 + threadIdx.x; i < v1; i += NT) mine[i] = x[i];
  raise_flags(peers, cap, 0, world, rank, blk, round);
  if (!wait_flags(local, cap, 0, world, blk, round, err)) {
    for (long i = v0 + threadIdx.x; i < v1; i += NT) x[i] = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
    return;  // NaN output (bf16 and fp32 all-ones = NaN): the caller cannot use a partial sum by accident
  }
  for (long i = v0 + threadIdx.x; i < v1; i += NT) {
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    for (int p = 0; p < world; ++p) add_vec<T>(acc, ((const uint4*)peers.base[p])[i]);
    x[i] = pack_vec<T>(acc);
  }
  raise_flags(peers, cap, 1, world, rank, blk, round);
  wait_flags(local, cap, 1, world, blk, round, err);
}

}  // namespace ipcar

using ipcar::Ctx;
using ipcar::contexts;

// region = cap data bytes + 2 flag sets x MAXW x MAXB x 4 B; returns a context id
int64_t ipc_ar_create(int64_t cap, int64_t world, int64_t rank) {
  SFT_CHECK(world >= 1 && world <= ipcar::MAXW && rank >= 0 && rank < world, "ipc_ar_create: 1 <= world <= 8");
  SFT_CHECK(cap > 0 && cap % 16 == 0, "ipc_ar_create: capacity a positive multiple of 16 bytes");
  Ctx c;
  c.cap = cap;
  c.world = (int)world;
  c.rank = (int)rank;
  const long bytes = cap + 2L * ipcar::MAXW * ipcar::MAXB * 4;
  if (hipExtMallocWithFlags((void**)&c.local, bytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, c.local) == hipSuccess) {
      c.uncached = true;
    } else {
      (void)hipGetLastError();
      C10_HIP_CHECK(hipFree(c.local));
      c.local = nullptr;
    }
  } else {
    (void)hipGetLastError();
    c.local = nullptr;
  }
  if (c.local == nullptr) C10_HIP_CHECK(hipMalloc((void**)&c.local, bytes));
  C10_HIP_CHECK(hipMemset(c.local, 0, bytes));
  C10_HIP_CHECK(hipMalloc((void**)&c.err, sizeof(int)));
  C10_HIP_CHECK(hipMemset(c.err, 0, sizeof(int)));
  C10_HIP_CHECK(hipHostMalloc((void**)&c.err_host, sizeof(int), hipHostMallocDefault));
  *c.err_host = 0;
  C10_HIP_CHECK(hipEventCreateWithFlags(&c.ev, hipEventDisableTiming));
  C10_HIP_CHECK(hipDeviceSynchronize());
  contexts().push_back(c);
  return (int64_t)contexts().size() - 1;
}

static Ctx& ctx_at(int64_t id) {
  SFT_CHECK(id >= 0 && id < (int64_t)contexts().size() && contexts()[id].local != nullptr, "ipc_ar: bad context");
  return contexts()[id];
}

// the IPC handle of this rank's region (64 bytes as an int64 list, exchanged by the caller over the process group)
std::vector<int64_t> ipc_ar_handle(int64_t id) {
  Ctx& c = ctx_at(id);
  hipIpcMemHandle_t h;
  C10_HIP_CHECK(hipIpcGetMemHandle(&h, c.local));
  static_assert(sizeof(h) % 8 == 0, "handle size");
  std::vector<int64_t> out(sizeof(h) / 8);
  std::memcpy(out.data(), &h, sizeof(h));
  return out;
}

// handles: world x (64 / 8) int64, rank-major; the own entry is skipped
void ipc_ar_open(int64_t id, std::vector<int64_t> handles) {
  Ctx& c = ctx_at(id);
  const int per = (int)(sizeof(hipIpcMemHandle_t) / 8);
  SFT_CHECK((int)handles.size() == c.world * per, "ipc_ar_open: world x handle words");
  for (int p = 0; p < c.world; ++p) {
    if (p == c.rank) {
      c.peers.base[p] = c.local;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles.data() + (long)p * per, sizeof(h));
    void* ptr = nullptr;
    C10_HIP_CHECK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
    c.opened.push_back(ptr);
    c.peers.base[p] = (char*)ptr;
  }
  c.ready = true;
}

void ipc_ar_allreduce(at::Tensor x, int64_t id, int64_t round, int64_t blocks) {
  Ctx& c = ctx_at(id);
  SFT_CHECK(c.ready, "ipc_ar_allreduce: ipc_ar_open first");
  SFT_CHECK_CUDA(x);
  SFT_CHECK_CONTIG(x);
  SFT_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "ipc_ar_allreduce: bf16 or fp32");
  const long bytes = x.numel() * x.element_size();
  SFT_CHECK(bytes <= c.cap && bytes % 16 == 0, "ipc_ar_allreduce: message must fit the region, multiple of 16 bytes");
  SFT_CHECK((uintptr_t)x.data_ptr() % 16 == 0, "ipc_ar_allreduce: 16-byte aligned");
  if (bytes == 0) return;
  const long nvec = bytes / 16;
  const int nb = (int)std::max<long>(1, std::min<long>({(long)blocks, (long)ipcar::MAXB, (nvec + 255) / 256}));
  const unsigned r = (unsigned)round;
  if (x.scalar_type() == at::kBFloat16)
    ipcar::allreduce_kernel<u16><<<nb, ipcar::NT, 0, cur_stream()>>>((uint4*)x.data_ptr(), nvec, c.peers, c.cap,
                                                                     c.world, c.rank, r, c.err);
  else
    ipcar::allreduce_kernel<float><<<nb, ipcar::NT, 0, cur_stream()>>>((uint4*)x.data_ptr(), nvec, c.peers, c.cap,
                                                                       c.world, c.rank, r, c.err);
  SFT_LAUNCH_CHECK();
  C10_HIP_CHECK(hipMemcpyAsync(c.err_host, c.err, sizeof(int), hipMemcpyDeviceToHost, cur_stream()));
  C10_HIP_CHECK(hipEventRecord(c.ev, cur_stream()));
}

// the error word as of the last completed call, without waiting: -1 = that call has not finished yet, 0 = ok,
// 1 = a bounded wait timed out (its output was poisoned with NaN)
int64_t ipc_ar_poll(int64_t id) {
  Ctx& c = ctx_at(id);
  const hipError_t q = hipEventQuery(c.ev);
  if (q == hipErrorNotReady) {
    (void)hipGetLastError();
    return -1;
  }
  C10_HIP_CHECK(q);
  return *c.err_host;
}

// 1 if the region is uncached device memory (the fallback is plain hipMalloc)
int64_t ipc_ar_uncached(int64_t id) { return ctx_at(id).uncached ? 1 : 0; }

// device error word (1 = a wait timed out); synchronises the device
int64_t ipc_ar_check(int64_t id) {
  Ctx& c = ctx_at(id);
  int v = 0;
  C10_HIP_CHECK(hipDeviceSynchronize());
  C10_HIP_CHECK(hipMemcpy(&v, c.err, sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

void ipc_ar_destroy(int64_t id) {
  Ctx& c = ctx_at(id);
  C10_HIP_CHECK(hipDeviceSynchronize());
  for (void* p : c.opened) C10_HIP_CHECK(hipIpcCloseMemHandle(p));
  C10_HIP_CHECK(hipFree(c.local));
  C10_HIP_CHECK(hipFree(c.err));
  C10_HIP_CHECK(hipHostFree(c.err_host));
  C10_HIP_CHECK(hipEventDestroy(c.ev));
  c = Ctx{};
}

TORCH_LIBRARY_IMPL(sftamd, CUDA, m) { m.impl("ipc_ar_allreduce", &ipc_ar_allreduce); }

}  // namespace sftamd
