// One-shot all-reduce over peer-mapped device memory (the xGMI full mesh of one MI355X node).  SURVEY.md §2.2 /
// §2.4 "optional oneshot_allreduce P2P kernel"; the reference has no distributed path at all
// (DCML_MAT_Train.py:104-106 pins cuda:0).
//
// Why: the data-parallel gradient is ONE flat fp32 buffer of ~0.6 MB per minibatch (parallel/comm.FlatGrads).  A
// ring all-reduce over 8 GPUs takes 2(p-1) = 14 dependent hops of 1/8 of that, each bound by ONE xGMI link and by
// per-hop latency.  On a full mesh every GPU has a direct link to every peer, so each GPU can read its peers'
// buffers directly: one signal round + one read of (p-1) x 0.6 MB spread over all 7 links at once.
//
// Protocol (one launch per all-reduce, G workgroups, each owning the same contiguous slice of the buffer on every
// rank):
//   1. WG b copies its slice of the local gradient into this rank's shared buffer half (epoch parity), then
//      fences at system scope;
//   2. one lane per peer publishes `epoch` into flag[rank][b] of THAT peer's region (release, system scope), and
//      one lane per peer waits for flag[peer][b] >= epoch in this rank's region (acquire, system scope);
//   3. WG b sums slice b of every rank's buffer half in rank order 0..p-1 (so every rank gets bit-identical
//      results) and writes scale * sum to the output.
// Two buffer halves alternate by epoch parity: a rank can only overwrite half (e & 1) at epoch e + 2 after every
// peer signalled epoch e + 1 for the slice, i.e. after every peer's epoch-e kernel (same stream) has finished
// reading it.  Waits are bounded: a missing peer sets the local error word and the kernel exits (never a hang);
// the workgroup writes NaN over its output slice (the optimizer's non-finite guard then skips that step) and sets
// bit 31 of every PEER's error word too, so every rank's host check (`mdl_ar_error` / the asynchronous poll) raises,
// not only the one that timed out.  All cross-GPU traffic uses vector-memory loads / stores / atomics.
#include "common.h"
#include <cstring>

namespace {

constexpr int AR_MAXW = 16;
constexpr int AR_THREADS = 256;

struct ArArgs {
  float* region[AR_MAXW];   // every rank's shared region, mapped into this process (own one included)
  const float* src;         // local input [n]
  float* dst;               // local output [n] (may alias src)
  long long n;              // floats per buffer half
  long long flag_off;       // float offset of the flag array inside a region: flags[sender * G + wg]
  long long err_off;        // float offset of this rank's error word
  long long wait_cycles;    // bound of one peer wait (shader-clock cycles) before the error path
  int world, rank;
  unsigned epoch;
  float scale;
  int vec;                  // 1: src / dst / regions are 16-byte aligned and n % 4 == 0 (float4 path)
};

// Visibility: the publishing workgroup stores its slice with ordinary stores, then every thread fences at system
// scope (L2 write-back) before the barrier and the release-store of the flags; the waiting lanes' acquire-load at
// system scope invalidates this XCD's non-coherent cache lines, and the workgroup barrier orders every thread's
// peer reads after it — so ordinary (float4) loads of the peers' halves see the published data.
__global__ __launch_bounds__(AR_THREADS) void oneshot_allreduce_kernel(ArArgs a) {
  const int G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
  const long long half = (long long)(a.epoch & 1u) * a.n;
  const long long m = a.vec ? a.n >> 2 : a.n;   // items of this launch: float4s or floats
  const long long lo = m * b / G, hi = m * (b + 1) / G;
  // 1. publish this rank's slice
  float* mine = a.region[a.rank] + half;
  if (a.vec) {
    const float4* s4 = reinterpret_cast<const float4*>(a.src);
    float4* d4 = reinterpret_cast<float4*>(mine);
    for (long long i = lo + tid; i < hi; i += AR_THREADS) d4[i] = s4[i];
  } else {
    for (long long i = lo + tid; i < hi; i += AR_THREADS) mine[i] = a.src[i];
  }
  __threadfence_system();
  __syncthreads();
  // 2. signal every peer, then wait for every peer's signal for this slice
  __shared__ int timed_out;
  if (tid == 0) timed_out = 0;
  __syncthreads();
  if (tid < a.world) {
    unsigned* f = reinterpret_cast<unsigned*>(a.region[tid] + a.flag_off) + (long long)a.rank * G + b;
    __hip_atomic_store(f, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* w = reinterpret_cast<unsigned*>(a.region[a.rank] + a.flag_off) + (long long)tid * G + b;
    const long long t0 = clock64();
    while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
      __builtin_amdgcn_s_sleep(4);
      if (clock64() - t0 > a.wait_cycles) {   // a peer never arrived: flag the error, poison the slice
        // bits 0..15 = the peer this rank waited for (world <= 16); bit 31 is reserved for "a peer timed out"
        __hip_atomic_fetch_or(reinterpret_cast<unsigned*>(a.region[a.rank] + a.err_off), 1u << (tid & 15),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = 1;
        break;
      }
    }
  }
  __syncthreads();
  if (timed_out && tid < a.world && tid != a.rank) {
    // tell EVERY peer (bit 31 of its error word): a peer whose own waits succeeded has applied this step, but its
    // next poll raises too, so all ranks stop together instead of training on diverged replicas
    // system scope like every other cross-GPU access here: the peer's host poll sees it without waiting for the end
    // of this kernel's write-back
    __hip_atomic_fetch_or(reinterpret_cast<unsigned*>(a.region[tid] + a.err_off), 0x80000000u | (1u << (a.rank & 15)),
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (timed_out) {   // NaN output: FlatAdam's non-finite guard skips the step instead of applying a partial sum
    for (long long i = (a.vec ? 4 * lo : lo) + tid; i < (a.vec ? 4 * hi : hi); i += AR_THREADS) a.dst[i] = __int_as_float(0x7fc00000);
    return;
  }
  // 3. reduce the slice over ranks in a fixed order
  if (a.vec) {
    float4* d4 = reinterpret_cast<float4*>(a.dst);
    for (long long i = lo + tid; i < hi; i += AR_THREADS) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < a.world; ++r) {
        const float4 x = reinterpret_cast<const float4*>(a.region[r] + half)[i];
        s.x += x.x;
        s.y += x.y;
        s.z += x.z;
        s.w += x.w;
      }
      d4[i] = make_float4(s.x * a.scale, s.y * a.scale, s.z * a.scale, s.w * a.scale);
    }
  } else {
    for (long long i = lo + tid; i < hi; i += AR_THREADS) {
      float s = 0.f;
      for (int r = 0; r < a.world; ++r) s += a.region[r][half + i];
      a.dst[i] = s * a.scale;
    }
  }
}

long long flag_off_of(long long n) { return 2 * n; }
long long err_off_of(long long n, int G) { return 2 * n + (long long)AR_MAXW * G; }
size_t region_bytes(long long n, int G) { return (size_t)(err_off_of(n, G) + 64) * sizeof(float); }

}  // namespace

// region for n floats and G workgroups (zeroed)
MDL_API int mdl_ar_alloc(long long n, int G, void** out) {
  if (n <= 0 || G <= 0) return -1;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, region_bytes(n, G));
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, region_bytes(n, G));
  if (e != hipSuccess) return (int)e;
  *out = p;
  return 0;
}

MDL_API int mdl_ar_free(void* p) { return (int)hipFree(p); }

MDL_API int mdl_ar_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

MDL_API int mdl_ar_ipc_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  memcpy(out, &h, sizeof(h));
  return 0;
}

MDL_API int mdl_ar_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

MDL_API int mdl_ar_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

MDL_API int mdl_ar_run(void* const* regions, int world, int rank, const float* src, float* dst, long long n, int G,
                       unsigned epoch, float scale, long long wait_cycles, hipStream_t st) {
  if (world < 1 || world > AR_MAXW || rank < 0 || rank >= world || n <= 0 || G <= 0 || epoch == 0) return -1;
  ArArgs a{};
  bool aligned = (n & 3) == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0;
  for (int r = 0; r < world; ++r) {
    if (!regions[r]) return -2;
    a.region[r] = static_cast<float*>(regions[r]);
    aligned = aligned && ((uintptr_t)regions[r] & 15) == 0;
  }
  a.vec = aligned ? 1 : 0;
  a.src = src;
  a.dst = dst;
  a.n = n;
  a.flag_off = flag_off_of(n);
  a.err_off = err_off_of(n, G);
  a.world = world;
  a.rank = rank;
  a.epoch = epoch;
  a.scale = scale;
  a.wait_cycles = wait_cycles;
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3(G), dim3(AR_THREADS), 0, st, a);
  MDL_CHECK_LAUNCH();
  return 0;
}

// this rank's error word (synchronous read): nonzero = some peer never signalled within wait_cycles
MDL_API int mdl_ar_error(void* region, long long n, int G, unsigned* out) {
  return (int)hipMemcpy(out, static_cast<float*>(region) + err_off_of(n, G), sizeof(unsigned), hipMemcpyDeviceToHost);
}

// the same word copied asynchronously on `st` into host-visible memory (pinned): the trainer polls it once per
// iteration without a device synchronisation (parallel/oneshot.OneShotAllReduce.poll)
MDL_API int mdl_ar_error_async(void* region, long long n, int G, unsigned* out_host, hipStream_t st) {
  return (int)hipMemcpyAsync(out_host, static_cast<float*>(region) + err_off_of(n, G), sizeof(unsigned),
                             hipMemcpyDeviceToHost, st);
}
