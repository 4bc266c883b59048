// Micro-benchmark: where do the backward's fp32 no-return atomics execute?  The training backward's traffic (256
// workgroups x 8 waves, 22 matrices x 3 chunks, 4-row x 64 B wave-instructions) into a 32-copy workspace, with
//   place 0: copy = blockIdx % 32   (every copy written by ONE XCD: dispatch is round-robin over the 8 XCDs)
//   place 1: copy = (blockIdx / 8) % 32  (every copy written by all 8 XCDs)
//   place 2: copy = blockIdx % 8    (8 copies, one per XCD)
// and scope 0: atomicAdd (agent scope), 1: workgroup-scope __hip_atomic_fetch_add.  If the atomics ran in each
// XCD's L2, place 1 would lose updates (or be slow) and place 0 / 2 would be fast; equal times = memory-side unit.
// The final sum of every element is checked against the expected count.
// Build: hipcc -O3 --offload-arch=gfx950 tests/native/atomic_place_bench.hip -o tests/native/atomic_place_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int NMAT = 22, CHUNKS = 3, COPIES = 32, WAVES = 8, NBLK = 256;

__global__ __launch_bounds__(512) void atom_kernel(float* ws, int place, int scope, float v) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int copy = place == 0 ? blockIdx.x % COPIES : place == 1 ? (blockIdx.x / 8) % COPIES : blockIdx.x % 8;
  float* base = ws + (size_t)copy * NMAT * 4096;
  const int g = lane >> 4, c = lane & 15;
  for (int ch = 0; ch < CHUNKS; ++ch)
    for (int m = 0; m < NMAT; ++m) {
      float* M = base + m * 4096;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = 16 * (wave & 3) + 4 * g + (i & 3), col = 32 * (wave >> 2) + 16 * (i >> 2) + c;
        if (scope == 0) atomicAdd(M + row * 64 + col, v);
        else __hip_atomic_fetch_add(M + row * 64 + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
}

int main() {
  float* ws;
  const size_t n = (size_t)COPIES * NMAT * 4096;
  hipMalloc(&ws, n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> h(n);
  for (int scope = 0; scope < 2; ++scope)
    for (int place = 0; place < 3; ++place) {
      hipMemset(ws, 0, n * 4);
      const int iters = 20, warm = 3;
      for (int w = 0; w < warm; ++w) hipLaunchKernelGGL(atom_kernel, dim3(NBLK), dim3(512), 0, 0, ws, place, scope, 1.f);
      hipEventRecord(a);
      for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(atom_kernel, dim3(NBLK), dim3(512), 0, 0, ws, place, scope, 1.f);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      hipMemcpy(h.data(), ws, n * 4, hipMemcpyDeviceToHost);
      // expected per element of a written copy: (launches) x CHUNKS x (blocks per copy)
      const int ncopy = place == 2 ? 8 : COPIES;
      const double expect = (double)(iters + warm) * CHUNKS * (NBLK / ncopy);
      double maxerr = 0;
      for (size_t e = 0; e < (size_t)ncopy * NMAT * 4096; ++e) maxerr = fmax(maxerr, fabs(h[e] - expect));
      const double bytes = (double)NBLK * WAVES * CHUNKS * NMAT * 8 * 256;
      printf("scope %d place %d: %7.1f us per launch, %5.2f TB/s of added bytes, max |sum - expected| %.0f of %.0f\n",
             scope, place, ms / iters * 1e3, bytes / (ms / iters * 1e-3) / 1e12, maxerr, expect);
    }
  hipFree(ws);
  return 0;
}
