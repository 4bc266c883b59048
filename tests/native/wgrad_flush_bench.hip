// Micro-benchmark: the training backward's weight-gradient flush traffic (256 workgroups x 8 waves, NMAT 64x64
// matrices per chunk, 3 chunks per workgroup: the decoder backward at L = 33) in three forms, each followed by the
// reduction that folds the copies into one gradient:
//   mode 0: fp32 atomics into 32 copies (copy = blockIdx % 32), reduced over 32 copies       (rounds 2-5)
//   mode 1: one PRIVATE copy per workgroup: chunk 0 plain-stores its partial, later chunks load + add + store their
//           own earlier values (no atomics, fixed order: deterministic); reduced over 256 copies in a fixed order
//   mode 2: one slot per (workgroup, chunk), nontemporal plain stores; reduced over 768 slots
// Each wave owns a 16 x 32 block of every matrix: 8 floats per lane, two 16-byte accesses (fragment-native layout).
// Build: hipcc -O3 --offload-arch=gfx950 tests/native/wgrad_flush_bench.hip -o tests/native/wgrad_flush_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int CHUNKS = 3, WAVES = 8, NBLK = 256, MATF = 4096;

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void flush_kernel(float* ws, int mode, int nmat, float v) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const size_t per = (size_t)nmat * MATF;
  for (int ch = 0; ch < CHUNKS; ++ch) {
    if (mode == 0) {
      float* base = ws + (size_t)(blockIdx.x % 32) * per;
      for (int m = 0; m < nmat; ++m) {
        float* M = base + (size_t)m * MATF;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = 16 * (wave & 3) + 4 * g + (i & 3), col = 32 * (wave >> 2) + 16 * (i >> 2) + c;
          atomicAdd(M + row * 64 + col, v);
        }
      }
    } else {
      const size_t slot = mode == 1 ? blockIdx.x : (size_t)blockIdx.x * CHUNKS + ch;
      float* base = ws + slot * per;
      for (int m = 0; m < nmat; ++m) {
        f4* M = (f4*)(base + (size_t)m * MATF + wave * 512) + lane * 2;   // wave block = 512 floats, lane-owned 8
        f4 a = {v, v, v, v}, b = a;
        if (mode == 1 && ch > 0) {
          a += M[0];
          b += M[1];
          M[0] = a;
          M[1] = b;
        } else if (mode == 1) {
          M[0] = a;
          M[1] = b;
        } else {
          __builtin_nontemporal_store(a, M);
          __builtin_nontemporal_store(b, M + 1);
        }
      }
    }
  }
}

// g[i] = Σ_k ws[k * per + i] over `copies` copies, fixed order
__global__ __launch_bounds__(256) void reduce_kernel(float* g, const float* ws, size_t per, int copies) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < per; i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= copies; k += 8) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = ws[(size_t)(k + j) * per + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += t[j];
    }
    for (; k < copies; ++k) s += ws[(size_t)k * per + i];
    g[i] = s;
  }
}

int main() {
  const int nmats[2] = {22, 14};
  for (int mi = 0; mi < 2; ++mi) {
    const int nmat = nmats[mi];
    const size_t per = (size_t)nmat * MATF;
    float *ws, *g;
    hipMalloc(&ws, (size_t)NBLK * CHUNKS * per * 4);
    hipMalloc(&g, per * 4);
    hipEvent_t a, b, c;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventCreate(&c);
    std::vector<float> h(per);
    for (int mode = 0; mode < 3; ++mode) {
      const int copies = mode == 0 ? 32 : mode == 1 ? NBLK : NBLK * CHUNKS;
      const int iters = 20;
      float ms_f = 0.f, ms_r = 0.f;
      for (int it = -3; it < iters; ++it) {
        if (mode == 0) hipMemsetAsync(ws, 0, (size_t)32 * per * 4);
        hipEventRecord(a);
        hipLaunchKernelGGL(flush_kernel, dim3(NBLK), dim3(512), 0, 0, ws, mode, nmat, 1.f);
        hipEventRecord(b);
        hipLaunchKernelGGL(reduce_kernel, dim3(1024), dim3(256), 0, 0, g, ws, per, copies);
        hipEventRecord(c);
        hipEventSynchronize(c);
        float x, y;
        hipEventElapsedTime(&x, a, b);
        hipEventElapsedTime(&y, b, c);
        if (it >= 0) { ms_f += x; ms_r += y; }
      }
      hipMemcpy(h.data(), g, per * 4, hipMemcpyDeviceToHost);
      double maxerr = 0;
      for (size_t e = 0; e < per; ++e) maxerr = fmax(maxerr, fabs(h[e] - (double)NBLK * CHUNKS));
      printf("nmat %d mode %d: flush %7.1f us, reduce %6.1f us (%d copies), total %7.1f us, max err %.0f\n", nmat, mode,
             ms_f / iters * 1e3, ms_r / iters * 1e3, copies, (ms_f + ms_r) / iters * 1e3, maxerr);
    }
    hipFree(ws);
    hipFree(g);
  }
  return 0;
}
