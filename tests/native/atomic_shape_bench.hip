// Micro-benchmark: fp32 no-return atomics of a 64x64 weight-gradient block per wave-instruction shape, with the
// training backward's traffic (256 workgroups x 8 waves, 22 matrices x 3 chunks, 32 workspace copies).
//   shape 0: 4 rows x 64 B per wave-instruction (16x16 accumulator as it stands: lane (g, c) -> row 4g + r, col c)
//   shape 1: 2 rows x 128 B (two 16-column tiles side by side)
//   shape 2: 1 row x 256 B
// Build: hipcc -O3 --offload-arch=gfx950 tests/native/atomic_shape_bench.hip -o /tmp/atomic_shape_bench
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NMAT = 22, CHUNKS = 3, COPIES = 32, WAVES = 8;

__global__ __launch_bounds__(512) void atom_kernel(float* ws, int shape, float v) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* base = ws + (size_t)(blockIdx.x % COPIES) * NMAT * 4096;
  const int g = lane >> 4, c = lane & 15;
  for (int ch = 0; ch < CHUNKS; ++ch)
    for (int m = 0; m < NMAT; ++m) {
      float* M = base + m * 4096;
      // each wave owns 512 elements (16 rows x 32 cols) of the 64x64 block: 8 instructions
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        int row, col;
        if (shape == 0) {        // 4 rows x 16 cols: rows 16(w&3) + 4g + (i&3), cols 32(w>>2) + 16(i>>2) + c
          row = 16 * (wave & 3) + 4 * g + (i & 3);
          col = 32 * (wave >> 2) + 16 * (i >> 2) + c;
        } else if (shape == 1) { // 2 rows x 32 cols
          row = 16 * (wave & 3) + 2 * i + (lane >> 5);
          col = 32 * (wave >> 2) + (lane & 31);
        } else {                 // 1 row x 64 cols (two instructions per row pair of the 16 x 32 region)
          row = 16 * (wave & 3) + 2 * i + (wave >> 2);
          col = lane;
        }
        atomicAdd(M + row * 64 + col, v);
      }
    }
}

int main() {
  float* ws;
  const size_t n = (size_t)COPIES * NMAT * 4096;
  hipMalloc(&ws, n * 4);
  hipMemset(ws, 0, n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int shape = 0; shape < 3; ++shape) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(atom_kernel, dim3(256), dim3(512), 0, 0, ws, shape, 1.f);
    hipEventRecord(a);
    for (int it = 0; it < 20; ++it) hipLaunchKernelGGL(atom_kernel, dim3(256), dim3(512), 0, 0, ws, shape, 1.f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = 256.0 * WAVES * CHUNKS * NMAT * 8 * 256;
    printf("shape %d: %.1f us per launch, %.2f TB/s of added bytes\n", shape, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e12);
  }
  hipFree(ws);
  return 0;
}
