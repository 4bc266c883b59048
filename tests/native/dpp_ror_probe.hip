// Probe: direction of DPP row_ror:4 / row_ror:12 on gfx950 (which source lane each lane reads) — the speculative
// decode's PAIR head exchange depends on it.  Prints, per destination lane 0..15, the source lane id.
// Build: hipcc -O2 --offload-arch=gfx950 tests/native/dpp_ror_probe.hip -o tests/native/dpp_ror_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int x = threadIdx.x;
  out[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x124, 0xF, 0xF, false);
  out[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x12C, 0xF, 0xF, false);
  out[128 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false);
}
int main() {
  int* d;
  int h[192];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[3] = {"row_ror:4 (0x124)", "row_ror:12 (0x12C)", "row_shr:1 (0x111)"};
  for (int t = 0; t < 3; ++t) {
    printf("%s: dst lane <- src lane:", nm[t]);
    for (int i = 0; i < 16; ++i) printf(" %d<-%d", i, h[64 * t + i]);
    printf("\n");
  }
  return 0;
}
