// Probe of the DPP moves the one-wave decode relies on: row_newbcast:n and bank-masked row_ror:8 (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int N> __device__ float bc(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x150 + N, 0xF, 0xF, false));
}
template <int B> __device__ float ror(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, -x), __builtin_bit_cast(int, x), 0x128, 0xF, B, false));
}
__global__ void k(float* out) {
  const float x = (float)threadIdx.x;
  out[threadIdx.x] = bc<0>(x);
  out[64 + threadIdx.x] = bc<5>(x);
  out[128 + threadIdx.x] = bc<15>(x);
  out[192 + threadIdx.x] = ror<0xC>(x);
  out[256 + threadIdx.x] = ror<0x3>(x);
}
int main() {
  float* d; hipMalloc(&d, 320 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[320]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[5] = {"newbcast0", "newbcast5", "newbcast15", "ror8 banks 0xC (old=-x)", "ror8 banks 0x3 (old=-x)"};
  for (int t = 0; t < 5; ++t) {
    printf("%s:", names[t]);
    for (int i = 0; i < 64; ++i) printf(" %g", h[t * 64 + i]);
    printf("\n");
  }
  return 0;
}
