#include "../../mat_dcml_amd/csrc/common.h"
using namespace mdl;
__global__ void k(const float* in, float* out) {
  const int l = threadIdx.x;
  float x = in[l];
  out[l] = group_sum<16>(x);
  out[64 + l] = group_sum<8>(x);
  out[128 + l] = group_sum<64>(x);
  out[192 + l] = group_max<32>(x);
  out[256 + l] = cross_row_sum(x);
  out[320 + l] = xor16_partner(x);
  out[384 + l] = xor32_partner(x);
  out[448 + l] = group_sum<4>(x);
}
int main() {
  float h[64], o[512], *d, *dout;
  for (int i = 0; i < 64; ++i) h[i] = (float)((i * 37) % 64) + 0.25f * i;
  hipMalloc(&d, 256); hipMalloc(&dout, 2048);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, dout);
  hipMemcpy(o, dout, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    double s16 = 0, s8 = 0, s64 = 0, s4 = 0, m32 = -1e30, cr = 0;
    for (int j = 0; j < 64; ++j) {
      if (j / 16 == l / 16) s16 += h[j];
      if (j / 8 == l / 8) s8 += h[j];
      if (j / 4 == l / 4) s4 += h[j];
      if (j / 32 == l / 32) m32 = h[j] > m32 ? h[j] : m32;
      if ((j & 15) == (l & 15)) cr += h[j];
      s64 += h[j];
    }
    double want[8] = {s16, s8, s64, m32, cr, h[l ^ 16], h[l ^ 32], s4};
    for (int t = 0; t < 8; ++t) if (fabs(o[t * 64 + l] - want[t]) > 1e-3) { if (bad < 10) printf("t%d lane %d got %f want %f\n", t, l, o[t*64+l], want[t]); ++bad; }
  }
  printf(bad ? "FAIL %d\n" : "OK\n", bad);
  return bad != 0;
}
