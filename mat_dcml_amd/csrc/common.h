// Shared device helpers for the MI355X (gfx950, CDNA4) kernels of mat_dcml_amd.
// - Philox4x32-10 counter RNG, bit-identical to mat_dcml_amd/utils/philox.py
// - wave64 reductions (CDNA wavefront = 64 lanes)
// - bf16 <-> f32 helpers and MFMA fragment types
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MDL_API extern "C" __attribute__((visibility("default")))
#define MDL_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

namespace mdl {

// ------------------------------------------------------------------------------------------ Philox
struct u4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__host__ __device__ __forceinline__ u4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                      uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2511F53u, c0, hi0, lo0);
    mulhilo(0xCD9E8D57u, c2, hi1, lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// uniform in (0,1) from the 24 high bits, centred — matches utils/philox.py:u01_open (exact in fp32 and fp64)
__host__ __device__ __forceinline__ double u01_open(uint32_t u) { return ((double)(u >> 8) + 0.5) * (1.0 / 16777216.0); }
__host__ __device__ __forceinline__ float u01_open_f(uint32_t u) { return ((float)(u >> 8) + 0.5f) * (1.0f / 16777216.0f); }

enum Purpose : uint32_t {
  P_MASTER = 1, P_ARRIVE = 2, P_WORKER_PR = 3, P_NOISE = 4, P_DISABLE = 5, P_DOWNLOAD = 6, P_UPLOAD = 7,
  P_DONE = 8, P_SHANNON = 9, P_POLICY = 16
};

// ------------------------------------------------------------------------------------------ wave64 reductions
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
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------------------ bf16
typedef unsigned short bf16_t;
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {  // round-to-nearest-even: one v_cvt_pk_bf16_f32 on gfx950
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16
// resolution): one rcp, one exp and a degree-5 polynomial instead of the libm erff.  The exp(-x^2/2) factor is
// shared with the Gaussian pdf of the GELU derivative.
__device__ __forceinline__ float phi_and_pdf(float x, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __frcp_rn(1.0f + 0.3275911f * z);
  const float e = __expf(-z * z);
  float poly = 1.061405429f;
  poly = fmaf(poly, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  const float erf_abs = 1.0f - poly * t * e;
  pdf = 0.39894228040143268f * e;
  return 0.5f + 0.5f * copysignf(erf_abs, x);
}
__device__ __forceinline__ float gelu_erf(float x) {
  float pdf;
  return x * phi_and_pdf(x, pdf);
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float pdf;
  const float cdf = phi_and_pdf(x, pdf);
  return cdf + x * pdf;
}

}  // namespace mdl
