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

// uniform in (0,1) from the 24 high bits, centred — matches utils/philox.py:u01_open.  Exact in fp64.  The fp32
// variant rounds the top value (u >> 8 == 2^24 - 1) up to exactly 1.0f (found by tests/native/host_checks.hip);
// its one user (workload noise in [0.8, 1.2]) is closed at the top by design and the torch path rounds the same way.
__host__ __device__ __forceinline__ double u01_open(uint32_t u) { return ((double)(u >> 8) + 0.5) * (1.0 / 16777216.0); }
__host__ __device__ __forceinline__ float u01_open_f(uint32_t u) { return ((float)(u >> 8) + 0.5f) * (1.0f / 16777216.0f); }

enum Purpose : uint32_t {
  P_MASTER = 1, P_ARRIVE = 2, P_WORKER_PR = 3, P_NOISE = 4, P_DISABLE = 5, P_DOWNLOAD = 6, P_UPLOAD = 7,
  P_DONE = 8, P_SHANNON = 9, P_POLICY = 16
};

// ------------------------------------------------------------------------------------------ cross-lane (VALU)
// __shfl_xor compiles to ds_bpermute_b32: an LDS-pipe round trip per step.  These use DPP (within 16-lane rows)
// and v_permlane16/32_swap (across rows) instead: plain VALU ops, no lgkmcnt wait.  Every lane of a group ends
// with bit-identical results (each step adds the same two operands in the same order).
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_ROR8 = 0x128;
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
// v_permlane16/32_swap of a register with (an opaque copy of) itself: r[0] = the even rows / low half of x
// everywhere, r[1] = the odd rows / high half.  (With the SAME value for both operands hipcc folds r[1] into
// r[0], so the copy is hidden behind an empty asm.)
__device__ __forceinline__ void swap16(float x, float& even, float& odd) {
  unsigned a = __builtin_bit_cast(unsigned, x), b = a;
  asm volatile("" : "+v"(b));
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  even = __builtin_bit_cast(float, (unsigned)r[0]);
  odd = __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ void swap32(float x, float& lo, float& hi) {
  unsigned a = __builtin_bit_cast(unsigned, x), b = a;
  asm volatile("" : "+v"(b));
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  lo = __builtin_bit_cast(float, (unsigned)r[0]);
  hi = __builtin_bit_cast(float, (unsigned)r[1]);
}
// value of lane ^ 16 / lane ^ 32
__device__ __forceinline__ float xor16_partner(float x) {
  float e, o;
  swap16(x, e, o);
  return ((threadIdx.x >> 4) & 1) ? e : o;
}
__device__ __forceinline__ float xor32_partner(float x) {
  float lo, hi;
  swap32(x, lo, hi);
  return ((threadIdx.x >> 5) & 1) ? lo : hi;
}
// sum / max over aligned groups of N lanes, N in {2, 4, 8, 16, 32, 64}
template <int N>
__device__ __forceinline__ float group_sum(float x) {
  x += dppf<DPP_XOR1>(x);
  if (N > 2) x += dppf<DPP_XOR2>(x);
  if (N > 4) x += dppf<DPP_ROW_HALF_MIRROR>(x);
  if (N > 8) x += dppf<DPP_ROW_MIRROR>(x);
  if (N > 16) {
    float e, o;
    swap16(x, e, o);
    x = e + o;
  }
  if (N > 32) {
    float lo, hi;
    swap32(x, lo, hi);
    x = lo + hi;
  }
  return x;
}
template <int N>
__device__ __forceinline__ float group_max(float x) {
  x = fmaxf(x, dppf<DPP_XOR1>(x));
  if (N > 2) x = fmaxf(x, dppf<DPP_XOR2>(x));
  if (N > 4) x = fmaxf(x, dppf<DPP_ROW_HALF_MIRROR>(x));
  if (N > 8) x = fmaxf(x, dppf<DPP_ROW_MIRROR>(x));
  if (N > 16) x = fmaxf(x, xor16_partner(x));
  if (N > 32) x = fmaxf(x, xor32_partner(x));
  return x;
}
// sum over the lanes sharing lane & 15 (the 4 rows of 16): lane ^ 16, lane ^ 32 partners
__device__ __forceinline__ float cross_row_sum(float x) {
  float a, b;
  swap16(x, a, b);
  x = a + b;
  swap32(x, a, b);
  return a + b;
}

// ------------------------------------------------------------------------------------------ wave64 reductions
__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }
__device__ __forceinline__ float wave_max(float v) { return group_max<64>(v); }
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

// 2^x as ONE v_exp_f32.  exp2f() compiles to a denormal-safe sequence (range compare, two selects, an add and a
// v_ldexp_f32 around the v_exp) — 7 VALU per element in the attention loops.  Softmax arguments are <= 0 and a
// probability below 2^-126 is irrelevant, so the raw instruction (exp2(-inf) = 0) is exact enough everywhere here.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16
// resolution): one rcp, one exp and a degree-5 polynomial instead of the libm erff.  The exp(-x^2/2) factor is
// shared with the Gaussian pdf of the GELU derivative.
__device__ __forceinline__ float phi_and_pdf(float x, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  // v_rcp_f32 (1 ulp): __frcp_rn's IEEE-rounded reciprocal expanded to a 5-instruction div_scale / div_fmas /
  // div_fixup sequence per element, a third of the training kernels' GELU cost (the A&S error is 1.5e-7 anyway)
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * z);
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
// GELU(x) and GELU'(x) from ONE erf evaluation
__device__ __forceinline__ float gelu_erf_both(float x, float& grad) {
  float pdf;
  const float cdf = phi_and_pdf(x, pdf);
  grad = fmaf(x, pdf, cdf);
  return x * cdf;
}

}  // namespace mdl
