// RL math kernels: GAE reverse scan (reference mat_src/mat/utils/shared_buffer.py:207-238).
//
// gae_reverse_scan: one lane per (env, agent, objective) sequence; the T-step reverse recurrence
//   delta_t = r_t + gamma * V(t+1) * m(t+1) - V(t);  g_t = delta_t + gamma*lambda*m(t+1)*g_{t+1}
// runs in registers, V = denormalised value (x*std + mean from the ValueNorm statistics in meanstd[2]).
// Loads of step t are independent of the recurrence, so the compiler can issue them ahead (T is 50).
#include "common.h"

__global__ __launch_bounds__(256) void gae_reverse_scan_kernel(
    const float* __restrict__ rew, const float* __restrict__ vpred, const float* __restrict__ masks,
    const float* __restrict__ meanstd, float* __restrict__ adv, float* __restrict__ ret,
    int T, int n, float gamma, float lam) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float mean = meanstd[0], sd = meanstd[1];
  float g = 0.f;
  float v_next = vpred[(size_t)T * n + i] * sd + mean;
  for (int t = T - 1; t >= 0; --t) {
    const float v = vpred[(size_t)t * n + i] * sd + mean;
    const float m = masks[(size_t)(t + 1) * n + i];
    const float delta = rew[(size_t)t * n + i] + gamma * v_next * m - v;
    g = delta + gamma * lam * m * g;
    adv[(size_t)t * n + i] = g;
    ret[(size_t)t * n + i] = g + v;
    v_next = v;
  }
}

MDL_API int mdl_gae_reverse_scan(const float* rew, const float* vpred, const float* masks, const float* meanstd,
                                 float* adv, float* ret, int T, int n, float gamma, float lam, hipStream_t s) {
  const int bs = 256;
  hipLaunchKernelGGL(gae_reverse_scan_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, s, rew, vpred, masks, meanstd,
                     adv, ret, T, n, gamma, lam);
  MDL_CHECK_LAUNCH();
  return 0;
}

// Philox test/fill kernel: out[i] = philox(c0 = i, c1, c2, c3; k0, k1) as 4 uint32 (stored in int64 for torch).
__global__ void philox_fill_kernel(int64_t* out, int n, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                   uint32_t k1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mdl::u4 r = mdl::philox4x32_10((uint32_t)i, c1, c2, c3, k0, k1);
  out[4 * i + 0] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

MDL_API int mdl_philox_fill(int64_t* out, int n, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                            hipStream_t s) {
  hipLaunchKernelGGL(philox_fill_kernel, dim3((n + 255) / 256), dim3(256), 0, s, out, n, c1, c2, c3, k0, k1);
  MDL_CHECK_LAUNCH();
  return 0;
}

// Repack fp32 Linear weights (64 x 64, [out][in]) into the MFMA B-fragment order used by the fused kernels, for W
// (forward) and W^T (backward) — all matrices of the model in ONE launch after each optimizer step.
// fragment element (ct, ks, lane, j) = M[16*ct + (lane & 15)][32*ks + 8*(lane >> 4) + j]
struct PackEnt { const float* src; unsigned short* fw; unsigned short* bw; };

__global__ __launch_bounds__(256) void pack_weights_kernel(const PackEnt* tab) {
  const PackEnt e = tab[blockIdx.x];
  for (int idx = threadIdx.x; idx < 4096; idx += 256) {
    const int j = idx & 7, lane = (idx >> 3) & 63, ks = (idx >> 9) & 1, ct = idx >> 10;
    const int n = 16 * ct + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + j;
    if (e.fw) e.fw[idx] = mdl::f2bf(e.src[n * 64 + k]);
    if (e.bw) e.bw[idx] = mdl::f2bf(e.src[k * 64 + n]);
  }
}

MDL_API int mdl_pack_weights(const void* tab, int n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(pack_weights_kernel, dim3(n), dim3(256), 0, s, (const PackEnt*)tab);
  MDL_CHECK_LAUNCH();
  return 0;
}
