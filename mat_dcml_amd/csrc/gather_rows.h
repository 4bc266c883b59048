// Minibatch row gather shared by rl_ops.hip (its own launch, gather_rows_kernel) and ppo.hip (the NEXT minibatch's
// gather folded into the fused update's adam_pack launch, whose ~100 workgroups leave most CUs idle).
//   dst_k[r, :] = src_k[idx[r], :] for up to GATHER_MAX row-major fp32 tensors; entries flagged `norm` are
//   standardised on the fly with the masked_sums statistics: (x - mean) / (std + eps), std the population std — the
//   normalised advantage of the reference (mat_trainer.py:193-197), computed only for the rows a minibatch reads.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr int GATHER_MAX = 10;
constexpr int GATHER_CHUNK = 4096;   // floats per work item of a wide row (a multiple of 1024)
struct GatherEnt { const float* src; float* dst; int width; int norm; };
struct GatherArgs { GatherEnt e[GATHER_MAX]; const int64_t* idx; const double* sums; int rows; int n; float eps; };

__device__ __forceinline__ void gather_norm_params(const GatherArgs& a, const GatherEnt& e, float& mean, float& sd) {
  mean = 0.f;
  sd = 1.f;
  if (!e.norm) return;
  const double cnt = a.sums[2] < 1.0 ? 1.0 : a.sums[2];
  const double m = a.sums[0] / cnt;
  double var = a.sums[1] / cnt - m * m;
  var = var < 0.0 ? 0.0 : var;
  mean = (float)m;
  sd = (float)sqrt(var) + a.eps;
}

// entry k by workgroup bx of gx (any block size): narrow rows (w < 1024, DCML's 33 x 7) as one flat element loop
// over the minibatch (coalesced across rows); wide rows (SMAC's 27 x 1288) as (row, 4096-float chunk) items with
// float4 lanes when the width and both bases allow it
__device__ __forceinline__ void gather_entry(const GatherArgs& a, int k, int bx, int gx) {
  const GatherEnt e = a.e[k];
  float mean, sd;
  gather_norm_params(a, e, mean, sd);
  const int w = e.width, nt = blockDim.x, tid = threadIdx.x;
  if (w < 1024) {
    const int total = a.rows * w;
    for (int i = bx * nt + tid; i < total; i += gx * nt) {
      const int r = i / w, c = i - r * w;
      float v = e.src[(size_t)a.idx[r] * w + c];
      if (e.norm) v = (v - mean) / sd;
      e.dst[i] = v;
    }
    return;
  }
  const bool vec = (w & 3) == 0 && ((reinterpret_cast<uintptr_t>(e.src) | reinterpret_cast<uintptr_t>(e.dst)) & 15) == 0;
  const int nch = (w + GATHER_CHUNK - 1) / GATHER_CHUNK;
  for (int item = bx; item < a.rows * nch; item += gx) {
    const int r = item / nch, c0 = (item - r * nch) * GATHER_CHUNK;
    const int cn = min(GATHER_CHUNK, w - c0);
    const float* src = e.src + (size_t)a.idx[r] * w + c0;
    float* dst = e.dst + (size_t)r * w + c0;
    if (vec) {   // blockDim >= 256: at most 4 float4 per lane, the loads issued before the stores
      const float4* s4 = (const float4*)src;
      float4* d4 = (float4*)dst;
      float4 v[GATHER_CHUNK / 1024];
#pragma unroll
      for (int j = 0; j < GATHER_CHUNK / 1024; ++j) {
        const int c = tid + nt * j;
        v[j] = c < (cn >> 2) ? s4[c] : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < GATHER_CHUNK / 1024; ++j) {
        const int c = tid + nt * j;
        if (e.norm) {
          v[j].x = (v[j].x - mean) / sd; v[j].y = (v[j].y - mean) / sd;
          v[j].z = (v[j].z - mean) / sd; v[j].w = (v[j].w - mean) / sd;
        }
        if (c < (cn >> 2)) d4[c] = v[j];
      }
    } else {
      for (int c = tid; c < cn; c += nt) {
        float v = src[c];
        if (e.norm) v = (v - mean) / sd;
        dst[c] = v;
      }
    }
  }
}

// Row-per-wave form for the fused update (narrow rows only, every width <= 1024): the (entry, row) items are dealt
// round robin over the waves, a row's floats over the lanes (coalesced; one index load per row) — many independent
// waves instead of one element per thread, so it finishes within the Adam launch it shares.
__device__ __forceinline__ void gather_rows_wavewise(const GatherArgs& a, int wave_id, int nwaves, int lane) {
  const int items = a.n * a.rows;
  for (int it = wave_id; it < items; it += nwaves) {
    const int k = it / a.rows, r = it - k * a.rows;
    const GatherEnt e = a.e[k];
    float mean, sd;
    gather_norm_params(a, e, mean, sd);
    const int w = e.width;
    const float* src = e.src + (size_t)a.idx[r] * w;
    float* dst = e.dst + (size_t)r * w;
    for (int c = lane; c < w; c += 64) {
      float v = src[c];
      if (e.norm) v = (v - mean) / sd;
      dst[c] = v;
    }
  }
}

// host: the x-extent of a gather over every entry (items of the widest entry, capped)
inline int gather_grid_x(const GatherArgs& a, int threads) {
  long long items = 0;
  for (int k = 0; k < a.n; ++k) {
    const long long w = a.e[k].width;
    const long long it = w < 1024 ? ((long long)a.rows * w + threads - 1) / threads
                                  : (long long)a.rows * ((w + GATHER_CHUNK - 1) / GATHER_CHUNK);
    items = items > it ? items : it;
  }
  return (int)(items < 1 ? 1 : (items < 8192 ? items : 8192));
}

inline int gather_check(const GatherArgs& a) {
  if (a.n < 1 || a.n > GATHER_MAX || a.rows < 0) return -1;
  for (int k = 0; k < a.n; ++k)
    if (a.e[k].width < 1 || (long long)a.rows * a.e[k].width >= (1ll << 31)) return -2;
  return 0;
}
