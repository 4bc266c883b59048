// RL math kernels: GAE reverse scan (reference mat_src/mat/utils/shared_buffer.py:207-238).
//
// gae_reverse_scan: one lane per (env, agent, objective) sequence; the T-step reverse recurrence
//   delta_t = r_t + gamma * V(t+1) * m(t+1) - V(t);  g_t = delta_t + gamma*lambda*m(t+1)*g_{t+1}
// runs in registers, V = denormalised value (x*std + mean with the per-objective ValueNorm statistics
// meanstd = [means(n_obj) | stds(n_obj)]); the mask is shared by the n_obj objectives of an (env, agent) pair
// (mo_shared_buffer.py / dmo_shared_buffer.py keep one mask per agent).  Loads of step t are independent of the
// recurrence, so the compiler can issue them ahead (T is 50).
#include "common.h"
#include "gather_rows.h"

__global__ __launch_bounds__(256) void gae_reverse_scan_kernel(
    const float* __restrict__ rew, const float* __restrict__ vpred, const float* __restrict__ masks,
    const float* __restrict__ meanstd, float* __restrict__ adv, float* __restrict__ ret,
    int T, int n, int n_obj, float gamma, float lam) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int o = i % n_obj, im = i / n_obj, nm = n / n_obj;
  const float mean = meanstd[o], sd = meanstd[n_obj + o];
  float g = 0.f;
  float v_next = vpred[(size_t)T * n + i] * sd + mean;
  for (int t = T - 1; t >= 0; --t) {
    const float v = vpred[(size_t)t * n + i] * sd + mean;
    const float m = masks[(size_t)(t + 1) * nm + im];
    const float delta = rew[(size_t)t * n + i] + gamma * v_next * m - v;
    g = delta + gamma * lam * m * g;
    adv[(size_t)t * n + i] = g;
    ret[(size_t)t * n + i] = g + v;
    v_next = v;
  }
}

MDL_API int mdl_gae_reverse_scan(const float* rew, const float* vpred, const float* masks, const float* meanstd,
                                 float* adv, float* ret, int T, int n, int n_obj, float gamma, float lam,
                                 hipStream_t s) {
  if (n_obj <= 0 || n % n_obj) return -1;
  const int bs = 256;
  hipLaunchKernelGGL(gae_reverse_scan_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, s, rew, vpred, masks, meanstd,
                     adv, ret, T, n, n_obj, gamma, lam);
  MDL_CHECK_LAUNCH();
  return 0;
}

// The same scan with the ValueNorm statistics derived in-kernel from the running moments (valuenorm.py
// running_mean_var: d = max(debias, eps), mean = m / d, var = max(m2 / d - mean^2, 1e-2); nvn = 1 or n_obj entries)
// and the bootstrap value V(T) taken from next_value (also written into the buffer's last slot): one launch per
// epoch instead of the scan + ~10 torch launches of the statistics and the slot copy.
__global__ __launch_bounds__(256) void gae_reverse_scan_vn_kernel(
    const float* __restrict__ rew, float* __restrict__ vpred, const float* __restrict__ masks,
    const float* __restrict__ next_value, const float* __restrict__ rm, const float* __restrict__ rmsq,
    const float* __restrict__ deb, float eps, int nvn, float* __restrict__ adv, float* __restrict__ ret,
    int T, int n, int n_obj, float gamma, float lam) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int o = i % n_obj, im = i / n_obj, nm = n / n_obj;
  float mean = 0.f, sd = 1.f;
  if (rm) {
    const int k = nvn == 1 ? 0 : o;
    const float d = fmaxf(deb[0], eps);
    mean = rm[k] / d;
    sd = sqrtf(fmaxf(rmsq[k] / d - mean * mean, 1e-2f));
  }
  const float nv = next_value[i];
  vpred[(size_t)T * n + i] = nv;
  float g = 0.f;
  float v_next = nv * sd + mean;
  // the loads of GAE_PF steps are issued together (rolled: one dependent load latency per step, ~50 us for
  // SMAC's 100 steps); the recurrence itself is a few FMAs per step
  constexpr int GAE_PF = 8;
  int t = T - 1;
  for (; t >= GAE_PF - 1; t -= GAE_PF) {
    float vv[GAE_PF], mm[GAE_PF], rr[GAE_PF];
#pragma unroll
    for (int u = 0; u < GAE_PF; ++u) {
      vv[u] = vpred[(size_t)(t - u) * n + i];
      mm[u] = masks[(size_t)(t - u + 1) * nm + im];
      rr[u] = rew[(size_t)(t - u) * n + i];
    }
#pragma unroll
    for (int u = 0; u < GAE_PF; ++u) {
      const float v = vv[u] * sd + mean;
      const float delta = rr[u] + gamma * v_next * mm[u] - v;
      g = delta + gamma * lam * mm[u] * g;
      adv[(size_t)(t - u) * n + i] = g;
      ret[(size_t)(t - u) * n + i] = g + v;
      v_next = v;
    }
  }
  for (; t >= 0; --t) {
    const float v = vpred[(size_t)t * n + i] * sd + mean;
    const float m = masks[(size_t)(t + 1) * nm + im];
    const float delta = rew[(size_t)t * n + i] + gamma * v_next * m - v;
    g = delta + gamma * lam * m * g;
    adv[(size_t)t * n + i] = g;
    ret[(size_t)t * n + i] = g + v;
    v_next = v;
  }
}

MDL_API int mdl_gae_reverse_scan_vn(const float* rew, float* vpred, const float* masks, const float* next_value,
                                    const float* rm, const float* rmsq, const float* deb, float eps, int nvn,
                                    float* adv, float* ret, int T, int n, int n_obj, float gamma, float lam,
                                    hipStream_t s) {
  if (n_obj <= 0 || n % n_obj || (rm && nvn != 1 && nvn != n_obj)) return -1;
  const int bs = 256;
  hipLaunchKernelGGL(gae_reverse_scan_vn_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, s, rew, vpred, masks, next_value,
                     rm, rmsq, deb, eps, nvn, adv, ret, T, n, n_obj, gamma, lam);
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

// Random permutation of [0, n) in ONE launch (the per-epoch minibatch shuffle; torch.randperm on the device is a
// radix sort of ~10 launches).  A keyed 6-round Feistel network on [0, 2^(2h)) (2^(2h) >= n, round function =
// Philox4x32-10 of (half, round)) is a bijection; cycle walking (re-apply until the value lands below n) restricts
// it to a bijection of [0, n) — each lane walks its own cycle, which returns below n after < 4 steps on average.
__device__ __forceinline__ uint32_t feistel_perm(uint32_t x, int h, uint32_t k0, uint32_t k1) {
  const uint32_t mask = (1u << h) - 1u;
  uint32_t l = x >> h, r = x & mask;
#pragma unroll
  for (int rd = 0; rd < 6; ++rd) {
    const uint32_t f = mdl::philox4x32_10(r, (uint32_t)rd, 0x5EEDu, 0u, k0, k1).x;
    const uint32_t nr = (l ^ f) & mask;
    l = r;
    r = nr;
  }
  return (l << h) | r;
}

__global__ __launch_bounds__(256) void randperm_kernel(int64_t* out, int n, int h, uint32_t k0, uint32_t k1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i;
  do { x = feistel_perm(x, h, k0, k1); } while (x >= (uint32_t)n);
  out[i] = (int64_t)x;
}

MDL_API int mdl_randperm(int64_t* out, int n, uint32_t k0, uint32_t k1, hipStream_t s) {
  if (n <= 0 || n > (1 << 30)) return -1;
  int bits = 2;
  while ((1ll << bits) < (long long)n) ++bits;
  const int h = (bits + 1) / 2;
  hipLaunchKernelGGL(randperm_kernel, dim3((n + 255) / 256), dim3(256), 0, s, out, n, h, k0, k1);
  MDL_CHECK_LAUNCH();
  return 0;
}

// Repack fp32 Linear weights (64 x 64, [out][in]) into the MFMA fragment orders used by the fused kernels, for W
// (forward) and W^T (backward) — all matrices of the model in ONE launch after each optimizer step.
//  * B fragments (decode kernel, round-1 row-layout tiles):
//      element (ct, ks, lane, j) = M[16*ct + (lane & 15)][32*ks + 8*(lane >> 4) + j]
//  * A fragments with the permuted k order of the token-on-lane training tiles (mat_train_ct.h):
//      element (mt, s, lane, j) = M[16*mt + (lane & 15)][32*s + 16*(j >> 2) + 4*(lane >> 4) + (j & 3)]
struct PackEnt { const float* src; unsigned short* fw; unsigned short* bw; unsigned short* fa; unsigned short* ba; };

// grid (matrices, PACK_SPLIT): each workgroup packs 4096 / PACK_SPLIT elements of one matrix (34 single-workgroup
// matrices left the launch latency-bound at ~12.6 us; split over 8 it is a one-pass gather/scatter)
constexpr int PACK_SPLIT = 8;
__global__ __launch_bounds__(256) void pack_weights_kernel(const PackEnt* tab) {
  const PackEnt e = tab[blockIdx.x];
  constexpr int PER = 4096 / PACK_SPLIT;
  for (int idx = blockIdx.y * PER + threadIdx.x; idx < (blockIdx.y + 1) * PER; idx += 256) {
    const int j = idx & 7, lane = (idx >> 3) & 63, ks = (idx >> 9) & 1, ct = idx >> 10;
    const int n = 16 * ct + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + j;
    if (e.fw) e.fw[idx] = mdl::f2bf(e.src[n * 64 + k]);
    if (e.bw) e.bw[idx] = mdl::f2bf(e.src[k * 64 + n]);
    const int kp = 32 * ks + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
    if (e.fa) e.fa[idx] = mdl::f2bf(e.src[n * 64 + kp]);
    if (e.ba) e.ba[idx] = mdl::f2bf(e.src[kp * 64 + n]);
  }
}

MDL_API int mdl_pack_weights(const void* tab, int n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(pack_weights_kernel, dim3(n, PACK_SPLIT), dim3(256), 0, s, (const PackEnt*)tab);
  MDL_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------------------------------
// Advantage statistics + minibatch gather (reference mat_trainer.py:193-197 and shared_buffer.py:260-314).
//
// masked_sums: (Σ x, Σ x², count) over entries whose active mask is non-zero, in fp64 — a fixed-order two-pass
// reduction (per-block partials, then one block), so the statistics are bitwise repeatable (no float atomics).
// The mask has one entry per `mdiv` consecutive x entries (active_masks (…, 1) against advantages (…, n_obj)).
constexpr int SUM_BLOCKS = 240;

__global__ __launch_bounds__(256) void masked_sums_partial_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ mask, int n, int mdiv,
                                                                   double* __restrict__ part) {
  double s = 0.0, sq = 0.0, c = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    if (mask[i / mdiv] != 0.f) {
      const double v = (double)x[i];
      s += v;
      sq += v * v;
      c += 1.0;
    }
  }
  __shared__ double red[3][256];
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = sq;
  red[2][threadIdx.x] = c;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void masked_sums_final_kernel(const double* __restrict__ part, int nb,
                                                                 double* __restrict__ out) {
  __shared__ double red[3][256];
  for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = threadIdx.x < nb ? part[threadIdx.x * 3 + k] : 0.0;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) out[threadIdx.x] = red[threadIdx.x][0];
}

// out[3] and part[3 * SUM_BLOCKS] are device fp64 buffers
MDL_API int mdl_masked_sums(const float* x, const float* mask, int n, int mdiv, double* part, double* out,
                            hipStream_t s) {
  if (n < 0 || mdiv < 1) return -1;
  hipLaunchKernelGGL(masked_sums_partial_kernel, dim3(SUM_BLOCKS), dim3(256), 0, s, x, mask, n, mdiv, part);
  hipLaunchKernelGGL(masked_sums_final_kernel, dim3(1), dim3(256), 0, s, part, SUM_BLOCKS, out);
  MDL_CHECK_LAUNCH();
  return 0;
}

// mb_stats: per-minibatch return statistics of one PPO epoch, computed up front so that a data-parallel epoch needs
// ONE statistics all-reduce (with the advantage moments) instead of one per minibatch inside the loss.
// out[m] = (Σ ret_o (n_obj), Σ ret_o² (n_obj), token count, Σ active) over the rows perm[m*mb .. (m+1)*mb), each row
// `width` tokens.  Fixed-order two-pass fp64 reduction (bitwise repeatable, no float atomics).
constexpr int MBS_PARTS = 32;
constexpr int MBS_K = 6;   // 2 * n_obj + 2 for n_obj <= 2

__global__ __launch_bounds__(256) void mb_stats_partial_kernel(const float* __restrict__ ret,
                                                               const float* __restrict__ active,
                                                               const int64_t* __restrict__ perm, int mb, int width,
                                                               int n_obj, double* __restrict__ part) {
  const int m = blockIdx.y, K = 2 * n_obj + 2;
  double acc[MBS_K];
#pragma unroll
  for (int k = 0; k < MBS_K; ++k) acc[k] = 0.0;
  const int total = mb * width;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += MBS_PARTS * 256) {
    const long long row = perm[(long long)m * mb + i / width];
    const long long tok = row * width + i % width;
    for (int o = 0; o < n_obj; ++o) {
      const double r = (double)ret[tok * n_obj + o];
      acc[o] += r;
      acc[n_obj + o] += r * r;
    }
    acc[2 * n_obj] += 1.0;
    acc[2 * n_obj + 1] += (double)active[tok];
  }
  __shared__ double red[MBS_K][256];
#pragma unroll
  for (int k = 0; k < MBS_K; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < K; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < K) part[((size_t)m * MBS_PARTS + blockIdx.x) * K + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void mb_stats_final_kernel(const double* __restrict__ part, int n_mb, int K, double* __restrict__ out) {
  const int i = threadIdx.x;
  if (i >= n_mb * K) return;
  const int m = i / K, k = i % K;
  double s = 0.0;
  for (int p = 0; p < MBS_PARTS; ++p) s += part[((size_t)m * MBS_PARTS + p) * K + k];
  out[i] = s;
}

MDL_API int mdl_mb_stats(const float* ret, const float* active, const int64_t* perm, int n_mb, int mb, int width,
                         int n_obj, double* part, double* out, hipStream_t s) {
  if (n_obj < 1 || 2 * n_obj + 2 > MBS_K || n_mb < 1 || n_mb * (2 * n_obj + 2) > 1024) return -1;
  hipLaunchKernelGGL(mb_stats_partial_kernel, dim3(MBS_PARTS, n_mb), dim3(256), 0, s, ret, active, perm, mb, width,
                     n_obj, part);
  hipLaunchKernelGGL(mb_stats_final_kernel, dim3(1), dim3(1024), 0, s, part, n_mb, 2 * n_obj + 2, out);
  MDL_CHECK_LAUNCH();
  return 0;
}

// gather_rows (csrc/gather_rows.h): one launch gathers a minibatch's rows of up to GATHER_MAX tensors (blockIdx.y =
// the entry) and standardises the flagged ones (the advantages) on the fly.  The same body also runs inside the fused
// update's adam_pack launch for the next minibatch (csrc/ppo.hip).
__global__ __launch_bounds__(256) void gather_rows_kernel(GatherArgs a) {
  gather_entry(a, blockIdx.y, blockIdx.x, gridDim.x);
}

MDL_API int mdl_gather_rows(const GatherArgs* a, hipStream_t s) {
  if (const int rc = gather_check(*a)) return rc;
  if (a->rows == 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)gather_grid_x(*a, 256), a->n), dim3(256), 0, s, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------ rollout insert
// The DCML runner's per-step bookkeeping in ONE launch (runner/dcml_runner.py _track + insert; reference
// runner/dcml_runner.py:250-288 insert and shared_buffer.py insert): the buffer-slot copies of the step's
// observations / share obs / availability / actions / log-probs / values, the agent-expanded rewards and masks,
// and the episode accumulators with the finished-episode statistics.  Round 1 ran these as ~30 torch launches per
// env step (1,500 per PPO iteration).  Workgroups 1.. copy; workgroup 0 does the per-env part, its statistics
// reduced in a fixed order (bit-reproducible run to run).
struct InsSeg { const float* src; float* dst; int n; };
constexpr int INS_SEGS = 6;
struct InsArgs {
  InsSeg seg[INS_SEGS];
  int E, A, n_obj;
  const float *reward, *delay, *pay;
  const unsigned char* done;
  float *d_rew, *d_mask;          // rewards[t] (E, A, n_obj), masks[t + 1] (E, A, 1)
  float *ep_r, *ep_d, *ep_p;      // (E) running episode sums
  double* stats;                  // [4] += (finished episodes, Σ their reward, Σ delay, Σ payment)
};

__global__ __launch_bounds__(256) void rollout_insert_kernel(InsArgs a) {
  const int tid = threadIdx.x;
  if (blockIdx.x > 0) {
    const int stride = (gridDim.x - 1) * 256;
#pragma unroll
    for (int k = 0; k < INS_SEGS; ++k) {
      const InsSeg s = a.seg[k];
      for (int i = (blockIdx.x - 1) * 256 + tid; i < s.n; i += stride) s.dst[i] = s.src[i];
    }
    return;
  }
  __shared__ double red[4][256];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int e = tid; e < a.E; e += 256) {
    const float r = a.reward[e], dl = a.delay[e], py = a.pay[e];
    const bool d = a.done[e] != 0;
    for (int ag = 0; ag < a.A; ++ag) {
      const size_t o = (size_t)e * a.A + ag;
      a.d_mask[o] = d ? 0.f : 1.f;
      if (a.n_obj == 2) {
        a.d_rew[2 * o] = -dl;
        a.d_rew[2 * o + 1] = -py;
      } else {
        a.d_rew[o] = r;
      }
    }
    const float er = a.ep_r[e] + r, ed = a.ep_d[e] + dl, ep = a.ep_p[e] + py;
    if (d) {
      acc[0] += 1.0;
      acc[1] += (double)er;
      acc[2] += (double)ed;
      acc[3] += (double)ep;
    }
    a.ep_r[e] = d ? 0.f : er;
    a.ep_d[e] = d ? 0.f : ed;
    a.ep_p[e] = d ? 0.f : ep;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[k][tid] = acc[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w)
#pragma unroll
      for (int k = 0; k < 4; ++k) red[k][tid] += red[k][tid + w];
    __syncthreads();
  }
  if (tid < 4) a.stats[tid] += red[tid][0];
}

// The SMAC runner's per-step bookkeeping in one launch (runner/smac_runner.py _track_smac + _insert_smac; reference
// smac_runner.py insert: masks = 0 where every agent of the env is done, active masks = 0 for dead agents of running
// envs): slot copies, the agent-expanded rewards, masks, active masks, the episode reward sums and the
// (finished battles, Σ their reward, Σ won, Σ dead allies) statistics.  Replaces ~25 torch launches per env step.
struct SmacInsArgs {
  InsSeg seg[INS_SEGS];
  int E, A;
  const float* reward;            // [E]
  const unsigned char* dones;     // [E][A] (bool)
  const unsigned char* won;       // [E] (bool)
  const float* dead;              // [E] dead allies
  float *d_rew, *d_mask, *d_active;   // rewards[t], masks[t + 1], active_masks[t + 1]: (E, A, 1)
  float* ep_r;                    // (E) running episode reward
  double* stats;                  // [4]
};

__global__ __launch_bounds__(256) void smac_insert_kernel(SmacInsArgs a) {
  const int tid = threadIdx.x;
  if (blockIdx.x > 0) {
    const int stride = (gridDim.x - 1) * 256;
#pragma unroll
    for (int k = 0; k < INS_SEGS; ++k) {
      const InsSeg s = a.seg[k];
      if ((s.n & 3) == 0 && ((reinterpret_cast<uintptr_t>(s.src) | reinterpret_cast<uintptr_t>(s.dst)) & 15) == 0) {
        const float4* s4 = (const float4*)s.src;
        float4* d4 = (float4*)s.dst;
        for (int i = (blockIdx.x - 1) * 256 + tid; i < (s.n >> 2); i += stride) d4[i] = s4[i];
      } else {
        for (int i = (blockIdx.x - 1) * 256 + tid; i < s.n; i += stride) s.dst[i] = s.src[i];
      }
    }
    return;
  }
  __shared__ double red[4][256];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int e = tid; e < a.E; e += 256) {
    const float r = a.reward[e];
    int nd = 0;   // every agent's flag loaded (a short-circuit && chain was one dependent byte load per agent)
#pragma unroll 8
    for (int ag = 0; ag < a.A; ++ag) nd += a.dones[(size_t)e * a.A + ag] != 0;
    const bool d = nd == a.A;
    for (int ag = 0; ag < a.A; ++ag) {
      const size_t o = (size_t)e * a.A + ag;
      a.d_rew[o] = r;
      a.d_mask[o] = d ? 0.f : 1.f;
      a.d_active[o] = (d || a.dones[o] == 0) ? 1.f : 0.f;
    }
    const float er = a.ep_r[e] + r;
    if (d) {
      acc[0] += 1.0;
      acc[1] += (double)er;
    }
    acc[2] += a.won[e] ? 1.0 : 0.0;
    acc[3] += (double)a.dead[e];
    a.ep_r[e] = d ? 0.f : er;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[k][tid] = acc[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w)
#pragma unroll
      for (int k = 0; k < 4; ++k) red[k][tid] += red[k][tid + w];
    __syncthreads();
  }
  if (tid < 4) a.stats[tid] += red[tid][0];
}

MDL_API int mdl_smac_insert(const SmacInsArgs* a, hipStream_t s) {
  if (a->E < 1 || a->A < 1) return -1;
  int most = 0;
  for (int k = 0; k < INS_SEGS; ++k) {
    if (a->seg[k].n < 0 || (a->seg[k].n > 0 && (!a->seg[k].src || !a->seg[k].dst))) return -2;
    most = a->seg[k].n > most ? a->seg[k].n : most;
  }
  // one float4 per thread of the largest segment (SMAC's obs / state slots: ~1,100 workgroups): the copy is bound
  // by bytes in flight, and a 256-workgroup cap left each thread a dependent 4-iteration loop (13.9 us per step)
  int gx = (most / 4 + 255) / 256;
  gx = gx < 1 ? 1 : (gx > 2048 ? 2048 : gx);
  hipLaunchKernelGGL(smac_insert_kernel, dim3(gx + 1), dim3(256), 0, s, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}

MDL_API int mdl_rollout_insert(const InsArgs* a, hipStream_t s) {
  if (a->E < 1 || a->A < 1 || (a->n_obj != 1 && a->n_obj != 2)) return -1;
  int most = 0;
  for (int k = 0; k < INS_SEGS; ++k) {
    if (a->seg[k].n < 0 || (a->seg[k].n > 0 && (!a->seg[k].src || !a->seg[k].dst))) return -2;
    most = a->seg[k].n > most ? a->seg[k].n : most;
  }
  int gx = (most + 255) / 256;
  gx = gx < 1 ? 1 : (gx > 64 ? 64 : gx);
  hipLaunchKernelGGL(rollout_insert_kernel, dim3(gx + 1), dim3(256), 0, s, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}
