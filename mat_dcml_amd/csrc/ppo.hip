// Fused MAT-PPO loss (forward value + analytic gradients) and fused flat clip+Adam for gfx950.
//
// Loss = policy clip loss - entropy_coef * entropy + value_loss_coef * value loss, exactly as
// mat_trainer.py:54-156 (reference): importance weight exp(logp - old), clipped surrogate min, active-masked or
// plain means, ValueNorm-normalised returns (update with the minibatch first, beta = 0.99999, debiased, var
// clamped at 1e-2), clipped value prediction, Huber(delta) or MSE, max(orig, clipped).  Instead of ~80 autograd
// kernels the trainer runs:
//   ppo_reduce    — per-minibatch sums (returns, returns^2 per objective, active count), block partials + atomics
//   ppo_vn_update — ValueNorm running-moment update from those sums (one wave)
//   ppo_grad      — per-token loss terms and d(loss)/d(logp, entropy, value); loss scalars accumulated by atomics
// and feeds the gradients straight into the fused decoder/encoder backward kernels.
//   adam_norm / adam_step — global grad-norm (clip_grad_norm_ semantics: scale = min(1, max/(norm+1e-6)))
//   and one Adam update over the flat fp32 parameter / gradient / moment buffers (torch.optim.Adam maths,
//   L2 weight decay added to the gradient).
#include "common.h"
#include "gather_rows.h"

using namespace mdl;

struct PPOArgs {
  int n;            // tokens in the minibatch (sequences x agents)
  int n_obj;        // value objectives (1 or 2)
  const float* v;   // (n, n_obj)
  const float* logp;      // (n)
  const float* ent;       // (n)
  const float* old_logp;  // (n)
  const float* adv;       // (n, n_obj)  (already normalised)
  const float* vpred;     // (n, n_obj) old value predictions
  const float* ret;       // (n, n_obj) returns
  const float* active;    // (n)
  float* dv; float* dlogp; float* dent;
  float* stats;     // [0..n_obj) sum ret, [n_obj..2n_obj) sum ret^2, [2n_obj] count, [2n_obj+1] sum active
                    // (DP all-reduces the first 2n_obj+1: ValueNorm sees the global batch, losses stay local means)
  float* out;       // accumulators: policy loss, value loss, entropy, ratio (added to, never cleared here)
  float* vn;        // ValueNorm: running_mean[n_obj], running_mean_sq[n_obj], debiasing_term
  float clip, coef_v, coef_e, huber_delta, beta, eps, omb;   // omb = 1 - beta computed in double on the host
  int use_huber, use_clip_v, use_vam, use_pam, use_vn, update_vn;
  int n_lp;         // log-prob / entropy entries per token (continuous action type: one per action dimension)
  // round 6: old_logp / adv / vpred / ret / active are the rollout buffer's rows read through the epoch permutation
  // (sidx[minibatch sequence] = buffer sequence of L tokens; null = dense minibatch arrays), and the advantages are
  // standardised here from the epoch's masked sums ((x - mean) / (std + eps), rl_ops.hip gather_rows' arithmetic)
  const long long* sidx;
  int L;
  const double* adv_sums;   // null: adv already standardised
  float adv_eps;
};

__device__ __forceinline__ size_t ppo_src(const PPOArgs& a, int i) {
  if (!a.sidx) return (size_t)i;
  const int s = i / a.L;
  return (size_t)a.sidx[s] * (size_t)a.L + (size_t)(i - s * a.L);
}
__device__ __forceinline__ void adv_norm_params(const PPOArgs& a, float& mean, float& sd) {
  mean = 0.f;
  sd = 1.f;
  if (!a.adv_sums) return;
  const double cnt = a.adv_sums[2] < 1.0 ? 1.0 : a.adv_sums[2];
  const double m = a.adv_sums[0] / cnt;
  double var = a.adv_sums[1] / cnt - m * m;
  var = var < 0.0 ? 0.0 : var;
  mean = (float)m;
  sd = (float)sqrt(var) + a.adv_eps;
}

#define MAXOBJ 2

__global__ __launch_bounds__(256) void ppo_reduce_kernel(PPOArgs a) {
  __shared__ float sm[4][2 * MAXOBJ + 2];
  float acc[2 * MAXOBJ + 2];
  const int K = 2 * a.n_obj + 2;
#pragma unroll
  for (int k = 0; k < 2 * MAXOBJ + 2; ++k) acc[k] = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
    const size_t si = ppo_src(a, i);
    for (int o = 0; o < a.n_obj; ++o) {
      const float r = a.ret[si * a.n_obj + o];
      acc[o] += r;
      acc[a.n_obj + o] += r * r;
    }
    acc[2 * a.n_obj] += 1.f;
    acc[2 * a.n_obj + 1] += a.active[si];
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = 0; k < K; ++k) {
    const float s = wave_sum(acc[k]);
    if (lane == 0) sm[wid][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sm[w][threadIdx.x];
    atomicAdd(a.stats + threadIdx.x, s);
  }
}

__global__ void ppo_vn_update_kernel(PPOArgs a) {
  // reference ValueNorm.update (per_element_update False): w = beta for every minibatch
  const int o = threadIdx.x;
  const float cnt = a.stats[2 * a.n_obj];
  const float w = a.beta, omw = a.omb;   // 1 - 0.99999 rounded in fp32 is 0.13% off: take it from the host
  if (o < a.n_obj) {
    const float m = a.stats[o] / cnt, sq = a.stats[a.n_obj + o] / cnt;
    a.vn[o] = a.vn[o] * w + m * omw;
    a.vn[a.n_obj + o] = a.vn[a.n_obj + o] * w + sq * omw;
  }
  __syncthreads();
  if (o == 0) a.vn[2 * a.n_obj] = a.vn[2 * a.n_obj] * w + omw;
}

__device__ __forceinline__ float huber_grad(float e, float d) { return fabsf(e) <= d ? e : (e > 0.f ? d : -d); }
__device__ __forceinline__ float huber(float e, float d) {
  const float ae = fabsf(e);
  return ae <= d ? 0.5f * e * e : d * (ae - 0.5f * d);
}

// FUSE_VN (round 6): the ValueNorm update of ppo_vn_update_kernel is computed by EVERY workgroup from the running
// moments and this minibatch's statistics (the same fp32 expressions, so the same values), and the LAST workgroup to
// finish (an arrival counter) writes the new moments back — all reads of the old moments precede every arrival, so
// one launch replaces two.  ctr: a zeroed int the last workgroup re-zeroes.
template <bool FUSE_VN>
__device__ __forceinline__ void ppo_grad_body(const PPOArgs& a, unsigned int* ctr) {
  __shared__ float sm[4][4];
  const float sum_a = a.stats[2 * a.n_obj + 1], n = (float)a.n;
  const float inv_pa = a.use_pam ? 1.f / fmaxf(sum_a, 1.f) : 1.f / n;
  const float inv_va = (a.use_vam ? 1.f / fmaxf(sum_a, 1.f) : 1.f / n) / (float)a.n_obj;
  float mean[MAXOBJ], istd[MAXOBJ], vnew[2 * MAXOBJ + 1];
  {
    const float cnt = a.stats[2 * a.n_obj];
    for (int o = 0; o < 2 * a.n_obj + 1; ++o) {
      float x = a.vn[o];
      if (FUSE_VN) {   // ppo_vn_update_kernel's arithmetic
        if (o < a.n_obj) x = x * a.beta + (a.stats[o] / cnt) * a.omb;
        else if (o < 2 * a.n_obj) x = x * a.beta + (a.stats[o] / cnt) * a.omb;
        else x = x * a.beta + a.omb;
      }
      vnew[o] = x;
    }
    const float d = fmaxf(vnew[2 * a.n_obj], a.eps);
    for (int o = 0; o < a.n_obj; ++o) {
      const float m = vnew[o] / d;
      const float var = fmaxf(vnew[a.n_obj + o] / d - m * m, 1e-2f);
      mean[o] = a.use_vn ? m : 0.f;
      istd[o] = a.use_vn ? rsqrtf(var) : 1.f;
    }
  }
  float adv_mean, adv_sd;
  adv_norm_params(a, adv_mean, adv_sd);
  float pl = 0.f, vl = 0.f, el = 0.f, rl = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
    const size_t si = ppo_src(a, i);
    const float act = a.active[si];
    // policy: -min(r A, clip(r) A)
    // multi-objective MAT (momat / dmomat): one advantage per objective, the surrogate summed over objectives
    // (mat_trainer.py:129-139 on (B, A, n_obj) advantages: min(...).sum(-1))
    // continuous action type: one ratio per action dimension, the surrogate summed over dimensions.  Entropy
    // (transformer_policy.py:212-215 on (N, A) entropies): with policy active masks Σ(ent * active) / Σ active —
    // summed over the dimensions, per active token; without, the mean over every (token, dimension) entry.
    const float wp = a.use_pam ? act * inv_pa : inv_pa;
    const float we = a.use_pam ? wp : wp / (float)a.n_lp;
    const float inv_lp = 1.f / (float)a.n_lp;
    for (int k = 0; k < a.n_lp; ++k) {
      const size_t q = (size_t)i * a.n_lp + k;
      const float imp = __expf(a.logp[q] - a.old_logp[si * a.n_lp + k]);
      const float ic = fminf(fmaxf(imp, 1.f - a.clip), 1.f + a.clip);
      float dm = 0.f, sm_ = 0.f;
      for (int o = 0; o < a.n_obj; ++o) {
        float ad = a.adv[si * a.n_obj + o];
        if (a.adv_sums) ad = (ad - adv_mean) / adv_sd;
        const float s1 = imp * ad, s2 = ic * ad;
        if (s1 <= s2) dm += imp * ad;
        else dm += (imp >= 1.f - a.clip && imp <= 1.f + a.clip) ? imp * ad : 0.f;  // clamp passes grad inclusively
        sm_ += fminf(s1, s2);
      }
      pl -= sm_ * wp;
      a.dlogp[q] = -wp * dm;
      // entropy bonus
      a.dent[q] = -a.coef_e * we;
      el += a.ent[q] * we;
      rl += imp * inv_lp;
    }
    // value
    const float wv = a.use_vam ? act * inv_va : inv_va;
    for (int o = 0; o < a.n_obj; ++o) {
      const size_t j = (size_t)i * a.n_obj + o, sj = si * a.n_obj + o;
      const float v = a.v[j], vp = a.vpred[sj];
      const float dvc = v - vp;
      const float vc = vp + fminf(fmaxf(dvc, -a.clip), a.clip);
      const float tgt = (a.ret[sj] - mean[o]) * istd[o];
      const float eo = tgt - v, ec = tgt - vc;
      const float lo = a.use_huber ? huber(eo, a.huber_delta) : 0.5f * eo * eo;
      const float lc = a.use_huber ? huber(ec, a.huber_delta) : 0.5f * ec * ec;
      const float go = -(a.use_huber ? huber_grad(eo, a.huber_delta) : eo);
      const float gc = -(a.use_huber ? huber_grad(ec, a.huber_delta) : ec) * ((dvc >= -a.clip && dvc <= a.clip) ? 1.f : 0.f);
      float l, g;
      if (a.use_clip_v) {
        if (lo >= lc) { l = lo; g = go; } else { l = lc; g = gc; }
      } else { l = lo; g = go; }
      vl += l * wv;
      a.dv[j] = a.coef_v * wv * g;
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float r4[4] = {pl, vl, el, rl / n};
  for (int k = 0; k < 4; ++k) {
    const float s = wave_sum(r4[k]);
    if (lane == 0) sm[wid][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sm[w][threadIdx.x];
    atomicAdd(a.out + threadIdx.x, s);
  }
  if (FUSE_VN && threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(ctr, 1u) == gridDim.x - 1) {   // the last workgroup: every other one has read the old moments
      for (int o = 0; o < 2 * a.n_obj + 1; ++o) a.vn[o] = vnew[o];
      *ctr = 0u;
      __threadfence();
    }
  }
}
__global__ __launch_bounds__(256) void ppo_grad_kernel(PPOArgs a) { ppo_grad_body<false>(a, nullptr); }
__global__ __launch_bounds__(256) void ppo_grad_vn_kernel(PPOArgs a, unsigned int* ctr) { ppo_grad_body<true>(a, ctr); }

static int ppo_grid(int n) {
  int g = (n + 255) / 256;
  return g > 1024 ? 1024 : (g < 1 ? 1 : g);
}

MDL_API int mdl_ppo_loss(const PPOArgs* a, hipStream_t st) {
  if (a->n_obj < 1 || a->n_obj > MAXOBJ) return -1;
  hipMemsetAsync(a->stats, 0, sizeof(float) * (2 * a->n_obj + 2), st);
  hipLaunchKernelGGL(ppo_reduce_kernel, dim3(ppo_grid(a->n)), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  if (a->update_vn) {
    hipLaunchKernelGGL(ppo_vn_update_kernel, dim3(1), dim3(64), 0, st, *a);
    MDL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(ppo_grad_kernel, dim3(ppo_grid(a->n)), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}

// the reduce half alone (DP: all-reduce the sums between reduce and update)
MDL_API int mdl_ppo_reduce(const PPOArgs* a, hipStream_t st) {
  hipMemsetAsync(a->stats, 0, sizeof(float) * (2 * a->n_obj + 2), st);
  hipLaunchKernelGGL(ppo_reduce_kernel, dim3(ppo_grid(a->n)), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}

// ValueNorm update + loss gradients in ONE launch (FUSE_VN); ctr: a zeroed device uint the kernel leaves zeroed
MDL_API int mdl_ppo_finish_fused(const PPOArgs* a, unsigned int* ctr, hipStream_t st) {
  if (!a->update_vn) {
    hipLaunchKernelGGL(ppo_grad_kernel, dim3(ppo_grid(a->n)), dim3(256), 0, st, *a);
  } else {
    hipLaunchKernelGGL(ppo_grad_vn_kernel, dim3(ppo_grid(a->n)), dim3(256), 0, st, *a, ctr);
  }
  MDL_CHECK_LAUNCH();
  return 0;
}

MDL_API int mdl_ppo_finish(const PPOArgs* a, hipStream_t st) {
  if (a->update_vn) {
    hipLaunchKernelGGL(ppo_vn_update_kernel, dim3(1), dim3(64), 0, st, *a);
    MDL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(ppo_grad_kernel, dim3(ppo_grid(a->n)), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------- flat Adam
struct AdamArgs {
  int n;
  float* p; const float* g; float* m; float* v;
  float* sumsq;       // [1] grad norm (logging), [2] skipped steps, [3] Σ of the norms since the trainer cleared it,
                      // [4 .. 4 + ADAM_NB) per-workgroup Σ g² partials
  float lr, beta1, beta2, eps, wd, t, max_norm;   // t = optimizer steps attempted so far, this one included
  int clip;
  int npart;          // Σ g² partials written (the step sums exactly these; 0 = ADAM_NB)
};

// The norm pass writes one Σ g² partial per workgroup; every step workgroup sums the ADAM_NB partials itself in a
// fixed order (bit-identical norm everywhere, run to run) — no memset, no same-address atomics.  1024 partials: the
// single-GPU trainer computes them inside the gradient-workspace reduction (grad_reduce_norm_kernel, one workgroup
// per partial at the reduction's full width) and skips the norm launch.
constexpr int ADAM_NB = 1024;
constexpr int ADAM_NORM_NB = 128;   // the standalone norm pass (data-parallel path)

__global__ __launch_bounds__(256) void adam_norm_kernel(AdamArgs a) {
  __shared__ float sm[4];
  float s = 0.f;
  const int n4 = a.n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(a.g);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const float4 x = g4[i];
    s += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  for (int i = (n4 << 2) + blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x)
    s += a.g[i] * a.g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) a.sumsq[4 + blockIdx.x] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

__global__ __launch_bounds__(256) void adam_step_kernel(AdamArgs a) {
  __shared__ float snorm;
  if (threadIdx.x < 64) {   // wave 0: Σ of the ADAM_NB partials (ADAM_NB / 64 per lane, fixed order)
    float v = 0.f;
    const int np = a.npart > 0 ? a.npart : ADAM_NB;
    for (int j = threadIdx.x; j < np; j += 64) v += a.sumsq[4 + j];
    const float tot = wave_sum(v);
    if (threadIdx.x == 0) snorm = sqrtf(tot);
  }
  __syncthreads();
  const float norm = snorm;
  const float skipped = a.sumsq[2];   // read by every workgroup before workgroup 0 may bump it below
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.sumsq[1] = norm;
    a.sumsq[3] += norm;   // per-iteration logging sum (the eager path adds every step's norm, finite or not)
  }
  if (!isfinite(norm)) {   // non-finite guard: skip the whole step (params and moments untouched)
    if (blockIdx.x == 0 && threadIdx.x == 0) a.sumsq[2] = skipped + 1.f;   // skipped-step counter
    return;
  }
  const float scale = a.clip ? fminf(1.f, a.max_norm / (norm + 1e-6f)) : 1.f;
  // bias corrections from the APPLIED step count (attempted minus skipped non-finite steps, both on device), as
  // torch.optim.Adam, which never sees a skipped step; nobody writes sumsq[2] on a non-skipped step
  const float t = a.t - skipped;
  const float ib1 = 1.f / (1.f - powf(a.beta1, t)), ib2 = 1.f / (1.f - powf(a.beta2, t));
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
    float g = a.g[i] * scale;
    float p = a.p[i];
    if (a.wd != 0.f) g += a.wd * p;
    const float m = a.m[i] * a.beta1 + (1.f - a.beta1) * g;
    const float v = a.v[i] * a.beta2 + (1.f - a.beta2) * g * g;
    a.m[i] = m;
    a.v[i] = v;
    p -= a.lr * (m * ib1) / (sqrtf(v * ib2) + a.eps);
    a.p[i] = p;
  }
}

MDL_API int mdl_adam_scratch_floats() { return 4 + ADAM_NB; }

// norm_ready: the Σ g² partials are already in sumsq[4..] (mdl_grad_reduce_norm over the same final gradient)
MDL_API int mdl_adam(const AdamArgs* a, int norm_ready, hipStream_t st) {
  int g = (a->n + 255) / 256;
  if (g > 1024) g = 1024;
  AdamArgs b = *a;
  // the standalone norm pass (data parallelism: the all-reduced gradient) runs its round-4 grid of 128 workgroups and
  // the step sums exactly those partials; norm_ready: ADAM_NB partials from the workspace reduction
  b.npart = norm_ready ? ADAM_NB : ADAM_NORM_NB;
  if (!norm_ready) {
    hipLaunchKernelGGL(adam_norm_kernel, dim3(ADAM_NORM_NB), dim3(256), 0, st, b);
    MDL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(adam_step_kernel, dim3(g), dim3(256), 0, st, b);
  MDL_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------- dW workspace
// g[i] += sum_k ws[k * stride + i]; ws zeroed for the next minibatch (the training kernels spread their weight-
// gradient atomics over `copies` copies, see mat_train_common.h Ctx::gofs).
// all the copies' loads of an element first (independent, in flight together), then the zero stores: with the
// store after each load the loads serialised behind possibly-aliasing stores (32 dependent memory round trips)
__global__ __launch_bounds__(256) void grad_reduce_kernel(float* g, float* ws, int n, long long stride, int copies) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= copies; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ws[(size_t)(k + j) * stride + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < copies; ++k) s += ws[(size_t)k * stride + i];
    for (k = 0; k < copies; ++k) ws[(size_t)k * stride + i] = 0.f;
    g[i] += s;
  }
}

// ... and, for the whole flat buffer, the optimizer's Σ g² partials of the FINAL gradient in the same pass (one per
// workgroup, sumsq[4 + blockIdx], ADAM_NB workgroups: the Adam step then skips its norm launch)
__global__ __launch_bounds__(256) void grad_reduce_norm_kernel(float* g, float* ws, int n, long long stride, int copies,
                                                               float* sumsq) {
  __shared__ float sm[4];
  float q = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= copies; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ws[(size_t)(k + j) * stride + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < copies; ++k) s += ws[(size_t)k * stride + i];
    for (k = 0; k < copies; ++k) ws[(size_t)k * stride + i] = 0.f;
    const float gi = g[i] + s;
    g[i] = gi;
    q += gi * gi;
  }
  q = wave_sum(q);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) sumsq[4 + blockIdx.x] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

MDL_API int mdl_grad_reduce_norm(float* g, float* ws, int n, long long stride, int copies, float* sumsq, hipStream_t st) {
  hipLaunchKernelGGL(grad_reduce_norm_kernel, dim3(ADAM_NB), dim3(256), 0, st, g, ws, n, stride, copies, sumsq);
  MDL_CHECK_LAUNCH();
  return 0;
}

// Reduction of the private copies, one tile of 64 float4 (256 floats) per workgroup of 256 threads: wave w sums
// copies [w C/4, (w+1) C/4) of the tile (16 loads in flight, 1 KB coalesced per wave-instruction), wave 0 adds the
// four group sums in a fixed order — a fixed summation tree, so the result is deterministic, and 4x the memory
// parallelism of one thread per element walking all C copies (the 256-copy reduction was latency-bound: 32 round
// trips of 8 loads per thread).  Writes g[dst[.]] and returns this thread's Σ g² (wave 0's lanes; 0 elsewhere).
__device__ __forceinline__ float priv_reduce_tile(float* g, const float* ws, const int* dst, int tile, int lo, int n,
                                                  long long stride, int copies, int accumulate) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ f4v part[4][64];
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i4 = tile * 64 + e, n4 = n >> 2;
  const bool in = i4 >= (lo >> 2) && i4 < n4;   // [lo, n): a tile straddling a range bound reduces only its part
  const size_t st4 = (size_t)(stride >> 2);
  const int k0 = (copies * grp) >> 2, k1 = (copies * (grp + 1)) >> 2;
  f4v s = {0.f, 0.f, 0.f, 0.f};
  if (in) {
    const f4v* w4 = reinterpret_cast<const f4v*>(ws) + i4;
    int k = k0;
    for (; k + 16 <= k1; k += 16) {
      f4v v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = __builtin_nontemporal_load(w4 + (size_t)(k + j) * st4);
#pragma unroll
      for (int j = 0; j < 16; ++j) s += v[j];
    }
    for (; k < k1; ++k) s += __builtin_nontemporal_load(w4 + (size_t)k * st4);
  }
  part[grp][e] = s;
  __syncthreads();
  float q = 0.f;
  if (grp == 0 && in) {
    const f4v t = ((part[0][e] + part[1][e]) + part[2][e]) + part[3][e];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = dst[4 * i4 + j];
      const float gi = accumulate ? g[d] + t[j] : t[j];
      g[d] = gi;
      q += gi * gi;
    }
  }
  __syncthreads();   // part[] is reused by the next tile
  return q;
}

// Private-copy workspace (round 6, mat_train_common.h GradMode): one copy per workgroup of the backward launches,
// every entry a workgroup writes rewritten by its first chunk — so no zero fill, and a fixed summation order:
//   g[dst[s]] = (accumulate ? g[dst[s]] : 0) + Σ_{k < copies} ws[k * stride + s]   (k ascending)
// dst maps the fragment-order 64 x 64 weight gradients back to row-major (identity elsewhere); the loads run along
// the copies' own order (coalesced), the stores are the permuted ones.  sumsq (optional): the optimizer's Σ g²
// partial of the FINAL gradient per workgroup (sumsq[4 + blockIdx], ADAM_NB workgroups), as grad_reduce_norm.
__global__ __launch_bounds__(256) void grad_reduce_priv_kernel(float* g, const float* ws, const int* dst, int lo,
                                                               int n, long long stride, int copies, int accumulate,
                                                               float* sumsq) {
  __shared__ float sm[4];
  float q = 0.f;
  // [lo, n) in tiles of 256 floats (lo, n multiples of 4: parameter ranges are 16-float padded)
  const int t0 = lo >> 8, t1 = (n + 255) >> 8;
  for (int t = t0 + blockIdx.x; t < t1; t += gridDim.x) {
    // a tile straddling lo / n reduces only its in-range float4s: the elements outside belong to another call
    q += priv_reduce_tile(g, ws, dst, t, lo, n, stride, copies, accumulate);
  }
  if (!sumsq) return;
  q = wave_sum(q);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) sumsq[4 + blockIdx.x] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

// elements [lo, hi) of the flat gradient (a parameter range: no 64 x 64 matrix straddles it); sumsq whole-buffer only
MDL_API int mdl_grad_reduce_priv(float* g, const float* ws, const int* dst, int lo, int hi, long long stride,
                                 int copies, int accumulate, float* sumsq, hipStream_t st) {
  if (copies < 1 || lo < 0 || hi < lo || (sumsq && lo != 0) || (lo & 3) || (hi & 3) || (stride & 3)) return -1;
  hipLaunchKernelGGL(grad_reduce_priv_kernel, dim3(ADAM_NB), dim3(256), 0, st, g, ws, dst, lo, hi, stride, copies,
                     accumulate, sumsq);
  MDL_CHECK_LAUNCH();
  return 0;
}

MDL_API int mdl_grad_reduce(float* g, float* ws, int n, long long stride, int copies, hipStream_t st) {
  int grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3(grid), dim3(256), 0, st, g, ws, n, stride, copies);
  MDL_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------- fused update (round 6)
// The single-GPU end of a minibatch in TWO launches instead of four (grad_reduce + adam_norm / adam_step +
// pack_weights, and the flat-buffer memset): grad_reduce_priv_kernel folds the private workspace copies with the
// Σ g² partials, then adam_pack_kernel sums the partials in a fixed order (the same norm in every workgroup, run to
// run), applies clip + Adam, and repacks each 64 x 64 weight matrix it owns from LDS into the training kernels'
// fragment orders (csrc/rl_ops.hip pack_weights layout): workgroups 0 .. nmat-1 own one matrix each, the others
// update the remaining parameters (rest[]).
// (A one-launch cooperative variant with a grid barrier measured ~330 us per call: every workgroup's agent-scope
// fences wrote back / invalidated its XCD's L2 — two launches cost ~40 us.)
struct PackEntU { const float* src; unsigned short* fw; unsigned short* bw; unsigned short* fa; unsigned short* ba; };
struct UpdArgs {
  float* g; const float* ws; const int* dst; int n; long long stride; int copies; int accumulate;
  AdamArgs a;
  const PackEntU* tab; const int* mat_off; int nmat;   // packed matrices and their flat offsets
  const int* rest; int n_rest;                         // flat indices of every other parameter element
  unsigned int* bar;                                   // (unused: the one-launch variant's barrier words)
  GatherArgs ga;   // the NEXT minibatch's gather (ga.n = 0: none), run by extra workgroups of the adam_pack launch
  int ga_wg;       // their count
};

__device__ __forceinline__ float adam_elem(const AdamArgs& a, int i, float scale, float ib1, float ib2) {
  float g = a.g[i] * scale;
  float p = a.p[i];
  if (a.wd != 0.f) g += a.wd * p;
  const float m = a.m[i] * a.beta1 + (1.f - a.beta1) * g;
  const float v = a.v[i] * a.beta2 + (1.f - a.beta2) * g * g;
  a.m[i] = m;
  a.v[i] = v;
  p -= a.lr * (m * ib1) / (sqrtf(v * ib2) + a.eps);
  a.p[i] = p;
  return p;
}

__global__ __launch_bounds__(1024) void adam_pack_kernel(UpdArgs u) {
  __shared__ float snorm;
  __shared__ float Mf[4096];
  const int base = (int)gridDim.x - u.ga_wg;
  if ((int)blockIdx.x >= base) {   // the next minibatch's rows: independent of this update (and of its finite check)
    const int wpb = blockDim.x >> 6;
    gather_rows_wavewise(u.ga, ((int)blockIdx.x - base) * wpb + (int)(threadIdx.x >> 6), u.ga_wg * wpb,
                         threadIdx.x & 63);
    return;
  }
  const AdamArgs& a = u.a;
  if (threadIdx.x < 64) {   // Σ of the ADAM_NB partials of grad_reduce_priv, fixed order
    float v = 0.f;
    for (int j = threadIdx.x; j < ADAM_NB; j += 64) v += a.sumsq[4 + j];
    const float tot = wave_sum(v);
    if (threadIdx.x == 0) snorm = sqrtf(tot);
  }
  __syncthreads();
  const float norm = snorm;
  const float skipped = a.sumsq[2];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.sumsq[1] = norm;
    a.sumsq[3] += norm;
  }
  if (!isfinite(norm)) {   // non-finite guard: params, moments and packs untouched
    if (blockIdx.x == 0 && threadIdx.x == 0) a.sumsq[2] = skipped + 1.f;
    return;
  }
  const float scale = a.clip ? fminf(1.f, a.max_norm / (norm + 1e-6f)) : 1.f;
  const float t = a.t - skipped;
  const float ib1 = 1.f / (1.f - powf(a.beta1, t)), ib2 = 1.f / (1.f - powf(a.beta2, t));
  if ((int)blockIdx.x < u.nmat) {
    const int off = u.mat_off[blockIdx.x];
    for (int e = threadIdx.x; e < 4096; e += blockDim.x) Mf[e] = adam_elem(a, off + e, scale, ib1, ib2);
    __syncthreads();
    const PackEntU pe = u.tab[blockIdx.x];
    for (int idx = threadIdx.x; idx < 4096; idx += blockDim.x) {
      const int j = idx & 7, lane = (idx >> 3) & 63, ks = (idx >> 9) & 1, ct = idx >> 10;
      const int n = 16 * ct + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + j;
      if (pe.fw) pe.fw[idx] = mdl::f2bf(Mf[n * 64 + k]);
      if (pe.bw) pe.bw[idx] = mdl::f2bf(Mf[k * 64 + n]);
      const int kp = 32 * ks + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
      if (pe.fa) pe.fa[idx] = mdl::f2bf(Mf[n * 64 + kp]);
      if (pe.ba) pe.ba[idx] = mdl::f2bf(Mf[kp * 64 + n]);
    }
  } else {
    const int nb = base - u.nmat;
    for (int r = (blockIdx.x - u.nmat) * blockDim.x + threadIdx.x; r < u.n_rest; r += nb * blockDim.x)
      adam_elem(a, u.rest[r], scale, ib1, ib2);
  }
}

MDL_API int mdl_update_fused(const UpdArgs* u, hipStream_t st) {
  if (u->copies < 1 || u->nmat < 0 || u->n_rest < 0 || (u->n & 3) || (u->stride & 3)) return -1;
  UpdArgs v = *u;
  v.ga_wg = 0;
  if (v.ga.n > 0 && v.ga.rows > 0) {   // the next minibatch's gather: one wave per (entry, row) item, <= 384 WGs
    if (const int rc = gather_check(v.ga)) return rc;
    for (int k = 0; k < v.ga.n; ++k)
      if (v.ga.e[k].width > 1024) return -3;   // wide rows: the standalone gather (gather_rows_kernel)
    const int items = v.ga.n * v.ga.rows;
    v.ga_wg = (items + 15) / 16 < 384 ? (items + 15) / 16 : 384;
  }
  hipLaunchKernelGGL(grad_reduce_priv_kernel, dim3(ADAM_NB), dim3(256), 0, st, v.g, v.ws, v.dst, 0, v.n, v.stride,
                     v.copies, v.accumulate, v.a.sumsq);
  MDL_CHECK_LAUNCH();
  const int rest_wg = (v.n_rest + 1023) / 1024;   // 1024-thread workgroups: a matrix's 4096 elements in 4 steps
  hipLaunchKernelGGL(adam_pack_kernel, dim3(v.nmat + (rest_wg < 64 ? rest_wg : 64) + v.ga_wg), dim3(1024), 0, st, v);
  MDL_CHECK_LAUNCH();
  return 0;
}
