// Device-vectorised bid-first DCML environment for gfx950.
//
// One workgroup per env, one lane per worker (blockDim = W rounded up to 64).  dcml_env_step runs the whole
// reference env step for its env and then the next task's reset in the same launch, so a rollout step costs
// ONE launch for all E envs:
//   step  — DCML_BID_FIRST_MA_ENV_SingleProcess.py:57-144 + Worker.process (DCML_Worker_TIMESLOT_MultiProcess.py:46-112)
//   reset — DCML_BID_FIRST_MA_ENV_SingleProcess.py:157-274 (+ DCML_Master.reset, Worker.bid)
// Draw-for-draw identical to the torch path (mat_dcml_amd/envs/dcml/vec_env.py): same Philox counters, same
// float32 rounding for the bid profile (explicit __fmul_rn/__fadd_rn: no FMA contraction), worker maths in
// double.  The K-th order statistic is a rank count over the selected workers' delays staged in LDS.
#include "common.h"

using namespace mdl;

struct EnvCfg {
  int E, W, A, P, obs_dim, share_dim;
  int fixed, preset, max_disable, max_slot_iters, preset_rows, shannon;
  uint32_t k0, k1;
  double r_min, r_max, c_min, c_max, r_hi, c_hi, pr_min, pr_max;
  double rate, freq, bit_to_byte, continue_prob, alpha, beta, standalone_penalty, fixed_k_ratio;
  // Shannon links (Shannon.py:6-21): band = B_total / W, noise in mW, uniform ranges, path-loss exponent
  double band, noise, mp_lo, mp_hi, wp_lo, wp_hi, d_lo, d_hi, ple;
  float master_feature;
};

struct EnvState {
  const int64_t* gid;        // (E)
  const float* profiles;     // (W, P)
  int64_t* counter;          // (E) next task counter
  int64_t* task_ctr;         // (E) counter of the current task
  double* R; double* C; double* master_pr;   // (E)
  double* worker_pr;         // (E, W)
  bool* avail;               // (E, W)
  int64_t* n_disable;        // (E)
  int64_t* arrive;           // (E)
  float* lw;                 // (E, W, P)
  float* obs;                // (E, A, 7)
  float* share;              // (E, W+2)
  float* ava;                // (E, A, 2)
  int64_t* preset_idx;       // (E)
  const double* preset_master;   // (rows, 3)
  const double* preset_prs;      // (rows, W)
  const int64_t* preset_disable; // (rows)
  double* rate;              // (E, W) download rate per link (constant unless Shannon)
  double* up_rate;           // (E, W) upload rate per link (only reported in share_obs)
};

struct StepOut {
  const float* actions;  // (E, A)
  float* reward; bool* done; float* delay; float* payment;  // (E)
  double* dbg;           // optional (E, 6 + 3W) parity record: N, K, standalone, final delay, payment, reward, then
                         // per worker the transmission count n, the consumed slots and the worker's delay
};

#define MAXW 256
#define MAXP 64

__device__ __forceinline__ double geom_extra(uint32_t u, double pr) {
  if (!(pr > 0.0)) return 0.0;
  const double U = u01_open(u);
  double safe = fmin(fmax(pr, 1e-300), 1.0 - 1e-12);
  return floor(log(U) / log(safe));
}

// block-wide sum of one double per thread (blockDim <= MAXW); uses scratch[>= blockDim/64]
__device__ double block_sum_d(double v, double* scratch) {
  v = wave_sum_d(v);
  const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

// ----------------------------------------------------------------------------------------------- reset
__device__ void env_reset(const EnvCfg& c, const EnvState& s, int e) {
  __shared__ uint32_t s_key[MAXW];
  __shared__ unsigned long long s_ballot[MAXW / 64];
  __shared__ double s_red[MAXW / 64];
  const int w = threadIdx.x;
  const int W = c.W, P = c.P;
  const uint32_t g = (uint32_t)s.gid[e];
  const int64_t ctr64 = s.counter[e];
  const uint32_t ctr = (uint32_t)ctr64;
  // master draws (every lane computes them: cheaper than a broadcast)
  u4 um = philox4x32_10(ctr, g, 0u, P_MASTER, c.k0, c.k1);
  double R = c.r_min + floor(u01_open(um.x) * (c.r_hi - c.r_min + 1.0));
  double C = c.c_min + floor(u01_open(um.y) * (c.c_hi - c.c_min + 1.0));
  double mpr = c.pr_min + u01_open(um.z) * (c.pr_max - c.pr_min);
  int64_t dis = 1 + (int64_t)floor(u01_open(um.w) * (double)c.max_disable);
  u4 ua = philox4x32_10(ctr, g, 0u, P_ARRIVE, c.k0, c.k1);
  const int arrive = (int)floor(u01_open(ua.x) * (double)P);
  double wpr = 0.0;
  uint32_t key = 0xFFFFFFFFu;
  if (w < W) {
    u4 uw = philox4x32_10(ctr, g, (uint32_t)w, P_WORKER_PR, c.k0, c.k1);
    wpr = c.pr_min + u01_open(uw.x) * (c.pr_max - c.pr_min);
    key = uw.y;
  }
  if (c.preset) {
    int64_t idx = s.preset_idx[e];
    if (idx > c.preset_rows - 1) idx = c.preset_rows - 1;
    R = s.preset_master[idx * 3 + 0];
    C = s.preset_master[idx * 3 + 1];
    mpr = s.preset_master[idx * 3 + 2];
    if (w < W) wpr = s.preset_prs[idx * W + w];
    dis = s.preset_disable[idx];
  }
  double rate_dn = c.rate, rate_up = c.rate;
  if (c.shannon) {   // DCML_Master.get_transmission_rate (:41-45) + Shannon.upload/download (:14-21)
    mpr = 0.0;
    u4 um2 = philox4x32_10(ctr, g, 0xFFFFu, P_SHANNON, c.k0, c.k1);
    const double mp = c.mp_lo + u01_open(um2.x) * (c.mp_hi - c.mp_lo);
    if (w < W) {
      u4 us = philox4x32_10(ctr, g, (uint32_t)w, P_SHANNON, c.k0, c.k1);
      const double d = c.d_lo + u01_open(us.x) * (c.d_hi - c.d_lo);
      const double wp = c.wp_lo + u01_open(us.y) * (c.wp_hi - c.wp_lo);
      const double gain = pow(d, c.ple) / c.noise;
      rate_dn = c.band * log2(1.0 + mp * gain);
      rate_up = c.band * log2(1.0 + wp * gain);
    }
  }
  if (dis < 0) dis = 0;
  if (dis > W - 1) dis = W - 1;
  if (w < W) s_key[w] = key;
  __syncthreads();
  bool av = false;
  if (w < W) {
    int rank = 0;
    for (int v = 0; v < W; ++v) {
      const uint32_t kv = s_key[v];
      rank += (kv < key) || (kv == key && v < w);
    }
    av = rank >= dis;
  }
  // available-before-me count (prefix popcount over the block)
  const unsigned long long bal = __ballot(av);
  if ((threadIdx.x & 63) == 0) s_ballot[threadIdx.x >> 6] = bal;
  __syncthreads();
  int before = 0;
  {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = 0; i < wid; ++i) before += __popcll(s_ballot[i]);
    before += __popcll(s_ballot[wid] & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
  }
  // bid profile: clip(profile * U(0.8,1.2), 0, 1) in float32, no contraction
  float l0 = 0.f, l1 = 0.f, l2 = 0.f;
  if (w < W) {
    float* lwp = s.lw + ((size_t)e * W + w) * P;
    for (int k = 0; k < (P + 3) / 4; ++k) {
      u4 un = philox4x32_10(ctr, g, (uint32_t)w + ((uint32_t)k << 16), P_NOISE, c.k0, c.k1);
      uint32_t uu[4] = {un.x, un.y, un.z, un.w};
      for (int j = 0; j < 4 && 4 * k + j < P; ++j) {
        const float nf = __fadd_rn(__fmul_rn(u01_open_f(uu[j]), 0.4f), 0.8f);
        float v = __fmul_rn(s.profiles[w * P + 4 * k + j], nf);
        v = fminf(fmaxf(v, 0.f), 1.f);
        lwp[4 * k + j] = v;
      }
    }
    l0 = lwp[arrive];
    l1 = lwp[(arrive + 1) % P];
    l2 = lwp[(arrive + 2) % P];
  }
  const float Rn = (float)((R - c.r_min) / (c.r_max - c.r_min));
  const float Cn = (float)((C - c.c_min) / (c.c_max - c.c_min));
  const float denom = (float)(W - dis);
  if (w < W) {
    float* o = s.obs + ((size_t)e * c.A + w) * c.obs_dim;
    const float bf = (float)before;
    o[0] = Rn; o[1] = Cn;
    if (av) {
      o[2] = l0; o[3] = l1; o[4] = l2; o[5] = (float)wpr; o[6] = bf / denom;
    } else {
      o[2] = 1.f; o[3] = 1.f; o[4] = 1.f; o[5] = 1.f; o[6] = before >= 1 ? (bf - 1.f) / denom : 0.f;
    }
    s.worker_pr[(size_t)e * W + w] = wpr;
    s.avail[(size_t)e * W + w] = av;
    if (c.shannon) {   // share = R, C, upload/1e7, download/1e7 (ENV_SingleProcess.py:253-255)
      s.share[(size_t)e * c.share_dim + 2 + w] = (float)(rate_up / 1e7);
      s.share[(size_t)e * c.share_dim + 2 + W + w] = (float)(rate_dn / 1e7);
      s.rate[(size_t)e * W + w] = rate_dn;
      s.up_rate[(size_t)e * W + w] = rate_up;
    } else {
      s.share[(size_t)e * c.share_dim + 2 + w] = (float)wpr;
    }
    float* a = s.ava + ((size_t)e * c.A + w) * 2;
    a[0] = 1.f; a[1] = av ? 1.f : 0.f;
  }
  const double fa = av ? 1.0 : 0.0;
  const double n_av = block_sum_d(fa, s_red);
  const double s0 = block_sum_d(av ? (double)l0 : 0.0, s_red);
  const double s1 = block_sum_d(av ? (double)l1 : 0.0, s_red);
  const double s2 = block_sum_d(av ? (double)l2 : 0.0, s_red);
  const double sp = block_sum_d(av ? wpr : 0.0, s_red);
  if (threadIdx.x == 0) {
    const double na = n_av < 1.0 ? 1.0 : n_av;
    float* o = s.obs + ((size_t)e * c.A + W) * c.obs_dim;
    o[0] = Rn; o[1] = Cn;
    o[2] = (float)(s0 / na); o[3] = (float)(s1 / na); o[4] = (float)(s2 / na); o[5] = (float)(sp / na);
    o[6] = c.master_feature;
    float* a = s.ava + ((size_t)e * c.A + W) * 2;
    a[0] = 1.f; a[1] = 1.f;
    s.share[(size_t)e * c.share_dim + 0] = Rn;
    s.share[(size_t)e * c.share_dim + 1] = Cn;
    s.R[e] = R; s.C[e] = C; s.master_pr[e] = mpr;
    s.n_disable[e] = dis;
    s.arrive[e] = arrive;
    s.task_ctr[e] = ctr64;
    s.counter[e] = ctr64 + 1;
    s.preset_idx[e] = s.preset_idx[e] + 1;
  }
  __syncthreads();
}

__global__ __launch_bounds__(MAXW) void dcml_env_reset_kernel(EnvCfg c, EnvState s) {
  env_reset(c, s, blockIdx.x);
}

// ----------------------------------------------------------------------------------------------- step
__global__ __launch_bounds__(MAXW) void dcml_env_step_kernel(EnvCfg c, EnvState s, StepOut out) {
  __shared__ double s_red[MAXW / 64];
  __shared__ double s_delay[MAXW];
  const int e = blockIdx.x;
  const int w = threadIdx.x;
  const int W = c.W, P = c.P;
  const uint32_t g = (uint32_t)s.gid[e];
  const uint32_t ctr = (uint32_t)s.task_ctr[e];
  const float* act = out.actions + (size_t)e * c.A;
  const bool valid = w < W;
  const bool av = valid ? s.avail[(size_t)e * W + w] : false;
  double strat = 0.0;
  if (c.fixed) strat = av ? 1.0 : 0.0;
  else if (valid) strat = (double)act[w];
  const double N0 = block_sum_d(strat, s_red);
  double K;
  if (c.fixed) K = floor(N0 * c.fixed_k_ratio);
  else K = ceil(N0 * (double)act[W]);
  const bool standalone = (N0 == 0.0);
  double N = fmin(fmax(N0, 1.0), (double)W);
  K = fmin(fmax(K, 1.0), N);
  if (standalone) K = 1.0;
  const double R = s.R[e], C = s.C[e];
  const double r = ceil(R / K), cc = C;
  const double arrive = (double)s.arrive[e];
  const float* lw = s.lw + ((size_t)e * W + (valid ? w : 0)) * P;
  double delay = 0.0, nslots = 0.0, price0 = 0.0;
  int tp0 = 0;
  if (valid) {
    const double pr = s.worker_pr[(size_t)e * W + w];
    const double rate = c.shannon ? s.rate[(size_t)e * W + w] : c.rate;  // Worker.process: download rate, both legs
    double need = ceil((9.0 * r - 3.0) * cc) / c.freq;
    u4 ud = philox4x32_10(ctr, g, (uint32_t)w, P_DOWNLOAD, c.k0, c.k1);
    double n = 1.0 + geom_extra(ud.x, pr);
    const double transmit = ((ceil((r + 1.0) * cc) * c.bit_to_byte) / rate + 0.001) * n;
    price0 = floor(transmit) * 0.1;
    const double arrive_slot = floor(transmit + arrive);
    int tp = (int)fmod(arrive_slot, (double)P);
    tp0 = tp;
    const double frac = transmit - floor(transmit);
    const double lwt = (double)lw[tp];
    if (frac > lwt) need = need + frac - lwt;
    double availability = 0.0;
    const double up_unit = (r * c.bit_to_byte) / rate + 0.001;
    int it = 0;
    while (availability < need && it < c.max_slot_iters) {
      const double a = 1.0 - (double)lw[tp];
      u4 uu = philox4x32_10(ctr, g, (uint32_t)w + ((uint32_t)it << 16), P_UPLOAD, c.k0, c.k1);
      n += geom_extra(uu.x, pr);
      availability += a;
      nslots += 1.0;
      tp = (tp + 1) % P;
      ++it;
    }
    const double upload = up_unit * n + 0.02;
    delay = arrive_slot + nslots - arrive - (availability - need) + upload;
    if (out.dbg) {
      double* d = out.dbg + (size_t)e * (6 + 3 * W) + 6;
      d[w] = n;
      d[W + w] = nslots;
      d[2 * W + w] = delay;
    }
  }
  // K-th order statistic of the selected workers' delays (ties broken by index)
  const bool sel = valid && strat > 0.5;
  s_delay[w] = sel ? delay : INFINITY;
  __syncthreads();
  double mine = -1.0;
  if (sel) {
    int cnt = 0;
    for (int v = 0; v < W; ++v) {
      const double dv = s_delay[v];
      cnt += (dv < delay) || (dv == delay && v < w);
    }
    if (cnt == (int)K - 1) mine = delay;
  }
  // the selected ranks are a permutation of 0..nsel-1, so exactly one lane holds rank K-1
  double final_delay = block_sum_d(mine > 0.0 ? mine : 0.0, s_red);
  __shared__ double s_d0;
  if (threadIdx.x == 0) s_d0 = delay;  // worker 0: the standalone branch
  __syncthreads();
  if (standalone) final_delay = s_d0;
  const double end = ceil(final_delay);
  // price at index min(end, nslots) - 1 and the last price
  double price_end = price0, price_last = price0;
  if (valid) {
    const int cnt_end = (int)fmin(end, nslots);
    const int ns = (int)nslots;
    int tp = tp0;
    double acc = 0.0;
    for (int j = 0; j < ns; ++j) {
      acc += 1.0 - (double)lw[tp];
      if (j == cnt_end - 1) price_end = price0 + acc;
      tp = (tp + 1) % P;
    }
    price_last = price0 + acc;
  }
  double pay = block_sum_d(strat * price_end, s_red);
  __shared__ double s_last0;
  if (threadIdx.x == 0) s_last0 = price_last;
  __syncthreads();
  if (standalone) pay = s_last0;
  if (threadIdx.x == 0) {
    double rew = -(c.alpha * final_delay + c.beta * pay);
    if (standalone) rew *= c.standalone_penalty;
    u4 udn = philox4x32_10(ctr, g, 0u, P_DONE, c.k0, c.k1);
    out.reward[e] = (float)rew;
    out.done[e] = u01_open(udn.x) < c.continue_prob;
    out.delay[e] = (float)final_delay;
    out.payment[e] = (float)pay;
    if (out.dbg) {
      double* d = out.dbg + (size_t)e * (6 + 3 * W);
      d[0] = N; d[1] = K; d[2] = standalone ? 1.0 : 0.0; d[3] = final_delay; d[4] = pay; d[5] = rew;
    }
  }
  __syncthreads();
  env_reset(c, s, e);  // every step starts a new task (ENV_SingleProcess.py:139)
}

static int block_for(int W) { return ((W + 63) / 64) * 64; }

MDL_API int mdl_dcml_env_reset(const EnvCfg* c, const EnvState* s, hipStream_t st) {
  if (c->W > MAXW || c->P > MAXP) return -1;
  hipLaunchKernelGGL(dcml_env_reset_kernel, dim3(c->E), dim3(block_for(c->W)), 0, st, *c, *s);
  MDL_CHECK_LAUNCH();
  return 0;
}

MDL_API int mdl_dcml_env_step(const EnvCfg* c, const EnvState* s, const StepOut* o, hipStream_t st) {
  if (c->W > MAXW || c->P > MAXP) return -1;
  hipLaunchKernelGGL(dcml_env_step_kernel, dim3(c->E), dim3(block_for(c->W)), 0, st, *c, *s, *o);
  MDL_CHECK_LAUNCH();
  return 0;
}
