// Observation embedding for wide observations (SMAC 27m_vs_30m: obs_dim 1288) on MFMA — the part of the encoder's
// obs_encoder (ma_transformer.py:133-134: LayerNorm(obs_dim) -> Linear(obs_dim, 64) -> GELU) that the fused encoder
// kernels (mat_enc_ct.hip, `pre_in`) cannot hold in a lane.  Output: pre = W_e · LN_obs(x) + b_e, [tok][64] f32.
//
// One pass over x (the only large operand: 5 KB per token) by folding the LayerNorm into the GEMM:
//   LN_obs(x)_k = (x_k - mu) r g_k + b_k  =>  pre_f = r (W' x)_f - r mu c1_f + c0_f,
//   W' = W_e diag(g) (bf16, packed per optimizer step), c1_f = Σ_k W'_fk (of the rounded W'), c0_f = W_e b + b_e,
// with mu / r from the same pass (Σx, Σx² per token).  x enters the MFMA as a hi/lo bf16 pair (≈16 significant
// bits) so the r·mu·c1 cancellation keeps fp32-like accuracy.
//
// Backward (no gradient w.r.t. the data): with P_tf = dpre_tf r_t,
//   M = Pᵀ x (64 x od, token reduction on MFMA),  u_f = Σ_t P_tf mu_t,  db_f = Σ_t dpre_tf,
//   dW_fk = g_k (M_fk - u_f) + b_k db_f,   dg_k = Σ_f W_fk (M_fk - u_f),   db_obs_k = Σ_f W_fk db_f,   db_e = db.
#include "mat_train_common.h"

namespace {

constexpr int OE_TOK = 16;   // tokens per forward workgroup (its 4 waves split the k-steps)

struct OEArgs {
  int N, od, KS;               // tokens, obs dim, k-steps of 32 (ceil(od / 32))
  const float* x;              // [N][od]
  const float* we;             // [64][od] W_e
  const float* be;             // [64]
  const float* g;              // [od] LN_obs weight
  const float* b;              // [od] LN_obs bias
  bf16_t* wpack;               // [KS][4][64 lanes][8] W' A fragments (natural k order)
  float* c01;                  // [2][64] c1, c0
  float* pre;                  // [N][64]
  float* stat;                 // [N][2] mu, rstd
  // backward
  const float* dpre;           // [N][64]
  float* M;                    // [64][od] workspace (zeroed by the host)
  float* ud;                   // [2][64] u, db workspace (zeroed by the host)
  float *d_we, *d_be, *d_g, *d_b;
  const bf16_t* xh;            // [N][od] bf16 observations (non-null: read instead of x — half the bytes, and x is
                               // exact in bf16 so the lo half of the hi / lo split vanishes)
};

// W' = W_e diag(g) as bf16 A fragments + c1 (from the rounded values) / c0.  One block per output feature f.
__global__ __launch_bounds__(256) void obs_embed_pack_kernel(OEArgs a) {
  const int f = blockIdx.x;
  float s1 = 0.f, s0 = 0.f;
  for (int k = threadIdx.x; k < a.KS * 32; k += 256) {
    const bool in = k < a.od;
    const float w = in ? a.we[(size_t)f * a.od + k] : 0.f;
    const uint16_t wb = f2bf(in ? w * a.g[k] : 0.f);
    s1 += bf2f(wb);
    s0 += in ? w * a.b[k] : 0.f;
    // fragment position: k-step s = k / 32, lane = 16 (k%32 / 8) + f%16, j = k % 8, mt = f / 16
    const int s = k >> 5, kk = k & 31, lane = 16 * (kk >> 3) + (f & 15), j = kk & 7, mt = f >> 4;
    a.wpack[(((size_t)s * 4 + mt) * 64 + lane) * 8 + j] = wb;
  }
  __shared__ float red[2][256];
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s0;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.c01[f] = red[0][0];
    a.c01[64 + f] = red[1][0] + a.be[f];
  }
}

// forward: one 16-token tile per workgroup, the k-steps dealt round robin to its OE_WAVES waves (token on lane & 15,
// features 16mt + 4g + r in registers), partial sums reduced through LDS in fixed wave order.  Round 2 gave each
// wave its own 16 tokens and all 41 k-steps of SMAC's 1288-wide rows: the rollout's 864 tokens were 14 workgroups
// of a 41-step dependent load chain (40 us per call); round 3: 4 waves, one step's loads at a time (25 us).  Round 4:
// each wave requests the x rows and weight fragments of OE_PF steps before converting / multiplying any of them (one
// load latency per OE_PF steps; 8 waves x 3 steps measured slower, 30.6 us: most of its steps fell to the tail).
constexpr int OE_WAVES = 4;
// TPW 16-token tiles per workgroup share each wave's weight fragments: at the training minibatch (SMAC: 86,400
// tokens) the fragments were 4 KB of L2 reads per 2 KB of x per step (145 us, 3 TB/s); the rollout's 864 tokens keep
// one tile per workgroup (parallelism) and a deeper prefetch
template <int TPW> struct OECfg { static constexpr int PF = TPW == 1 ? 5 : 2; };
template <int TPW>
struct OEStep { float4 x0[TPW], x1[TPW]; uint4 xb[TPW]; bf16x8 w[4]; };
template <bool XB>
__device__ __forceinline__ void oe_mma(const float (&v)[8], const bf16x8 (&w)[4], bool ok, f32x4 (&acc)[4], float& sx,
                                       float& sxx) {
  bf16x8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float xv = ok ? v[j] : 0.f;
    sx += xv;
    sxx += xv * xv;
    const uint16_t h = f2bf(xv);
    hi[j] = (short)h;
    if (!XB) lo[j] = (short)f2bf(xv - bf2f(h));
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[mt], hi, acc[mt], 0, 0, 0);
    if (!XB) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[mt], lo, acc[mt], 0, 0, 0);
  }
}
__device__ __forceinline__ void oe_unpack8(const uint4 u, float (&v)[8]) {
  const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(q[j] << 16);
    v[2 * j + 1] = __uint_as_float(q[j] & 0xFFFF0000u);
  }
}
template <int TPW, bool XB>
__global__ __launch_bounds__(64 * OE_WAVES) void obs_embed_fwd_kernel(OEArgs a) {
  constexpr int PF = OECfg<TPW>::PF;
  __shared__ f32x4 part[OE_WAVES - 1][TPW][4][64];
  __shared__ float pst[OE_WAVES - 1][TPW][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  int tok[TPW];
  bool ok[TPW];
  const float* xr[TPW];
  const bf16_t* xbr[TPW];
  f32x4 acc[TPW][4];
  float sx[TPW], sxx[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    tok[t] = (blockIdx.x * TPW + t) * OE_TOK + c;
    ok[t] = tok[t] < a.N;
    if (XB) xbr[t] = a.xh + (size_t)(ok[t] ? tok[t] : 0) * a.od;
    else xr[t] = a.x + (size_t)(ok[t] ? tok[t] : 0) * a.od;
    sx[t] = sxx[t] = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  int s = wave;
  if ((a.od & (XB ? 7 : 3)) == 0) {   // 16-byte rows: the steps whose 32 dims are all inside the row, PF at a time
    const int nfull = a.od >> 5;
    for (; s + OE_WAVES * (PF - 1) < nfull; s += OE_WAVES * PF) {
      OEStep<TPW> st[PF];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int k0 = 32 * (s + OE_WAVES * u) + 8 * g;
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          if (XB) {
            st[u].xb[t] = *(const uint4*)(xbr[t] + k0);
          } else {
            st[u].x0[t] = *(const float4*)(xr[t] + k0);
            st[u].x1[t] = *(const float4*)(xr[t] + k0 + 4);
          }
        }
        const bf16_t* wp = a.wpack + ((size_t)(s + OE_WAVES * u) * 4 * 64 + lane) * 8;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) st[u].w[mt] = *(const bf16x8*)(wp + (size_t)mt * 64 * 8);
      }
      __builtin_amdgcn_sched_barrier(0);   // every load above issues before the first conversion / MFMA
#pragma unroll
      for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          float v[8];
          if (XB) {
            oe_unpack8(st[u].xb[t], v);
          } else {
            v[0] = st[u].x0[t].x; v[1] = st[u].x0[t].y; v[2] = st[u].x0[t].z; v[3] = st[u].x0[t].w;
            v[4] = st[u].x1[t].x; v[5] = st[u].x1[t].y; v[6] = st[u].x1[t].z; v[7] = st[u].x1[t].w;
          }
          oe_mma<XB>(v, st[u].w, ok[t], acc[t], sx[t], sxx[t]);
        }
    }
  }
  for (; s < a.KS; s += OE_WAVES) {   // the rest (and rows that are not float4-aligned), one step at a time
    const int k0 = 32 * s + 8 * g;
    bf16x8 w[4];
    const bf16_t* wp = a.wpack + ((size_t)s * 4 * 64 + lane) * 8;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) w[mt] = *(const bf16x8*)(wp + (size_t)mt * 64 * 8);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      float v[8];
      if (XB) {
        if ((a.od & 7) == 0 && k0 + 8 <= a.od) {
          oe_unpack8(*(const uint4*)(xbr[t] + k0), v);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = k0 + j < a.od ? bf2f(xbr[t][k0 + j]) : 0.f;
        }
      } else if ((a.od & 3) == 0 && k0 + 8 <= a.od) {
        const float4 p = *(const float4*)(xr[t] + k0), q = *(const float4*)(xr[t] + k0 + 4);
        v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w; v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = k0 + j < a.od ? xr[t][k0 + j] : 0.f;
      }
      oe_mma<XB>(v, w, ok[t], acc[t], sx[t], sxx[t]);
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) part[wave - 1][t][mt][lane] = acc[t][mt];
      pst[wave - 1][t][0][lane] = sx[t];
      pst[wave - 1][t][1][lane] = sxx[t];
    }
  }
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
#pragma unroll
    for (int w = 0; w < OE_WAVES - 1; ++w) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[t][mt] += part[w][t][mt][lane];
      sx[t] += pst[w][t][0][lane];
      sxx[t] += pst[w][t][1][lane];
    }
    const float sxt = cross_row_sum(sx[t]), sxxt = cross_row_sum(sxx[t]);
    const float mu = sxt / (float)a.od;
    const float var = fmaxf(sxxt / (float)a.od - mu * mu, 0.f);
    const float r = rsqrtf(var + 1e-5f);
    if (ok[t]) {
      float* out = a.pre + (size_t)tok[t] * 64 + 4 * g;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f32x4 y;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int f = 16 * mt + 4 * g + q;
          y[q] = r * acc[t][mt][q] - r * mu * a.c01[f] + a.c01[64 + f];
        }
        *(f32x4*)(out + 16 * mt) = y;
      }
      if (g == 0) {
        a.stat[2 * (size_t)tok[t]] = mu;
        a.stat[2 * (size_t)tok[t] + 1] = r;
      }
    }
  }
}

// backward step 1: M += Pᵀ x over a token range, for one 64-column block of x.  Token-major swizzled bf16 LDS tiles
// of 32 tokens (P, x hi, x lo); wave w owns output rows f in [16w, 16w+16); 4 column tiles of 16.  The next tile's
// global loads (float4 when od % 4 == 0) are issued before this tile's MFMAs; 64 token ranges per column block
// (SMAC: 21 x 64 = 1,344 workgroups).  Round 2 (16 ranges, scalar loads, no prefetch) ran at ~0.4 TB/s: 628 us.
constexpr int OEB_SPLIT = 64;   // token ranges per column block
struct OEBTile { float p[8], x[8]; };
__device__ __forceinline__ void oeb_load(const OEArgs& a, int t, int t_hi, int col0, OEBTile& T) {
  const int lc = threadIdx.x & 7;
  const bool ok = t < t_hi;
  const int k0 = col0 + 8 * lc;
  const float rr = ok ? a.stat[2 * (size_t)t + 1] : 0.f;
  if (ok) {
    const float4* dp = (const float4*)(a.dpre + (size_t)t * 64 + 8 * lc);
    const float4 d0 = dp[0], d1 = dp[1];
    T.p[0] = d0.x * rr; T.p[1] = d0.y * rr; T.p[2] = d0.z * rr; T.p[3] = d0.w * rr;
    T.p[4] = d1.x * rr; T.p[5] = d1.y * rr; T.p[6] = d1.z * rr; T.p[7] = d1.w * rr;
    if (a.xh) {   // bf16 observations
      const bf16_t* xb = a.xh + (size_t)t * a.od;
      if ((a.od & 7) == 0 && k0 + 8 <= a.od) {
        oe_unpack8(*(const uint4*)(xb + k0), T.x);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) T.x[j] = k0 + j < a.od ? bf2f(xb[k0 + j]) : 0.f;
      }
      return;
    }
    const float* xr = a.x + (size_t)t * a.od;
    if ((a.od & 3) == 0 && k0 + 8 <= a.od) {
      const float4 x0 = *(const float4*)(xr + k0), x1 = *(const float4*)(xr + k0 + 4);
      T.x[0] = x0.x; T.x[1] = x0.y; T.x[2] = x0.z; T.x[3] = x0.w; T.x[4] = x1.x; T.x[5] = x1.y; T.x[6] = x1.z; T.x[7] = x1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) T.x[j] = k0 + j < a.od ? xr[k0 + j] : 0.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) { T.p[j] = 0.f; T.x[j] = 0.f; }
  }
}
__global__ __launch_bounds__(256) void obs_embed_bwd_m_kernel(OEArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Pt[32 * 64], Xh[32 * 64], Xl[32 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c16 = lane & 15, g = lane >> 4;
  const int col0 = blockIdx.x * 64;
  const int t_lo = (int)((long long)a.N * blockIdx.y / OEB_SPLIT), t_hi = (int)((long long)a.N * (blockIdx.y + 1) / OEB_SPLIT);
  const int row = threadIdx.x >> 3, lc = threadIdx.x & 7;
  const int o = (row << 6) + ((lc ^ ((row >> 1) & 7)) << 3);
  RT acc;
  rt_zero(acc);
  OEBTile T;
  if (t_lo < t_hi) oeb_load(a, t_lo + row, t_hi, col0, T);
  for (int t0 = t_lo; t0 < t_hi; t0 += 32) {
    {   // stage this tile: 32 tokens x 64 values of P = dpre * r and of x (hi / lo); thread -> (row, 8-column chunk)
      uint4 up, uh, ul;
      uint32_t* p32 = (uint32_t*)&up;
      uint32_t* h32 = (uint32_t*)&uh;
      uint32_t* l32 = (uint32_t*)&ul;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p32[j] = (uint32_t)f2bf(T.p[2 * j]) | ((uint32_t)f2bf(T.p[2 * j + 1]) << 16);
        const uint16_t h0 = f2bf(T.x[2 * j]), h1 = f2bf(T.x[2 * j + 1]);
        h32[j] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        l32[j] = (uint32_t)f2bf(T.x[2 * j] - bf2f(h0)) | ((uint32_t)f2bf(T.x[2 * j + 1] - bf2f(h1)) << 16);
      }
      *(uint4*)(Pt + o) = up;
      *(uint4*)(Xh + o) = uh;
      *(uint4*)(Xl + o) = ul;
    }
    __syncthreads();
    if (t0 + 32 < t_hi) oeb_load(a, t0 + 32 + row, t_hi, col0, T);   // next tile in flight under the MFMAs
    const bf16x8 pa = ld_frag_T(Pt, 0, 16 * wave, lane);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      acc.v[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ld_frag_T(Xh, 0, 16 * ct, lane), acc.v[ct], 0, 0, 0);
      if (!a.xh)   // bf16 observations: the lo half is zero
        acc.v[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ld_frag_T(Xl, 0, 16 * ct, lane), acc.v[ct], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * wave + 4 * g + r, k = col0 + 16 * ct + c16;
      if (k < a.od) atomicAdd(a.M + (size_t)f * a.od + k, acc.v[ct][r]);
    }
}

// backward step 1b: u_f = Σ_t dpre_tf r_t mu_t and db_f = Σ_t dpre_tf (thread = (token lane, feature))
__global__ __launch_bounds__(256) void obs_embed_bwd_u_kernel(OEArgs a) {
  const int f = threadIdx.x & 63, tl = threadIdx.x >> 6;
  float u = 0.f, d = 0.f;
  // unrolled: 8 tokens' loads in flight per thread (the rolled loop was one dependent load latency per token:
  // 33 us for SMAC's 86,400-token minibatch)
#pragma unroll 8
  for (int t = blockIdx.x * 4 + tl; t < a.N; t += gridDim.x * 4) {
    const float dp = a.dpre[(size_t)t * 64 + f];
    u += dp * a.stat[2 * (size_t)t + 1] * a.stat[2 * (size_t)t];
    d += dp;
  }
  __shared__ float su[4][64], sd[4][64];
  su[tl][f] = u;
  sd[tl][f] = d;
  __syncthreads();
  if (tl == 0) {
    atomicAdd(a.ud + f, su[0][f] + su[1][f] + su[2][f] + su[3][f]);
    atomicAdd(a.ud + 64 + f, sd[0][f] + sd[1][f] + sd[2][f] + sd[3][f]);
  }
}

// backward step 2: parameter gradients from M, u, db (one thread per obs dim k; d_be by the first 64 threads)
__global__ __launch_bounds__(256) void obs_embed_bwd_fin_kernel(OEArgs a) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 64 && a.d_be) atomicAdd(a.d_be + threadIdx.x, a.ud[64 + threadIdx.x]);
  if (k >= a.od) return;
  const float gk = a.g[k], bk = a.b[k];
  float dg = 0.f, dbo = 0.f;
#pragma unroll 16   // 16 features' loads in flight (rolled: 64 dependent load latencies, 38 us)
  for (int f = 0; f < 64; ++f) {
    const float m = a.M[(size_t)f * a.od + k] - a.ud[f], db = a.ud[64 + f], w = a.we[(size_t)f * a.od + k];
    if (a.d_we) atomicAdd(a.d_we + (size_t)f * a.od + k, gk * m + bk * db);
    dg += w * m;
    dbo += w * db;
  }
  if (a.d_g) atomicAdd(a.d_g + k, dg);
  if (a.d_b) atomicAdd(a.d_b + k, dbo);
}

}  // namespace

MDL_API int mdl_obs_embed_pack(const OEArgs* a, hipStream_t st) {
  if (a->od < 1 || a->KS * 32 < a->od) return -1;
  hipLaunchKernelGGL(obs_embed_pack_kernel, dim3(64), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}

MDL_API int mdl_obs_embed_fwd(const OEArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  const int tiles = (a->N + OE_TOK - 1) / OE_TOK;
  const bool xb = a->xh != nullptr;
  if (tiles >= 4 * 1024) {   // enough tiles to fill the chip four per workgroup
    if (xb) hipLaunchKernelGGL((obs_embed_fwd_kernel<4, true>), dim3((tiles + 3) / 4), dim3(64 * OE_WAVES), 0, st, *a);
    else hipLaunchKernelGGL((obs_embed_fwd_kernel<4, false>), dim3((tiles + 3) / 4), dim3(64 * OE_WAVES), 0, st, *a);
  } else {
    if (xb) hipLaunchKernelGGL((obs_embed_fwd_kernel<1, true>), dim3(tiles), dim3(64 * OE_WAVES), 0, st, *a);
    else hipLaunchKernelGGL((obs_embed_fwd_kernel<1, false>), dim3(tiles), dim3(64 * OE_WAVES), 0, st, *a);
  }
  MDL_CHECK_LAUNCH();
  return 0;
}

MDL_API int mdl_obs_embed_bwd(const OEArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  hipMemsetAsync(a->M, 0, sizeof(float) * 64 * (size_t)a->od, st);
  hipMemsetAsync(a->ud, 0, sizeof(float) * 128, st);
  hipLaunchKernelGGL(obs_embed_bwd_m_kernel, dim3((a->od + 63) / 64, OEB_SPLIT), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  hipLaunchKernelGGL(obs_embed_bwd_u_kernel, dim3(256), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  hipLaunchKernelGGL(obs_embed_bwd_fin_kernel, dim3((a->od + 255) / 256), dim3(256), 0, st, *a);
  MDL_CHECK_LAUNCH();
  return 0;
}
