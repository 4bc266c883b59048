// mat_decode_persistent — the whole MAT autoregressive action decode in ONE launch (gfx950 / CDNA4).
//
// Replaces the reference's rollout hot loop: L full decoder passes per env step, each re-running every row
// (mat_src/mat/algorithms/utils/transformer_act.py:76-99, 37-75 for the "batch decision" stride mode).
// Exactness: decoder row i depends only on shifted actions 0..i, so decoding one row (or
// one block of rows) at a time against a KV cache of the earlier rows reproduces the full recompute.
//
// Work decomposition (D = 64, 2 heads x 32, n_block = NB):
//   * one 256-thread workgroup = 4 waves owns EPW envs; its 16-row MFMA tile holds (env, row) pairs of the
//     current pass (stochastic rollout: 1 row per env; deterministic stride mode: up to 16/EPW rows per env);
//   * every 64x64 Linear is a 16x64x64 GEMM on v_mfma_f32_16x16x32_bf16: wave w owns output columns
//     [16w, 16w+16); its B fragments (all 10·NB+1 decoder weight matrices) are loaded ONCE into VGPRs and stay
//     register-resident for the whole decode (one wave per SIMD, ~170 VGPRs of weights);
//   * activations move through LDS; the post-LN residual sums are kept in f32 and LayerNorm is fused into the
//     NEXT GEMM's A-fragment load (each lane normalises the 16 values it feeds the MFMA, row statistics by two
//     xor-shuffles), so no separate LN phase/barrier exists;
//   * the self- and cross-attention K/V caches of every block live in LDS as bf16 with an XOR-swizzled 16-byte
//     chunk order (conflict-free row gathers); attention over <= L cached rows runs on the VALU,
//     8 lanes per (tile row, head);
//   * the action head, availability masking, inverse-CDF categorical sampling / Normal sampling, log-probs and
//     the next row's action-embedding token are fused into the last phase.
// Inputs rep (encoder output, f32), ava, and the uniform / normal draws come from HBM — staged into LDS once at
// kernel start when they fit (`stage`), so no row of the sequential agent loop waits on an HBM miss (the rep row
// of phase D and the mask / draws of the head phase were first-touch loads on the critical path); outputs are
// actions and log-probs (B, L).  Numerics: bf16 MFMA operands, f32 accumulation, f32 LayerNorm / softmax / log-softmax.
#include "common.h"
#include <cstdlib>

using namespace mdl;

struct DecParams {
  const bf16_t* wpack;   // [(10*NB+1)][4 waves][2 ksteps][64 lanes][8]
  const float* bias;     // [(10*NB+1)][64]
  const float* lnp;      // [(3*NB+1)][2][64]  (ln1, ln2, ln3 per block; head LN last)
  const float* emb;      // [n_tok][64] = LN(GELU(W_a · token)) rows: start, action 0..A-1, zero
  const float* wh2;      // [act_dim][64]
  const float* bh2;      // [act_dim]
  const float* stdv;     // [act_dim]  sigmoid(log_std) * 0.5 (continuous agents)
  const float* rep;      // [B][L][64]
  const float* ava;      // [B][L][act_dim] or null
  const float* rnd_u;    // [B][L]
  const float* rnd_n;    // [B][L][act_dim]
  float* out_a;          // [B][L]
  float* out_lp;         // [B][L]
  int B, L, act_dim, n_disc, stride, deterministic, epw, rmax, n_tok, tok_start, tok_zero;
  int stage;             // 1: rep / ava / draws of the workgroup's envs are staged in LDS at kernel start
  int cont;              // 1: "Continuous" action type — every agent samples act_dim Gaussians and the next
                         //    row's input is LN(GELU(W_a · x + b_a)) of the sampled vector (not a token row)
  const float* wa;       // [64][act_dim] action-encoder weight (cont)
  const float* ba;       // [64] action-encoder bias (cont)
  const float* lnd;      // [2][64] decoder input LayerNorm (cont)
};

constexpr int SP = 68;   // f32 staging row pitch (floats)
constexpr int XP = 72;   // bf16 A staging row pitch (elements)

__device__ __forceinline__ int kv_off(int b, int kind, int m, int j, int col, int epw, int L) {
  // 64-element rows of 8 x 16-byte chunks; chunk index XOR (j & 7) spreads row gathers over all banks
  const int chunk = (col >> 3) ^ (j & 7);
  return ((((b * 4 + kind) * epw + m) * L + j) << 6) + (chunk << 3) + (col & 7);
}

#ifdef MDL_DECODE_PROF
__device__ unsigned long long g_attn_prof[8];
#define MDL_ATT_MARK(k) do { if (aprof) { const unsigned long long t_ = clock64(); g_attn_prof[k] += t_ - at_; at_ = t_; } } while (0)
#define MDL_ATT_INIT() const bool aprof = blockIdx.x == 0 && tid == 0; unsigned long long at_ = clock64()
#else
#define MDL_ATT_INIT() do { } while (0)
#define MDL_ATT_MARK(k) do { } while (0)
#endif

__device__ __forceinline__ f32x4 mfma2(const bf16x8 a[2], const bf16x8 w[2], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], w[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], w[1], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ bf16x8 pack8(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(v[j]);
  return r;
}

// A fragment from an f32 LDS row with fused LayerNorm.  Lane (g = lane>>4, r = lane&15) owns row r, columns
// 8g..8g+7 and 32+8g..32+8g+7.  xf receives the normalised f32 values (for the residual copy).
__device__ __forceinline__ void afrag_ln(const float* S, const float* gam, const float* bet, int lane,
                                        bf16x8 a[2], float xf[16]) {
  const int g = lane >> 4, r = lane & 15;
  const float* row = S + r * SP;
  float v[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) { v[j] = row[8 * g + j]; v[8 + j] = row[32 + 8 * g + j]; }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += v[j];
  s = cross_row_sum(s);
  const float mean = s * (1.f / 64.f);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) { const float d = v[j] - mean; q += d * d; }
  q = cross_row_sum(q);
  const float rstd = rsqrtf(q * (1.f / 64.f) + 1e-5f);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c0 = 8 * g + j, c1 = 32 + 8 * g + j;
    xf[j] = (v[j] - mean) * rstd * gam[c0] + bet[c0];
    xf[8 + j] = (v[8 + j] - mean) * rstd * gam[c1] + bet[c1];
  }
  a[0] = pack8(xf);
  a[1] = pack8(xf + 8);
}

// A fragment from an f32 row pointer (per lane) without normalisation
__device__ __forceinline__ void afrag_rowf(const float* row, int lane, bf16x8 a[2], float xf[16]) {
  const int g = lane >> 4;
  if (row) {
    const float4* p0 = (const float4*)(row + 8 * g);
    const float4* p1 = (const float4*)(row + 32 + 8 * g);
    float4 x0 = p0[0], x1 = p0[1], y0 = p1[0], y1 = p1[1];
    xf[0] = x0.x; xf[1] = x0.y; xf[2] = x0.z; xf[3] = x0.w; xf[4] = x1.x; xf[5] = x1.y; xf[6] = x1.z; xf[7] = x1.w;
    xf[8] = y0.x; xf[9] = y0.y; xf[10] = y0.z; xf[11] = y0.w; xf[12] = y1.x; xf[13] = y1.y; xf[14] = y1.z; xf[15] = y1.w;
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) xf[j] = 0.f;
  }
  a[0] = pack8(xf);
  a[1] = pack8(xf + 8);
}

__device__ __forceinline__ void afrag_xa(const bf16_t* XA, int lane, bf16x8 a[2]) {
  const int g = lane >> 4, r = lane & 15;
  a[0] = *(const bf16x8*)(XA + r * XP + 8 * g);
  a[1] = *(const bf16x8*)(XA + r * XP + 32 + 8 * g);
}

// write the normalised/raw f32 A-row values of this lane back to an f32 LDS staging buffer (row r, its cols)
__device__ __forceinline__ void store_xf(float* X, int lane, const float xf[16]) {
  const int g = lane >> 4, r = lane & 15;
#pragma unroll
  for (int j = 0; j < 8; ++j) { X[r * SP + 8 * g + j] = xf[j]; X[r * SP + 32 + 8 * g + j] = xf[8 + j]; }
}


// Causal attention of the pass's live tile rows over cached rows 0..i of their env.  lpi lanes (half a wave at
// the rollout shape) per (tile row, head): scores with lanes striding over the keys; P·V with the lanes split
// into 8 groups of 4 output dims x lpi/8 key groups (each lane sums ~i/(lpi/8) keys, the key groups combined by
// DPP / permlane shuffles).  An item's lanes live in one wave, so the score -> P·V hand-off through PR needs only
// a wave-level LDS wait.  Latency structure (the decode runs one row per env per step): only live items are
// visited (dead tile rows' XA rows are never consumed by a live row — MFMA rows are independent — and XA is
// zeroed once at kernel start), and the score / P·V loops issue all their LDS loads before using any of them
// (indices clamped to row i and masked, instead of per-key branches that serialised the load latencies).
template <int lpi>
__device__ __forceinline__ void attention_phase_t(const bf16_t* KV, const float* Q, float* PR, bf16_t* XA,
                                                  const int* ROWI, int R, int EPW, int L, int b, int kind,
                                                  float scale, int tid, int live) {
  const int u = tid & (lpi - 1);
  const int dg = u & 7, kg = u >> 3, nkg = lpi >> 3;
  MDL_ATT_INIT();
  for (int item = tid / lpi; item < 2 * live; item += 256 / lpi) {
    const int t = item >> 1, h = item & 1;
    const int i = ROWI[t];          // uniform over the item's lanes; >= 0 for every live row
    const int m = t / R;
    float* pr = PR + (t * 2 + h) * L;
    float q[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) q[d] = Q[t * SP + 32 * h + d];
    MDL_ATT_MARK(0);
    auto krow_of = [&](int j) { return KV + kv_off(b, kind, m, j, 0, EPW, L) - ((0 ^ (j & 7)) << 3); };
    // the first KR keys of every lane: loads for all of them first, then the dot products (four independent
    // 8-long FMA chains per key), masked beyond row i
    constexpr int KR = lpi >= 32 ? 2 : 4;
    bf16x8 kv[KR][4];
#pragma unroll
    for (int kk = 0; kk < KR; ++kk) {
      const int j = min(u + kk * lpi, i);
      const bf16_t* krow = krow_of(j);
#pragma unroll
      for (int lc = 0; lc < 4; ++lc) kv[kk][lc] = *(const bf16x8*)(krow + (((4 * h + lc) ^ (j & 7)) << 3));
    }
    float scr[KR];
    float mx = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < KR; ++kk) {
      float d4[4];
#pragma unroll
      for (int lc = 0; lc < 4; ++lc) {
        float d = 0.f;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) d += q[lc * 8 + jj] * bf2f((bf16_t)kv[kk][lc][jj]);
        d4[lc] = d;
      }
      scr[kk] = u + kk * lpi <= i ? ((d4[0] + d4[1]) + (d4[2] + d4[3])) * scale : -INFINITY;
      mx = fmaxf(mx, scr[kk]);
    }
    for (int j = u + KR * lpi; j <= i; j += lpi) {      // long rows only (L > KR * lpi)
      const bf16_t* krow = krow_of(j);
      float d4[4];
#pragma unroll
      for (int lc = 0; lc < 4; ++lc) {
        const bf16x8 k8 = *(const bf16x8*)(krow + (((4 * h + lc) ^ (j & 7)) << 3));
        float d = 0.f;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) d += q[lc * 8 + jj] * bf2f((bf16_t)k8[jj]);
        d4[lc] = d;
      }
      const float sc = ((d4[0] + d4[1]) + (d4[2] + d4[3])) * scale;
      pr[j] = sc;
      mx = fmaxf(mx, sc);
    }
    MDL_ATT_MARK(1);
    mx = group_max<lpi>(mx);
    MDL_ATT_MARK(2);
    float sum = 0.f;
#pragma unroll
    for (int kk = 0; kk < KR; ++kk) {
      const int j = u + kk * lpi;
      const float pj = j <= i ? __expf(scr[kk] - mx) : 0.f;
      if (j <= i) pr[j] = pj;
      sum += pj;
    }
    for (int j = u + KR * lpi; j <= i; j += lpi) {
      const float pj = __expf(pr[j] - mx);
      pr[j] = pj;
      sum += pj;
    }
    sum = group_sum<lpi>(sum);
    MDL_ATT_MARK(3);
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // PR written by this item's lanes (same wave)
    MDL_ATT_MARK(4);
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    const int lc = 4 * h + (dg >> 1), off = 4 * (dg & 1);
    for (int j0 = kg; j0 <= i; j0 += 4 * nkg) {         // 4 keys per lane per trip: loads first, then FMAs
      float pj[4];
      uint2 v4[4];
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const int j = j0 + uu * nkg, jc = min(j, i);
        pj[uu] = pr[jc];
        const bf16_t* vrow = KV + kv_off(b, kind + 1, m, jc, 0, EPW, L) - ((0 ^ (jc & 7)) << 3);
        v4[uu] = *(const uint2*)(vrow + ((lc ^ (jc & 7)) << 3) + off);
      }
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const float w = j0 + uu * nkg <= i ? pj[uu] : 0.f;
        acc0 += w * __uint_as_float(v4[uu].x << 16);
        acc1 += w * __uint_as_float(v4[uu].x & 0xFFFF0000u);
        acc2 += w * __uint_as_float(v4[uu].y << 16);
        acc3 += w * __uint_as_float(v4[uu].y & 0xFFFF0000u);
      }
    }
    MDL_ATT_MARK(5);
    if (lpi > 8) {   // reduce over the key groups kg: lane ^ 8 (DPP row_ror:8), then lane ^ 16
      acc0 += dppf<DPP_ROW_ROR8>(acc0); acc1 += dppf<DPP_ROW_ROR8>(acc1);
      acc2 += dppf<DPP_ROW_ROR8>(acc2); acc3 += dppf<DPP_ROW_ROR8>(acc3);
    }
    if (lpi > 16) {
      acc0 += xor16_partner(acc0); acc1 += xor16_partner(acc1);
      acc2 += xor16_partner(acc2); acc3 += xor16_partner(acc3);
    }
    if (kg == 0) {
      const float inv = 1.f / sum;
      bf16_t* xa = XA + t * XP + 32 * h + 4 * dg;
      xa[0] = f2bf(acc0 * inv); xa[1] = f2bf(acc1 * inv); xa[2] = f2bf(acc2 * inv); xa[3] = f2bf(acc3 * inv);
    }
    MDL_ATT_MARK(6);
  }
  MDL_ATT_MARK(7);
}

__device__ __forceinline__ void attention_phase(const bf16_t* KV, const float* Q, float* PR, bf16_t* XA,
                                                const int* ROWI, int R, int EPW, int L, int b, int kind,
                                                float scale, int tid, int lpi, int live) {
#ifdef MDL_LPI_ONLY32   // code-size experiment: rollout-only build (stride-mode passes need 16 / 8)
  attention_phase_t<32>(KV, Q, PR, XA, ROWI, R, EPW, L, b, kind, scale, tid, live);
#else
  if (lpi == 32) attention_phase_t<32>(KV, Q, PR, XA, ROWI, R, EPW, L, b, kind, scale, tid, live);
  else if (lpi == 16) attention_phase_t<16>(KV, Q, PR, XA, ROWI, R, EPW, L, b, kind, scale, tid, live);
  else attention_phase_t<8>(KV, Q, PR, XA, ROWI, R, EPW, L, b, kind, scale, tid, live);
#endif
}

// Action head: LN(head1 output) · W_h2 + b -> logits; availability mask, sampling, log-prob (16 lanes per row).
__device__ __forceinline__ void head_phase(const DecParams& p, const float* H1, float* LG, const float* lnh,
                                           const int* ROWI, int* PEND, int R, int s, int e, int env0, int tid,
                                           const float* AVA, const float* RU, const float* RN, bool stage,
                                           const float* wh2, const float* bh2, float* EROW) {
  const int t = tid >> 4, q = tid & 15;
  const int i = ROWI[t];
  const int AD = p.act_dim, L = p.L;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = H1[t * SP + 4 * q + k];
  float sm = v[0] + v[1] + v[2] + v[3];
  sm = group_sum<16>(sm);
  const float mean = sm * (1.f / 64.f);
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) { const float d = v[k] - mean; sq += d * d; }
  sq = group_sum<16>(sq);
  const float rstd = rsqrtf(sq * (1.f / 64.f) + 1e-5f);
  float hn[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) hn[k] = (v[k] - mean) * rstd * lnh[4 * q + k] + lnh[64 + 4 * q + k];
  for (int a = 0; a < AD; ++a) {
    const float* w = wh2 + a * 64 + 4 * q;
    float part = w[0] * hn[0] + w[1] * hn[1] + w[2] * hn[2] + w[3] * hn[3];
    part = group_sum<16>(part);
    if (q == 0) LG[t * SP + a] = part + bh2[a];
  }
  if (p.cont) {   // all act_dim dims are Gaussian; the 16 lanes of the row also build the next row's input
    if (i < 0 || i < s || i >= e) return;
    const int m = t / R;
    const size_t oi = (size_t)(env0 + m) * L + i, li = (size_t)m * L + i;
    const float* lg = LG + t * SP;
    float ev[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ev[k] = p.ba[4 * q + k];
    for (int a = 0; a < AD; ++a) {
      const float mean_a = lg[a], sd = p.stdv[a];
      const float x = p.deterministic ? mean_a : mean_a + sd * (stage ? RN[li * AD + a] : p.rnd_n[oi * AD + a]);
      if (q == 0) {
        const float z = (x - mean_a) / sd;
        p.out_a[oi * AD + a] = x;
        p.out_lp[oi * AD + a] = -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) ev[k] += p.wa[(4 * q + k) * AD + a] * x;
    }
    if (i + 1 >= L) return;
#pragma unroll
    for (int k = 0; k < 4; ++k) ev[k] = gelu_erf(ev[k]);
    float es = group_sum<16>(ev[0] + ev[1] + ev[2] + ev[3]);
    const float emean = es * (1.f / 64.f);
    float eq = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) { const float d = ev[k] - emean; eq += d * d; }
    eq = group_sum<16>(eq);
    const float erstd = rsqrtf(eq * (1.f / 64.f) + 1e-5f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cidx = 4 * q + k;
      EROW[m * 64 + cidx] = (ev[k] - emean) * erstd * p.lnd[cidx] + p.lnd[64 + cidx];
    }
    return;
  }
  if (q != 0 || i < 0 || i < s || i >= e) return;
  const int m = t / R, env = env0 + m;
  const float* lg = LG + t * SP;
  const size_t oi = (size_t)env * L + i;
  const size_t li = (size_t)m * L + i;                  // row in the staged (workgroup-local) inputs
  if (i < p.n_disc) {
    const float* av = p.ava ? (stage ? AVA + li * AD : p.ava + oi * AD) : nullptr;
    float mx = -INFINITY;
    int amax = 0;
    for (int a = 0; a < AD; ++a) {
      const float l = (av && av[a] == 0.f) ? -1e10f : lg[a];
      if (l > mx) { mx = l; amax = a; }
    }
    float se = 0.f;
    for (int a = 0; a < AD; ++a) se += __expf(((av && av[a] == 0.f) ? -1e10f : lg[a]) - mx);
    const float lse = mx + __logf(se);
    int act = amax;
    if (!p.deterministic) {
      const float uu = stage ? RU[li] : p.rnd_u[oi];
      float cdf = 0.f;
      int cnt = 0;
      for (int a = 0; a < AD; ++a) {
        cdf += __expf(((av && av[a] == 0.f) ? -1e10f : lg[a]) - lse);
        cnt += cdf < uu;
      }
      act = min(cnt, AD - 1);
    }
    const float la = (av && av[act] == 0.f) ? -1e10f : lg[act];
    p.out_a[oi] = (float)act;
    p.out_lp[oi] = la - lse;
    PEND[m * L + i] = act;
  } else {
    const int a = AD - 1;
    const float mean_a = lg[a], sd = p.stdv[a];
    const float x = p.deterministic ? mean_a : mean_a + sd * (stage ? RN[li * AD + a] : p.rnd_n[oi * AD + a]);
    const float z = (x - mean_a) / sd;
    p.out_a[oi] = x;
    p.out_lp[oi] = -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
    PEND[m * L + i] = -1;
  }
}

// Optional phase profiler (build with -DMDL_DECODE_PROF): thread 0 of workgroup 0 accumulates the core-clock
// cycles between consecutive barriers per phase; read back with mdl_decode_prof_read.
#ifdef MDL_DECODE_PROF
__device__ unsigned long long g_decode_prof[16];
#define MDL_PROF_MARK(k) do { if (prof_on) { const unsigned long long t_ = clock64(); prof[k] += t_ - prof_t; prof_t = t_; } } while (0)
// sub-phase marks: cycles since the previous (sub-)mark, WITHOUT resetting the phase timer's reference
#define MDL_PROF_SUB(k) do { if (prof_on) { const unsigned long long t_ = clock64(); prof[k] += t_ - prof_s; prof_s = t_; } } while (0)
#else
#define MDL_PROF_MARK(k) do { } while (0)
#define MDL_PROF_SUB(k) do { } while (0)
#endif

template <int NB>
__global__ __launch_bounds__(256, 1) void mat_decode_kernel(DecParams p) {
#ifdef MDL_DECODE_PROF
  const bool prof_on = blockIdx.x == 0 && threadIdx.x == 0;
  unsigned long long prof[16] = {0}, prof_t = clock64(), prof_s = prof_t;
#endif
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NG = 10 * NB + 1;
  constexpr int NLN = 3 * NB + 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g4 = lane >> 4, c16 = lane & 15;
  const int EPW = p.epw, L = p.L, AD = p.act_dim;
  const int env0 = blockIdx.x * EPW;
  const int n_env = min(EPW, p.B - env0);
  const int RMAX = p.rmax;

  // ---------------------------------------------------------------- LDS carve (16-byte aligned pieces)
  const size_t kv_elems = (size_t)NB * 4 * EPW * L * 64;
  bf16_t* KV = (bf16_t*)smem;
  char* ptr = smem + ((kv_elems * 2 + 15) & ~(size_t)15);
  float* S = (float*)ptr;   ptr += 16 * SP * 4;
  float* Q = (float*)ptr;   ptr += 16 * SP * 4;
  float* XR = (float*)ptr;  ptr += 16 * SP * 4;
  bf16_t* XA = (bf16_t*)ptr; ptr += 16 * XP * 2;
  float* LNP = (float*)ptr; ptr += NLN * 128 * 4;
  float* PR = (float*)ptr;  ptr += ((EPW * RMAX * 2 * L * 4 + 15) & ~15);
  int* TOK = (int*)ptr;     ptr += ((EPW * L * 4 + 15) & ~15);
  int* PEND = (int*)ptr;    ptr += ((EPW * L * 4 + 15) & ~15);
  int* ROWI = (int*)ptr;    ptr += 16 * 4;
  float* EROW = (float*)ptr; ptr += EPW * 64 * 4;            // cont: next row's input embedding per env
  float* REP = (float*)ptr;                                  // staged inputs (p.stage): [EPW][L][64]
  auto pad4 = [](size_t n) { return (n + 3) & ~(size_t)3; };  // keep every region 16-byte aligned
  float* AVA = REP + pad4((size_t)EPW * L * 64);             // [EPW][L][AD]
  float* RU = AVA + pad4((size_t)EPW * L * AD);              // [EPW][L]
  float* RN = RU + pad4((size_t)EPW * L);                    // [EPW][L][AD]
  float* EMB = RN + pad4((size_t)EPW * L * AD);              // [n_tok][64] action-embedding rows (float4 reads)
  float* WH2 = EMB + (size_t)p.n_tok * 64;                   // [AD][64], then bh2 [AD]
  const bool stage = p.stage != 0;

  // ---------------------------------------------------------------- one-time loads
  bf16x8 wb[NG][2];
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      wb[gi][ks] = *(const bf16x8*)(p.wpack + ((size_t)((gi * 4 + wave) * 2 + ks) * 64 + lane) * 8);
  }
  float bcol[NG];
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) bcol[gi] = p.bias[gi * 64 + 16 * wave + c16];
  for (int i = tid; i < NLN * 128; i += 256) LNP[i] = p.lnp[i];
  for (int i = tid; i < EPW * L; i += 256) { TOK[i] = (i % L == 0) ? p.tok_start : p.tok_zero; PEND[i] = -1; }
  for (int i = tid; i < 16 * XP; i += 256) XA[i] = 0;   // dead tile rows keep finite A-operand rows
  if (stage) {   // the workgroup's envs are contiguous in every input
    const int nrow = n_env * L;
    const float4* src = (const float4*)(p.rep + (size_t)env0 * L * 64);
    float4* dst = (float4*)REP;
    for (int i = tid; i < nrow * 16; i += 256) dst[i] = src[i];
    if (p.ava) for (int i = tid; i < nrow * AD; i += 256) AVA[i] = p.ava[(size_t)env0 * L * AD + i];
    if (p.rnd_u) for (int i = tid; i < nrow; i += 256) RU[i] = p.rnd_u[(size_t)env0 * L + i];
    if (p.rnd_n) for (int i = tid; i < nrow * AD; i += 256) RN[i] = p.rnd_n[(size_t)env0 * L * AD + i];
    for (int i = tid; i < p.n_tok * 64; i += 256) EMB[i] = p.emb[i];
    for (int i = tid; i < AD * 65; i += 256) WH2[i] = i < AD * 64 ? p.wh2[i] : p.bh2[i - AD * 64];
  }
  const float* emb = stage ? EMB : p.emb;
  const float* wh2 = stage ? WH2 : p.wh2;
  const float* bh2 = stage ? WH2 + AD * 64 : p.bh2;
  __syncthreads();

  const float scale = 0.17677669529663687f;  // 1/sqrt(32)

  // ---------------------------------------------------------------- block schedule (transformer_act.py:37-75)
  int prev_s = -1, s = 0, e = 1;
  while (true) {
    int lo = prev_s >= 0 ? prev_s + 1 : 0;
    if (lo > s) lo = s;
    for (int plo = lo; plo < e; plo += RMAX) {
      const int R = min(RMAX, e - plo);
      if (tid < 16) {
        const int m = tid / R, rr = tid % R;
        ROWI[tid] = (m < n_env && rr < R && tid < EPW * R) ? plo + rr : -1;
      }
      __syncthreads();
      MDL_PROF_MARK(0);
      // per-lane tile rows for the C layout (rows 4*g4 + r) and the A layout (row c16)
      int crow_i[4], crow_m[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { crow_i[r] = ROWI[4 * g4 + r]; crow_m[r] = (4 * g4 + r) / R; }
      const int arow_i = ROWI[c16], arow_m = c16 / R;
      const int live = n_env * R;                           // live tile rows this pass
      const int lpi = live <= 4 ? 32 : (live <= 8 ? 16 : 8);

#pragma unroll
      for (int b = 0; b < NB; ++b) {
        bf16x8 a[2];
        float xf[16];
        // ---------------- [A] x = emb(token) (b == 0) or LN3(S) ; q1, k1, v1
        if (b == 0) {
          const float* row = nullptr;
          if (arow_i >= 0)
            row = (p.cont && arow_i > 0) ? EROW + arow_m * 64 : emb + (size_t)TOK[arow_m * L + arow_i] * 64;
          afrag_rowf(row, lane, a, xf);
        } else {
          afrag_ln(S, LNP + (3 * (b - 1) + 2) * 128, LNP + (3 * (b - 1) + 2) * 128 + 64, lane, a, xf);
        }
        if (wave == 0) store_xf(XR, lane, xf);
        {
          f32x4 q1 = mfma2(a, wb[b * 10 + 0], f32x4{0, 0, 0, 0});
          f32x4 k1 = mfma2(a, wb[b * 10 + 1], f32x4{0, 0, 0, 0});
          f32x4 v1 = mfma2(a, wb[b * 10 + 2], f32x4{0, 0, 0, 0});
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * g4 + r;
            Q[row * SP + col] = q1[r] + bcol[b * 10 + 0];
            if (crow_i[r] >= 0) {
              KV[kv_off(b, 0, crow_m[r], crow_i[r], col, EPW, L)] = f2bf(k1[r] + bcol[b * 10 + 1]);
              KV[kv_off(b, 1, crow_m[r], crow_i[r], col, EPW, L)] = f2bf(v1[r] + bcol[b * 10 + 2]);
            }
          }
        }
        __syncthreads();
        MDL_PROF_MARK(1);
        // ---------------- [B] causal self-attention over cached rows 0..i
        attention_phase(KV, Q, PR, XA, ROWI, R, EPW, L, b, 0, scale, tid, lpi, live);
        __syncthreads();
        MDL_PROF_MARK(2);
        // ---------------- [C] proj1 + bias + residual x -> S
        afrag_xa(XA, lane, a);
        {
          f32x4 acc = mfma2(a, wb[b * 10 + 3], f32x4{0, 0, 0, 0});
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * g4 + r;
            S[row * SP + col] = acc[r] + bcol[b * 10 + 3] + XR[row * SP + col];
          }
        }
        __syncthreads();
        MDL_PROF_MARK(3);
        // ---------------- [D] x1 = LN1(S); k2, v2 from x1; q2 from rep_i
        afrag_ln(S, LNP + (3 * b + 0) * 128, LNP + (3 * b + 0) * 128 + 64, lane, a, xf);
        {
          bf16x8 ar[2];
          float rf[16];
          const float* rrow = arow_i < 0 ? nullptr
                              : stage ? REP + ((size_t)arow_m * L + arow_i) * 64
                                      : p.rep + ((size_t)(env0 + arow_m) * L + arow_i) * 64;
          afrag_rowf(rrow, lane, ar, rf);
          f32x4 k2 = mfma2(a, wb[b * 10 + 5], f32x4{0, 0, 0, 0});
          f32x4 v2 = mfma2(a, wb[b * 10 + 6], f32x4{0, 0, 0, 0});
          f32x4 q2 = mfma2(ar, wb[b * 10 + 4], f32x4{0, 0, 0, 0});
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * g4 + r;
            Q[row * SP + col] = q2[r] + bcol[b * 10 + 4];
            if (crow_i[r] >= 0) {
              KV[kv_off(b, 2, crow_m[r], crow_i[r], col, EPW, L)] = f2bf(k2[r] + bcol[b * 10 + 5]);
              KV[kv_off(b, 3, crow_m[r], crow_i[r], col, EPW, L)] = f2bf(v2[r] + bcol[b * 10 + 6]);
            }
          }
        }
        __syncthreads();
        MDL_PROF_MARK(4);
        // ---------------- [E] causal cross-attention (q = rep rows, k/v = x1 rows)
        attention_phase(KV, Q, PR, XA, ROWI, R, EPW, L, b, 2, scale, tid, lpi, live);
        __syncthreads();
        MDL_PROF_MARK(5);
        // ---------------- [F] proj2 + bias + rep_i -> S
        afrag_xa(XA, lane, a);
        {
          f32x4 acc = mfma2(a, wb[b * 10 + 7], f32x4{0, 0, 0, 0});
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * g4 + r;
            float res = 0.f;
            if (crow_i[r] >= 0)
              res = stage ? REP[((size_t)crow_m[r] * L + crow_i[r]) * 64 + col]
                          : p.rep[((size_t)(env0 + crow_m[r]) * L + crow_i[r]) * 64 + col];
            S[row * SP + col] = acc[r] + bcol[b * 10 + 7] + res;
          }
        }
        __syncthreads();
        MDL_PROF_MARK(6);
        // ---------------- [G] x2 = LN2(S) -> XR ; h = GELU(mlp1(x2)) -> XA
        MDL_PROF_SUB(12);
        afrag_ln(S, LNP + (3 * b + 1) * 128, LNP + (3 * b + 1) * 128 + 64, lane, a, xf);
        MDL_PROF_SUB(13);
        if (wave == 0) store_xf(XR, lane, xf);
        {
          f32x4 acc = mfma2(a, wb[b * 10 + 8], f32x4{0, 0, 0, 0});
          MDL_PROF_SUB(14);
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) XA[(4 * g4 + r) * XP + col] = f2bf(gelu_erf(acc[r] + bcol[b * 10 + 8]));
        }
        MDL_PROF_SUB(15);
        __syncthreads();
        MDL_PROF_MARK(7);
        // ---------------- [H] mlp2 + bias + residual x2 -> S
        afrag_xa(XA, lane, a);
        {
          f32x4 acc = mfma2(a, wb[b * 10 + 9], f32x4{0, 0, 0, 0});
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * g4 + r;
            S[row * SP + col] = acc[r] + bcol[b * 10 + 9] + XR[row * SP + col];
          }
        }
        __syncthreads();
        MDL_PROF_MARK(8);
      }
      // ---------------- [I] head1: GELU(W_h1 · LN3(S) + b) -> Q (f32 staging)
      {
        bf16x8 a[2];
        float xf[16];
        afrag_ln(S, LNP + (3 * (NB - 1) + 2) * 128, LNP + (3 * (NB - 1) + 2) * 128 + 64, lane, a, xf);
        f32x4 acc = mfma2(a, wb[NG - 1], f32x4{0, 0, 0, 0});
        const int col = 16 * wave + c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) Q[(4 * g4 + r) * SP + col] = gelu_erf(acc[r] + bcol[NG - 1]);
      }
      __syncthreads();
      MDL_PROF_MARK(9);
      // ---------------- [J] head LN + W_h2 -> logits; mask, sample, log-prob; record pending tokens
      head_phase(p, Q, S, LNP + 3 * NB * 128, ROWI, PEND, R, s, e, env0, tid, AVA, RU, RN, stage, wh2, bh2, EROW);
      __syncthreads();
      MDL_PROF_MARK(10);
    }
    // apply the block's actions to the token rows of the next passes (in-block rows kept at zero, as the reference)
    for (int idx = tid; idx < n_env * L; idx += 256) {
      const int m = idx / L, i = idx % L;
      if (i >= s && i < e) {
        const int a = PEND[m * L + i];
        if (a >= 0 && i + 1 < L) TOK[m * L + i + 1] = 1 + a;
      }
    }
    __syncthreads();
    MDL_PROF_MARK(11);
    prev_s = s;
    if (e >= L) break;
    if (e < p.n_disc) { s = e; e = min(e + p.stride, p.n_disc); }
    else { s = e; e = min(e + 1, L); }
  }
#ifdef MDL_DECODE_PROF
  if (prof_on)
    for (int k = 0; k < 16; ++k) g_decode_prof[k] = prof[k];
#endif
}

#ifdef MDL_DECODE_PROF
MDL_API int mdl_decode_prof_read(unsigned long long* out) {
  int rc = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_decode_prof), sizeof(unsigned long long) * 16, 0,
                                    hipMemcpyDeviceToHost);
  if (rc == 0) rc = (int)hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_attn_prof), sizeof(unsigned long long) * 8, 0,
                                             hipMemcpyDeviceToHost);
  return rc;
}
#endif

size_t mat_decode_stage_bytes(int epw, int L, int AD, int n_tok) {
  return ((size_t)epw * L * (64 + 2 * AD + 1) + (size_t)n_tok * 64 + (size_t)AD * 65) * 4 + 64;   // + padding
}

size_t mat_decode_lds_bytes(int NB, int epw, int rmax, int L) {
  size_t kv = (size_t)NB * 4 * epw * L * 64 * 2;
  kv = (kv + 15) & ~(size_t)15;
  size_t rest = 3 * 16 * SP * 4 + 16 * XP * 2 + (3 * NB + 1) * 128 * 4 + ((epw * rmax * 2 * L * 4 + 15) & ~15) +
                2 * ((epw * L * 4 + 15) & ~15) + 16 * 4 + (size_t)epw * 64 * 4;
  return kv + rest;
}

// Tile geometry: EPW envs per workgroup (largest power of two <= min(16, B) that fits the 160 KiB LDS of a CU
// with one row per env), then RMAX rows per env per pass (largest <= 16/EPW that still fits).
// Returns EPW | (RMAX << 8), or 0 if even one env does not fit.
MDL_API int mdl_mat_decode_geometry(int NB, int L, int B) {
  int cap = 16;
  while (cap > 1 && cap > B) cap >>= 1;
  for (int epw = cap; epw >= 1; epw >>= 1) {
    if (mat_decode_lds_bytes(NB, epw, 1, L) <= 160 * 1024) {
      int rmax = 16 / epw;
      while (rmax > 1 && mat_decode_lds_bytes(NB, epw, rmax, L) > 160 * 1024) --rmax;
      return epw | (rmax << 8);
    }
  }
  return 0;
}

MDL_API int mdl_mat_decode(const DecParams* p, int NB, hipStream_t st) {
  const int epw = p->epw;
  if (epw <= 0 || p->act_dim > 64 || p->act_dim < 1) return -1;
  if (p->cont && (!p->wa || !p->ba || !p->lnd || p->n_disc != 0)) return -5;
  if (p->rmax < 1 || p->rmax * epw > 16) return -4;
  size_t lds = mat_decode_lds_bytes(NB, epw, p->rmax, p->L);
  if (lds > 160 * 1024) return -2;
  const int grid = (p->B + epw - 1) / epw;
  // stage the per-row inputs in LDS when they fit next to the KV caches (MAT_DCML_DECODE_STAGE=0 disables)
  DecParams q = *p;
  static const bool stage_ok = [] { const char* e = getenv("MAT_DCML_DECODE_STAGE"); return !(e && e[0] == '0'); }();
  const size_t sb = mat_decode_stage_bytes(epw, p->L, p->act_dim, p->n_tok);
  q.stage = stage_ok && lds + sb <= 160 * 1024 && (p->rep != nullptr);
  if (q.stage) lds += sb;
  p = &q;
  switch (NB) {
    case 1:
      hipFuncSetAttribute((const void*)mat_decode_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(mat_decode_kernel<1>, dim3(grid), dim3(256), lds, st, *p); break;
    case 2:
      hipFuncSetAttribute((const void*)mat_decode_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(mat_decode_kernel<2>, dim3(grid), dim3(256), lds, st, *p); break;
    case 3:
      hipFuncSetAttribute((const void*)mat_decode_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(mat_decode_kernel<3>, dim3(grid), dim3(256), lds, st, *p); break;
    default: return -3;
  }
  MDL_CHECK_LAUNCH();
  return 0;
}
