// mat_decode_persistent — the whole MAT autoregressive action decode in ONE launch (gfx950 / CDNA4).
//
// Replaces the reference's rollout hot loop: L full decoder passes per env step, each re-running every row
// (mat_src/mat/algorithms/utils/transformer_act.py:76-99, 37-75 for the "batch decision" stride mode).
// Exactness: decoder row i depends only on shifted actions 0..i, so decoding one row (or
// one block of rows) at a time against a KV cache of the earlier rows reproduces the full recompute.
//
// Work decomposition (D = 64, 2 heads x 32, n_block = NB):
//   * one 256-thread workgroup = 4 waves owns one env (EPW = 1); its 16-row MFMA tile holds the agent rows of the
//     current pass (stochastic rollout: 1 row; deterministic stride mode: up to 16 rows);
//   * every 64x64 Linear is a 16x64x64 GEMM on v_mfma_f32_16x16x32_bf16: wave w owns output columns
//     [16w, 16w+16); its B fragments (all 10·NB+1 decoder weight matrices) are loaded ONCE into VGPRs and stay
//     register-resident for the whole decode (one wave per SIMD, ~170 VGPRs of weights);
//   * activations move through LDS; the post-LN residual sums are kept in f32 and LayerNorm is fused into the
//     NEXT GEMM's A-fragment load (each lane normalises the 16 values it feeds the MFMA, row statistics by two
//     xor-shuffles), so no separate LN phase/barrier exists;
//   * the self- and cross-attention K/V caches of every block live in LDS as ONE token-major swizzled bf16 array
//     (tile.h tmo: row = (block, kind, agent row), 16-byte chunks XOR-swizzled by row) and attention runs on MFMA
//     (round 2): the pass's query rows are the 16 B-operand columns, the cached keys the A rows, so one
//     v_mfma_f32_16x16x32_bf16 pair scores 32 keys for every live query and P·V is 4 more — the round-1 VALU
//     attention (one wave, a lane per key, two 32-lane reductions and an LDS round trip for P) was half of every
//     agent step (profiles/r2_decode);
//   * the action head, availability masking, inverse-CDF categorical sampling / Normal sampling, log-probs and
//     the next row's action-embedding token are fused into the last phase.
// Inputs rep (encoder output, f32), ava, and the uniform / normal draws come from HBM — staged into LDS once at
// kernel start when they fit (`stage`), so no row of the sequential agent loop waits on an HBM miss (the rep row
// of phase D and the mask / draws of the head phase were first-touch loads on the critical path); outputs are
// actions and log-probs (B, L).  Numerics: bf16 MFMA operands, f32 accumulation, f32 LayerNorm / softmax / log-softmax.
#include "tile.h"
#include "decode_params.h"
#include <cstdlib>

using namespace mdl;

constexpr int SP = 68;   // f32 staging row pitch (floats)
constexpr int XP = 72;   // bf16 A staging row pitch (elements)

// K / V caches: one token-major swizzled array, row (block b, kind (0 self K, 1 self V, 2 cross K, 3 cross V), agent j)
__device__ __forceinline__ int kv_row(int b, int kind, int j, int L) { return (b * 4 + kind) * L + j; }
__device__ __forceinline__ int kv_off(int b, int kind, int j, int col, int L) { return tmo(kv_row(b, kind, j, L), col); }
__device__ __forceinline__ f32x4 mfma2(const bf16x8 a[2], const bf16x8 w[2], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], w[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], w[1], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ uint32_t pk2f(float a, float b) {   // one v_cvt_pk_bf16_f32 (RNE)
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, b2v));
}
__device__ __forceinline__ bf16x8 pack8(const float* v) {   // 4 packed conversions
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(bf16x8, (u4v){pk2f(v[0], v[1]), pk2f(v[2], v[3]), pk2f(v[4], v[5]), pk2f(v[6], v[7])});
}

// A fragment from an f32 LDS row with fused LayerNorm.  Lane (g = lane>>4, r = lane&15) owns row r, columns
// 8g..8g+7 and 32+8g..32+8g+7.  xf receives the normalised f32 values (for the residual copy).
// One pass: Σx and Σx² reduce together (one cross-row exchange chain instead of two) and the elementwise work runs
// on packed fp32 pairs (v_pk_add / v_pk_mul / v_pk_fma_f32) — this load sits at the head of 3 phases per block.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void afrag_ln(const float* S, const float* gam, const float* bet, int lane,
                                        bf16x8 a[2], float xf[16]) {
  const int g = lane >> 4, r = lane & 15;
  const float* row = S + r * SP;
  f2 v[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = *(const f2*)(row + 8 * g + 2 * j);
    v[4 + j] = *(const f2*)(row + 32 + 8 * g + 2 * j);
  }
  f2 s2 = (v[0] + v[1]) + (v[2] + v[3]) + ((v[4] + v[5]) + (v[6] + v[7]));
  f2 q2 = v[0] * v[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) q2 = v[j] * v[j] + q2;
  f2 sq = {s2.x + s2.y, q2.x + q2.y};   // (Σx, Σx²) of the lane's 16 values
  float a0, b0, a1, b1;
  swap16(sq.x, a0, b0);
  swap16(sq.y, a1, b1);
  sq = f2{a0 + b0, a1 + b1};
  swap32(sq.x, a0, b0);
  swap32(sq.y, a1, b1);
  const float mean = (a0 + b0) * (1.f / 64.f);
  const float var = fmaxf((a1 + b1) * (1.f / 64.f) - mean * mean, 0.f);
  const float rstd = rsqrtf(var + 1e-5f);
  const f2 mr = {mean, mean}, rr = {rstd, rstd};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c0 = 8 * g + 2 * j, c1 = 32 + 8 * g + 2 * j;
    const f2 y0 = (v[j] - mr) * rr * *(const f2*)(gam + c0) + *(const f2*)(bet + c0);
    const f2 y1 = (v[4 + j] - mr) * rr * *(const f2*)(gam + c1) + *(const f2*)(bet + c1);
    xf[2 * j] = y0.x; xf[2 * j + 1] = y0.y;
    xf[8 + 2 * j] = y1.x; xf[8 + 2 * j + 1] = y1.y;
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


__device__ __forceinline__ float xrow_max(float x) {   // max over the 4 lane rows g of a column c
  float a, b;
  swap16(x, a, b);
  x = fmaxf(a, b);
  swap32(x, a, b);
  return fmaxf(a, b);
}

// Causal attention of the pass's query rows t (agent row plo + t for t < R, else dead) over the cached rows 0..i, head h
// = wave (waves 0, 1).  Scores Sᵀ = K·Qᵀ in 32-key chunks: the A rows are keys in the permuted order pi(t, m) =
// 8(m>>2) + 4t + (m&3), so lane (g, c) of the two MFMA outputs holds S[query c][keys kb + 8g + j] (j < 8) — already
// the B operand of Oᵀ = Vᵀ·Pᵀ, whose A operand comes from ds_read_b64_tr_b16 of the token-major V cache.
// Single-pass online softmax in log2 units; P enters as a hi/lo bf16 pair (fp32-like P·V).  O (bf16) -> XA rows.
// Masked keys (j > i, or rows of other caches beyond the chunk) get P = 0; every cache row is finite (zeroed at
// kernel start, plus 32 zero rows after the last cache) so 0 · V stays 0.
__device__ __forceinline__ void attention_mfma(const bf16_t* KV, int rowK, int rowV, const bf16_t* QT, int qrow0,
                                               bf16_t* XA, int plo, int R, int imax, int wave, int lane) {
  if (wave >= 2) return;
  const int h = wave, g = lane >> 4, c = lane & 15;
  constexpr float SL2 = 0.17677669529663687f * 1.4426950408889634f;   // 1/sqrt(32) * log2(e)
  const int iq = c < R ? plo + c : -1;
  const bf16x8 qB = lda_tm(QT, qrow0 + c, 4 * h + g);
  float m = -INFINITY, l = 0.f;
  f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb <= imax; kb += 32) {
    float sc[8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16x8 a = lda_tm(KV, rowK + kb + 8 * (c >> 2) + 4 * t + (c & 3), 4 * h + g);
      const f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qB, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) sc[4 * t + i] = r[i];
    }
    float cm = -INFINITY;
    const int d0 = iq - kb - 8 * g;   // key j visible iff j <= d0
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = j <= d0 ? sc[j] : -INFINITY;   // raw scores; the scale goes into the exp2 argument (one FMA)
      cm = fmaxf(cm, sc[j]);
    }
    const float nm = fmaxf(m, xrow_max(cm) * SL2);
    const float mr = nm == -INFINITY ? 0.f : nm;
    const float alpha = fast_exp2(m - mr);   // raw v_exp_f32 (exp2f's denormal-safe sequence is 7 VALU)
    float ps = 0.f;
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = fast_exp2(fmaf(sc[j], SL2, -mr));
      ps += sc[j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hi[i] = pk2f(sc[2 * i], sc[2 * i + 1]);
      lo[i] = pk2f(sc[2 * i] - __uint_as_float(hi[i] << 16), sc[2 * i + 1] - __uint_as_float(hi[i] & 0xFFFF0000u));
    }
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    const bf16x8 ph = __builtin_bit_cast(bf16x8, (u4v){hi[0], hi[1], hi[2], hi[3]});
    const bf16x8 pl = __builtin_bit_cast(bf16x8, (u4v){lo[0], lo[1], lo[2], lo[3]});
    l = l * alpha + ps;
    o0 *= alpha;
    o1 *= alpha;
    const bf16x8 va = ld_frag_T(KV, rowV + kb, 32 * h, lane), vb = ld_frag_T(KV, rowV + kb, 32 * h + 16, lane);
    o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, ph, o0, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pl, o0, 0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb, ph, o1, 0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb, pl, o1, 0, 0, 0);
    m = nm;
  }
  l = cross_row_sum(l);
  const float il = l > 0.f ? 1.f / l : 0.f;
  bf16_t* xa = XA + c * XP + 32 * h + 4 * g;
  *(uint2*)xa = make_uint2(pk2f(o0[0] * il, o0[1] * il), pk2f(o0[2] * il, o0[3] * il));
  *(uint2*)(xa + 16) = make_uint2(pk2f(o1[0] * il, o1[1] * il), pk2f(o1[2] * il, o1[3] * il));
}

// inclusive prefix sum over the 64 lanes: DPP row_shr 1, 2, 4, 8 within each 16-lane row (zero fill), then the
// totals of the lower rows (3 readlanes) — VALU only, no ds_bpermute round trips
__device__ __forceinline__ float wave_incl_scan(float x, int lane) {
  x += dppf<0x111>(x);
  x += dppf<0x112>(x);
  x += dppf<0x114>(x);
  x += dppf<0x118>(x);
  const float t0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 15));
  const float t1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 31));
  const float t2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 47));
  const int r = lane >> 4;
  return x + ((r >= 1 ? t0 : 0.f) + (r >= 2 ? t1 : 0.f) + (r >= 3 ? t2 : 0.f));
}

// categorical sample over <= 4 register logits (every lane of the row computes it alike): availability mask,
// inverse-CDF draw (argmax when deterministic); returns the action, its masked logit and the log-sum-exp
constexpr int SMALL_AD = 4;
#define SMALL_AD_ 4
__device__ __forceinline__ int sample_small(const float* lgr, int AD, const float* av, float uu, bool det, float& la,
                                            float& lse) {
  float l[SMALL_AD];
#pragma unroll
  for (int a = 0; a < SMALL_AD; ++a) l[a] = a < AD ? ((av && av[a] == 0.f) ? -1e10f : lgr[a]) : -INFINITY;
  float mx = l[0];
  int amax = 0;
#pragma unroll
  for (int a = 1; a < SMALL_AD; ++a) if (l[a] > mx) { mx = l[a]; amax = a; }
  float e[SMALL_AD], se = 0.f;
#pragma unroll
  for (int a = 0; a < SMALL_AD; ++a) { e[a] = a < AD ? __expf(l[a] - mx) : 0.f; se += e[a]; }
  lse = mx + __logf(se);
  int act = amax;
  if (!det) {
    const float inv = 1.f / se;
    float cdf = 0.f;
    int cnt = 0;
#pragma unroll
    for (int a = 0; a < SMALL_AD; ++a) {
      cdf += e[a] * inv;
      cnt += (a < AD) & (cdf < uu);
    }
    act = min(cnt, AD - 1);
  }
  la = l[0];
#pragma unroll
  for (int a = 1; a < SMALL_AD; ++a) la = act == a ? l[a] : la;
  return act;
}

// next row's block-0 operands (tile row 0 of the next pass) from the token table: lane q of the row writes
// columns 4q .. 4q+3 of the query, K, V (bf16) and the residual x (f32)
__device__ __forceinline__ void write_next_row0(const float* QKV0, const float* emb, int tok, int row, int L, int q,
                                                bf16_t* QT, bf16_t* KV, float* XR) {
  const float4* tq = (const float4*)(QKV0 + (size_t)tok * 192) + q;
  const float4 vq = tq[0], vk = tq[16], vv = tq[32];
  const float4 ve = ((const float4*)(emb + (size_t)tok * 64))[q];
  *(uint2*)(QT + tmo(0, 4 * q)) = make_uint2(pk2f(vq.x, vq.y), pk2f(vq.z, vq.w));
  *(uint2*)(KV + kv_off(0, 0, row, 4 * q, L)) = make_uint2(pk2f(vk.x, vk.y), pk2f(vk.z, vk.w));
  *(uint2*)(KV + kv_off(0, 1, row, 4 * q, L)) = make_uint2(pk2f(vv.x, vv.y), pk2f(vv.z, vv.w));
  *(float4*)(XR + 4 * q) = ve;
}

// Action head: LN(head1 output) · W_h2 + b -> logits; availability mask, sampling, log-prob (16 lanes per row).
__device__ __forceinline__ void head_phase(const DecParams& p, const float* H1, float* LG, const float* lnh,
                                           int plo, int* PEND, int R, int s, int e, int env0, int tid,
                                           const float* AVA, const float* RU, const float* RN, bool stage,
                                           const float* wh2, const float* bh2, float* EROW,
                                           bool fast0, const float* QKV0, const float* emb, bf16_t* QT, bf16_t* KV,
                                           float* XR) {
  const int t = tid >> 4, q = tid & 15;
  const int i = t < R ? plo + t : -1;   // one env per workgroup: tile row t = agent row plo + t
  const int AD = p.act_dim, L = p.L;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = H1[t * SP + 4 * q + k];
  // one pass: Σx and Σx² reduce side by side (two independent DPP chains instead of two dependent ones)
  const float sm = group_sum<16>((v[0] + v[1]) + (v[2] + v[3]));
  const float sq = group_sum<16>((v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]));
  const float mean = sm * (1.f / 64.f);
  const float rstd = rsqrtf(fmaxf(sq * (1.f / 64.f) - mean * mean, 0.f) + 1e-5f);
  float hn[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) hn[k] = (v[k] - mean) * rstd * lnh[4 * q + k] + lnh[64 + 4 * q + k];
  // logits: up to 4 actions (DCML's 2) unrolled with every row lane holding all of them in registers (the
  // discrete sampling below reads them there, no LDS round trip); larger heads loop and go through LG
  constexpr int SMALL = SMALL_AD;
  const bool small = AD <= SMALL;
  float lgr[SMALL];
  if (small) {
#pragma unroll
    for (int a = 0; a < SMALL; ++a) {
      float part = 0.f;
      if (a < AD) {
        const float4 w = *(const float4*)(wh2 + a * 64 + 4 * q);
        part = w.x * hn[0] + w.y * hn[1] + w.z * hn[2] + w.w * hn[3];
      }
      lgr[a] = group_sum<16>(part) + (a < AD ? bh2[a] : 0.f);
      if (q == 0 && a < AD) LG[t * SP + a] = lgr[a];
    }
  } else {
    for (int a = 0; a < AD; ++a) {
      const float* w = wh2 + a * 64 + 4 * q;
      float part = w[0] * hn[0] + w[1] * hn[1] + w[2] * hn[2] + w[3] * hn[3];
      part = group_sum<16>(part);
      if (q == 0) LG[t * SP + a] = part + bh2[a];
    }
  }
  if (p.cont) {   // all act_dim dims are Gaussian; the 16 lanes of the row also build the next row's input
    if (i < 0 || i < s || i >= e) return;
    const int m = t / R;
    const size_t oi = (size_t)(env0 + m) * L + i, li = (size_t)m * L + i;
    const float* lg = LG + t * SP;
    float ev[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ev[k] = p.ba[4 * q + k];
    int cat = -1;   // Available_Continuous: the categorical choice over logits 0, 1 (every lane of the row alike)
    if (p.avail_cont) {
      const float* av = p.ava ? (stage ? AVA + li * AD : p.ava + oi * AD) : nullptr;
      const float l0 = (av && av[0] == 0.f) ? -1e10f : lg[0], l1 = (av && av[1] == 0.f) ? -1e10f : lg[1];
      const float mx = fmaxf(l0, l1), lse = mx + __logf(__expf(l0 - mx) + __expf(l1 - mx));
      if (p.deterministic) cat = l1 > l0 ? 1 : 0;
      else {
        const float uu = stage ? RU[li] : p.gen ? draw_u(p, env0 + m, i) : p.rnd_u[oi];
        cat = __expf(l0 - lse) < uu ? 1 : 0;
      }
      if (q == 0) p.out_lp[oi * (AD - 1)] = (cat ? l1 : l0) - lse;
    }
    for (int a = 0; a < AD; ++a) {
      float x;
      if (cat >= 0 && a < 2) {
        x = a == cat ? 1.f : 0.f;
        if (q == 0) p.out_a[oi * AD + a] = x;
      } else {
        const float mean_a = lg[a], sd = p.stdv[a];
        x = p.deterministic ? mean_a : mean_a + sd * (stage ? RN[li * AD + a] : p.gen ? draw_n(p, env0 + m, i, a) : p.rnd_n[oi * AD + a]);
        if (q == 0) {
          const float z = (x - mean_a) / sd;
          p.out_a[oi * AD + a] = x;
          p.out_lp[cat >= 0 ? oi * (AD - 1) + a - 1 : oi * AD + a] = -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
        }
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
  if (i < 0 || i < s || i >= e) return;
  if (q != 0 && !(fast0 && i < p.n_disc && i + 1 < L)) return;   // fast0: the row's 16 lanes sample alike
  const int m = t / R, env = env0 + m;
  const float* lg = LG + t * SP;
  const size_t oi = (size_t)env * L + i;
  const size_t li = (size_t)m * L + i;                  // row in the staged (workgroup-local) inputs
  if (i < p.n_disc) {
    const float* av = p.ava ? (stage ? AVA + li * AD : p.ava + oi * AD) : nullptr;
    const float uu = p.deterministic ? 0.f : stage ? RU[li] : p.gen ? draw_u(p, env, i) : p.rnd_u[oi];
    int act;
    float la, lse;
    if (small) {   // registers, fully unrolled
      act = sample_small(lgr, AD, av, uu, p.deterministic != 0, la, lse);
    } else {
      float mx = -INFINITY;
      int amax = 0;
      for (int a = 0; a < AD; ++a) {
        const float l = (av && av[a] == 0.f) ? -1e10f : lg[a];
        if (l > mx) { mx = l; amax = a; }
      }
      float se = 0.f;
      for (int a = 0; a < AD; ++a) se += __expf(((av && av[a] == 0.f) ? -1e10f : lg[a]) - mx);
      lse = mx + __logf(se);
      act = amax;
      if (!p.deterministic) {
        float cdf = 0.f;
        int cnt = 0;
        for (int a = 0; a < AD; ++a) {
          cdf += __expf(((av && av[a] == 0.f) ? -1e10f : lg[a]) - lse);
          cnt += cdf < uu;
        }
        act = min(cnt, AD - 1);
      }
      la = (av && av[act] == 0.f) ? -1e10f : lg[act];
    }
    if (q == 0) {
      p.out_a[oi] = (float)act;
      p.out_lp[oi] = la - lse;
      PEND[m * L + i] = act;
    }
    if (fast0 && i + 1 < L) write_next_row0(QKV0, emb, 1 + act, i + 1, L, q, QT, KV, XR);
  } else {
    const int a = AD - 1;
    const float mean_a = lg[a], sd = p.stdv[a];
    const float x = p.deterministic ? mean_a : mean_a + sd * (stage ? RN[li * AD + a] : p.gen ? draw_n(p, env, i, a) : p.rnd_n[oi * AD + a]);
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

// an LDS pointer held in a VGPR (opaque to uniformity analysis), address space kept for ds_* instructions
template <typename T>
__device__ __forceinline__ T* lds_v(T* p) {
  auto q = (__attribute__((address_space(3))) T*)p;
  asm volatile("" : "+v"(q));
  return (T*)q;
}

// STG: the inputs are staged in LDS (p.stage) — a compile-time switch, so every table / row pointer of the agent
// loop is statically an LDS or a global pointer (a runtime select made them generic: flat loads waiting on both
// counters, vmcnt(0) lgkmcnt(0), in the head / next-row / residual reads of every agent step)
template <int NB, bool STG>
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
  const size_t kv_elems = ((size_t)NB * 4 * L + 32) * 64;    // + 32 zero rows: chunk reads past the last cache
  bf16_t* KV = (bf16_t*)smem;
  char* ptr = smem + ((kv_elems * 2 + 15) & ~(size_t)15);
  float* S = (float*)ptr;   ptr += 16 * SP * 4;
  float* Q = (float*)ptr;   ptr += 16 * SP * 4;   // head1 output (f32)
  float* XR = (float*)ptr;  ptr += 16 * SP * 4;
  bf16_t* XA = (bf16_t*)ptr; ptr += 16 * XP * 2;
  bf16_t* QT = (bf16_t*)ptr; ptr += 16 * 64 * 2;   // attention queries, token-major swizzled (tile.h tmo)
  const bool q2pre = p.q2pre != 0;
  bf16_t* Q2T = (bf16_t*)ptr;                        // [NB][L + 16] precomputed cross-attention queries (q2pre)
  if (q2pre) ptr += (size_t)NB * (L + 16) * 64 * 2;
  float* LNP = (float*)ptr; ptr += NLN * 128 * 4;
  int* TOK = (int*)ptr;     ptr += ((EPW * L * 4 + 15) & ~15);
  int* PEND = (int*)ptr;    ptr += ((EPW * L * 4 + 15) & ~15);
  float* EROW = (float*)ptr; ptr += EPW * 64 * 4;            // cont: next row's input embedding per env
  float* REP = (float*)ptr;                                  // staged inputs (p.stage): [EPW][L][64]
  auto pad4 = [](size_t n) { return (n + 3) & ~(size_t)3; };  // keep every region 16-byte aligned
  float* AVA = REP + pad4((size_t)EPW * L * 64);             // [EPW][L][AD]
  float* RU = AVA + pad4((size_t)EPW * L * AD);              // [EPW][L]
  float* RN = RU + pad4((size_t)EPW * L);                    // [EPW][L][AD]
  float* EMB = RN + pad4((size_t)EPW * L * AD);              // [n_tok][64] action-embedding rows (float4 reads)
  float* WH2 = EMB + (size_t)p.n_tok * 64;                   // [AD][64], then bh2 [AD]
  float* QKV0S = WH2 + pad4((size_t)AD * 65);                // [n_tok][3][64] block-0 token table (p.qkv0)
  float* HW4 = QKV0S + (size_t)p.n_tok * 192;                // wide head: [16][AD] float4 of the folded W_h2
  float* HGC = HW4 + (size_t)AD * 64;                        //   then G[AD], C[AD]
#ifndef MDL_DECODE_SGPR_CARVE
  // the carve's region bases as VGPRs (LDS addresses are VGPR operands anyway): as ~20 uniform SGPR values live
  // across the agent loop they were the bulk of the kernel's SGPR spills (v_writelane / v_readlane + hazard nops)
  KV = lds_v(KV); S = lds_v(S); Q = lds_v(Q); XR = lds_v(XR); XA = lds_v(XA); QT = lds_v(QT); Q2T = lds_v(Q2T);
  LNP = lds_v(LNP); TOK = lds_v(TOK); PEND = lds_v(PEND); EROW = lds_v(EROW); REP = lds_v(REP); AVA = lds_v(AVA);
  RU = lds_v(RU); RN = lds_v(RN); EMB = lds_v(EMB); WH2 = lds_v(WH2); QKV0S = lds_v(QKV0S); HW4 = lds_v(HW4);
  HGC = lds_v(HGC);
#endif
  constexpr bool stage = STG;
  // wide fused head (one-row discrete passes, 4 < AD <= 64: SMAC's 36 actions): lane a of every wave computes logit a
  // from the folded LayerNorm (p.hfold) and the wave samples with ballots / a prefix scan — replaces the generic head
  // phase's per-action loop of 16-lane reductions and its three serial passes over the logits
  const bool whead = stage && p.hfold != nullptr && !p.cont && AD > SMALL_AD;
  const bool fast0 = p.qkv0 != nullptr && !p.cont && p.stride == 1;   // one row per pass, token inputs

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
  // folded head (one-row discrete passes, <= 4 actions): this lane's column 16 wave + c16 of W_h2 diag(gamma_h)
  float hw[SMALL_AD_], hG[SMALL_AD_], hC[SMALL_AD_];
#pragma unroll
  for (int a = 0; a < SMALL_AD_; ++a) {
    const bool in = p.hfold && a < AD;
    hw[a] = in ? p.hfold[a * 64 + 16 * wave + c16] : 0.f;
    hG[a] = in ? p.hfold[AD * 64 + a] : 0.f;
    hC[a] = in ? p.hfold[AD * 65 + a] : 0.f;
  }
  for (int i = tid; i < NLN * 128; i += 256) LNP[i] = p.lnp[i];
  for (int i = tid; i < EPW * L; i += 256) { TOK[i] = (i % L == 0) ? p.tok_start : p.tok_zero; PEND[i] = -1; }
  for (int i = tid; i < 16 * XP; i += 256) XA[i] = 0;   // dead tile rows keep finite A-operand rows
  for (size_t i = (size_t)tid * 8; i < kv_elems; i += 256 * 8) *(uint4*)(KV + i) = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < 16 * 64; i += 256) QT[i] = 0;
  if (q2pre)
    for (size_t i = (size_t)tid * 8; i < (size_t)NB * (L + 16) * 64; i += 256 * 8) *(uint4*)(Q2T + i) = make_uint4(0, 0, 0, 0);
  if (stage) {   // the workgroup's envs are contiguous in every input
    const int nrow = n_env * L;
    const float4* src = (const float4*)(p.rep + (size_t)env0 * L * 64);
    float4* dst = (float4*)REP;
    for (int i = tid; i < nrow * 16; i += 256) dst[i] = src[i];
    if (p.ava) for (int i = tid; i < nrow * AD; i += 256) AVA[i] = p.ava[(size_t)env0 * L * AD + i];
    if (p.gen && !p.deterministic) {
      for (int i = tid; i < nrow; i += 256) RU[i] = draw_u(p, env0 + i / L, i % L);
      for (int i = tid; i < nrow * AD; i += 256) RN[i] = draw_n(p, env0 + i / (L * AD), (i / AD) % L, i % AD);
    } else {
      if (p.rnd_u) for (int i = tid; i < nrow; i += 256) RU[i] = p.rnd_u[(size_t)env0 * L + i];
      if (p.rnd_n) for (int i = tid; i < nrow * AD; i += 256) RN[i] = p.rnd_n[(size_t)env0 * L * AD + i];
    }
    for (int i = tid; i < p.n_tok * 64; i += 256) EMB[i] = p.emb[i];
    for (int i = tid; i < AD * 65; i += 256) WH2[i] = i < AD * 64 ? p.wh2[i] : p.bh2[i - AD * 64];
    if (p.qkv0) for (int i = tid; i < p.n_tok * 192; i += 256) QKV0S[i] = p.qkv0[i];
    if (whead) {   // transposed: float4 (kq, a) = W'[a][4kq .. 4kq+3], so lane a's reads are consecutive (no conflicts)
      for (int i = tid; i < AD * 64; i += 256) {
        const int a = i >> 6, k = i & 63;
        HW4[((k >> 2) * AD + a) * 4 + (k & 3)] = p.hfold[i];
      }
      for (int i = tid; i < 2 * AD; i += 256) HGC[i] = p.hfold[AD * 64 + i];
    }
  }
  const float* emb = stage ? EMB : p.emb;
  const float* wh2 = stage ? WH2 : p.wh2;
  const float* bh2 = stage ? WH2 + AD * 64 : p.bh2;
  const float* qkv0 = stage ? QKV0S : p.qkv0;
  __syncthreads();
  if (q2pre) {   // q2 of every agent row, every block: one MFMA pass over 16-row tiles of rep before the agent loop
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      for (int t0 = 0; t0 < L; t0 += 16) {
        bf16x8 a[2];
        float xf[16];
        const int ri = t0 + c16;
        const float* rrow = ri >= L ? nullptr : stage ? REP + (size_t)ri * 64 : p.rep + ((size_t)env0 * L + ri) * 64;
        afrag_rowf(rrow, lane, a, xf);
        const f32x4 q2 = mfma2(a, wb[b * 10 + 4], f32x4{0, 0, 0, 0});
        const int col = 16 * wave + c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = t0 + 4 * g4 + r;
          if (row < L) Q2T[(size_t)b * (L + 16) * 64 + tmo(row, col)] = f2bf(q2[r] + bcol[b * 10 + 4]);
        }
      }
    }
  }
  if (fast0 && tid < 64) {   // row 0 (the start token): block-0 query / K / V / residual x from the table
    const float* tq = qkv0 + (size_t)p.tok_start * 192;
    QT[tmo(0, tid)] = f2bf(tq[tid]);
    KV[kv_off(0, 0, 0, tid, L)] = f2bf(tq[64 + tid]);
    KV[kv_off(0, 1, 0, tid, L)] = f2bf(tq[128 + tid]);
    XR[tid] = emb[(size_t)p.tok_start * 64 + tid];
  }
  __syncthreads();
  // (the head phase's float4 table reads need 16-byte rows: QKV0S / EMB are float4-aligned pieces of the carve)

  // ---------------------------------------------------------------- block schedule (transformer_act.py:37-75)
  int prev_s = -1, s = 0, e = 1;
  while (true) {
    int lo = prev_s >= 0 ? prev_s + 1 : 0;
    if (lo > s) lo = s;
    for (int plo = lo; plo < e; plo += RMAX) {
      const int R = min(RMAX, e - plo);
      // tile row t = agent row plo + t (t < R; one env per workgroup) — known to every lane, so a pass starts
      // without publishing a row table (the previous pass ended on a barrier)
      MDL_PROF_MARK(0);
      // per-lane tile rows for the C layout (rows 4*g4 + r) and the A layout (row c16)
      int crow_i[4], crow_m[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { crow_i[r] = 4 * g4 + r < R ? plo + 4 * g4 + r : -1; crow_m[r] = 0; }
      const int arow_i = c16 < R ? plo + c16 : -1, arow_m = 0;
      const int imax = plo + R - 1;                         // last live agent row of the pass

#pragma unroll
      for (int b = 0; b < NB; ++b) {
        bf16x8 a[2];
        float xf[16];
        // ---------------- [A] x = emb(token) (b == 0) or LN3(S) ; q1, k1, v1   (fast0: block 0's came from the table)
        if (!(fast0 && b == 0)) {
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
            QT[tmo(row, col)] = f2bf(q1[r] + bcol[b * 10 + 0]);
            if (crow_i[r] >= 0) {
              KV[kv_off(b, 0, crow_i[r], col, L)] = f2bf(k1[r] + bcol[b * 10 + 1]);
              KV[kv_off(b, 1, crow_i[r], col, L)] = f2bf(v1[r] + bcol[b * 10 + 2]);
            }
          }
        }
        __syncthreads();
        }
        MDL_PROF_MARK(1);
        // ---------------- [B] causal self-attention over cached rows 0..i
        attention_mfma(KV, kv_row(b, 0, 0, L), kv_row(b, 1, 0, L), QT, 0, XA, plo, R, imax, wave, lane);
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
          f32x4 k2 = mfma2(a, wb[b * 10 + 5], f32x4{0, 0, 0, 0});
          f32x4 v2 = mfma2(a, wb[b * 10 + 6], f32x4{0, 0, 0, 0});
          if (!q2pre) {
            bf16x8 ar[2];
            float rf[16];
            const float* rrow = arow_i < 0 ? nullptr
                                : stage ? REP + ((size_t)arow_m * L + arow_i) * 64
                                        : p.rep + ((size_t)(env0 + arow_m) * L + arow_i) * 64;
            afrag_rowf(rrow, lane, ar, rf);
            const f32x4 q2 = mfma2(ar, wb[b * 10 + 4], f32x4{0, 0, 0, 0});
#pragma unroll
            for (int r = 0; r < 4; ++r) QT[tmo(4 * g4 + r, 16 * wave + c16)] = f2bf(q2[r] + bcol[b * 10 + 4]);
          }
          const int col = 16 * wave + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (crow_i[r] >= 0) {
              KV[kv_off(b, 2, crow_i[r], col, L)] = f2bf(k2[r] + bcol[b * 10 + 5]);
              KV[kv_off(b, 3, crow_i[r], col, L)] = f2bf(v2[r] + bcol[b * 10 + 6]);
            }
          }
        }
        __syncthreads();
        MDL_PROF_MARK(4);
        // ---------------- [E] causal cross-attention (q = rep rows, k/v = x1 rows)
        attention_mfma(KV, kv_row(b, 2, 0, L), kv_row(b, 3, 0, L), q2pre ? Q2T + (size_t)b * (L + 16) * 64 : QT,
                       q2pre ? plo : 0, XA, plo, R, imax, wave, lane);
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
      // ---------------- [I+J fused] one discrete row per pass, <= 4 actions, head LayerNorm folded into the logit
      // weights (p.hfold).  J1, every wave: head1 of its 16 columns for the row, GELU, and the partial sums
      // Σx, Σx², Σ_c (W_h2 γ)[a, c] x_c of those columns -> LDS; J2, every wave alike: combine the 4 partials,
      // logits = rstd (P_a - mean G_a) + C_a, sample, and write its slice of the next row's block-0 operands.
      // (Round 2 ran the whole head in wave 0: 8 MFMAs, 4 GELUs and serial reductions per lane; 4.3k cycles.)
      if (fast0 && AD <= SMALL_AD && plo < p.n_disc && p.hfold) {
        float* PART = Q;   // [4 waves][8] partial sums (the head1 staging buffer is unused on this path)
        {
          bf16x8 a[2];
          float xf[16];
          afrag_ln(S, LNP + (3 * (NB - 1) + 2) * 128, LNP + (3 * (NB - 1) + 2) * 128 + 64, lane, a, xf);
          const f32x4 acc = mfma2(a, wb[NG - 1], f32x4{0, 0, 0, 0});
          if (g4 == 0) {   // lanes 0..15: tile row 0 (element r = 0), column 16 wave + c16
            const float x = gelu_erf(acc[0] + bcol[NG - 1]);
            const float s1 = group_sum<16>(x), s2 = group_sum<16>(x * x);
            float pa[SMALL_AD];
#pragma unroll
            for (int aa = 0; aa < SMALL_AD; ++aa) pa[aa] = aa < AD ? group_sum<16>(x * hw[aa]) : 0.f;
            if (c16 == 0) {
              PART[wave * 8 + 0] = s1;
              PART[wave * 8 + 1] = s2;
#pragma unroll
              for (int aa = 0; aa < SMALL_AD; ++aa) PART[wave * 8 + 2 + aa] = pa[aa];
            }
          }
        }
        __syncthreads();
        MDL_PROF_MARK(9);
        if (g4 == 0) {
          float s1 = 0.f, s2 = 0.f, pa[SMALL_AD];
#pragma unroll
          for (int aa = 0; aa < SMALL_AD; ++aa) pa[aa] = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) {   // fixed order: every wave computes bit-identical logits
            s1 += PART[w * 8 + 0];
            s2 += PART[w * 8 + 1];
#pragma unroll
            for (int aa = 0; aa < SMALL_AD; ++aa) pa[aa] += PART[w * 8 + 2 + aa];
          }
          const float mean = s1 * (1.f / 64.f);
          const float rstd = rsqrtf(fmaxf(s2 * (1.f / 64.f) - mean * mean, 0.f) + 1e-5f);
          float lgr[SMALL_AD];
#pragma unroll
          for (int aa = 0; aa < SMALL_AD; ++aa) lgr[aa] = rstd * (pa[aa] - mean * hG[aa]) + hC[aa];
          const int i = plo;
          const size_t oi = (size_t)env0 * L + i, li = (size_t)i;
          const float* av = p.ava ? (stage ? AVA + li * AD : p.ava + oi * AD) : nullptr;
          const float uu = p.deterministic ? 0.f : stage ? RU[li] : p.gen ? draw_u(p, env0, i) : p.rnd_u[oi];
          float la, lse;
          const int act = sample_small(lgr, AD, av, uu, p.deterministic != 0, la, lse);
          if (wave == 0 && c16 == 0) {
            p.out_a[oi] = (float)act;
            p.out_lp[oi] = la - lse;
            PEND[i] = act;
          }
          if (i + 1 < L && c16 < 4) write_next_row0(qkv0, emb, 1 + act, i + 1, L, 4 * wave + c16, QT, KV, XR);
        }
        __syncthreads();
        MDL_PROF_MARK(10);
      } else if (fast0 && whead && plo < p.n_disc) {
        float* HX = Q;   // the row's 64 head1 outputs (the head1 staging buffer)
        {   // J1, every wave: head1 of its 16 columns for the row, GELU -> HX
          bf16x8 a[2];
          float xf[16];
          afrag_ln(S, LNP + (3 * (NB - 1) + 2) * 128, LNP + (3 * (NB - 1) + 2) * 128 + 64, lane, a, xf);
          const f32x4 acc = mfma2(a, wb[NG - 1], f32x4{0, 0, 0, 0});
          if (g4 == 0) HX[16 * wave + c16] = gelu_erf(acc[0] + bcol[NG - 1]);
        }
        __syncthreads();
        MDL_PROF_MARK(9);
        {   // J2, every wave alike (bit-identical): lane a = action a
          const bool aok = lane < AD;
          const int ac = aok ? lane : 0;
          const float4* hx4 = (const float4*)HX;
          const float4* w4 = (const float4*)HW4;
          float s1 = 0.f, s2 = 0.f, pa = 0.f;
#pragma unroll
          for (int kq = 0; kq < 16; ++kq) {
            const float4 x = hx4[kq], w = w4[kq * AD + ac];
            s1 += (x.x + x.y) + (x.z + x.w);
            s2 += (x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w);
            pa += (w.x * x.x + w.y * x.y) + (w.z * x.z + w.w * x.w);
          }
          const float mean = s1 * (1.f / 64.f);
          const float rstd = rsqrtf(fmaxf(s2 * (1.f / 64.f) - mean * mean, 0.f) + 1e-5f);
          const int i = plo;
          const size_t oi = (size_t)env0 * L + i, li = (size_t)i;
          const float lg = rstd * (pa - mean * HGC[ac]) + HGC[AD + ac];
          const float l = aok ? ((p.ava && AVA[li * AD + ac] == 0.f) ? -1e10f : lg) : -INFINITY;
          const float mx = wave_max(l);
          int act = __ffsll((unsigned long long)__ballot(l == mx)) - 1;   // first maximum (argmax)
          const float e = aok ? __expf(l - mx) : 0.f;
          const float lse = mx + __logf(wave_sum(e));
          if (!p.deterministic) {   // inverse CDF: the number of actions whose running probability is below u
            const float cdf = wave_incl_scan(aok ? __expf(l - lse) : 0.f, lane);
            const float uu = RU[li];
            act = min((int)__popcll((unsigned long long)__ballot(aok && cdf < uu)), AD - 1);
          }
          act = __builtin_amdgcn_readfirstlane(act);
          const float la = __shfl(l, act, 64);
          if (wave == 0 && lane == 0) {
            p.out_a[oi] = (float)act;
            p.out_lp[oi] = la - lse;
            PEND[i] = act;
          }
          if (g4 == 0 && c16 < 4 && i + 1 < L) write_next_row0(qkv0, emb, 1 + act, i + 1, L, 4 * wave + c16, QT, KV, XR);
        }
        __syncthreads();
        MDL_PROF_MARK(10);
      } else {
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
      head_phase(p, Q, S, LNP + 3 * NB * 128, plo, PEND, R, s, e, env0, tid, AVA, RU, RN, stage, wh2, bh2, EROW,
                 fast0, qkv0, emb, QT, KV, XR);
      __syncthreads();
      MDL_PROF_MARK(10);
      }
    }
    // apply the block's actions to the token rows of the next passes (in-block rows kept at zero, as the reference);
    // fast0 passes read no token rows (the head phase already wrote the next row's block-0 operands)
    if (!fast0) {
      for (int idx = tid; idx < n_env * L; idx += 256) {
        const int m = idx / L, i = idx % L;
        if (i >= s && i < e) {
          const int a = PEND[m * L + i];
          if (a >= 0 && i + 1 < L) TOK[m * L + i + 1] = 1 + a;
        }
      }
      __syncthreads();
    }
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
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_decode_prof), sizeof(unsigned long long) * 16, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

size_t mat_decode_stage_bytes(int epw, int L, int AD, int n_tok) {
  const size_t wide = AD > SMALL_AD ? (size_t)AD * 66 : 0;   // wide fused head: folded W_h2 (transposed), G, C
  return ((size_t)epw * L * (64 + 2 * AD + 1) + (size_t)n_tok * (64 + 192) + (size_t)AD * 65 + wide) * 4 + 96;   // + padding
}

size_t mat_decode_lds_bytes(int NB, int epw, int rmax, int L) {
  (void)rmax;
  size_t kv = ((size_t)NB * 4 * L + 32) * 64 * 2;
  kv = (kv + 15) & ~(size_t)15;
  size_t rest = 3 * 16 * SP * 4 + 16 * XP * 2 + 16 * 64 * 2 + (3 * NB + 1) * 128 * 4 + 2 * ((epw * L * 4 + 15) & ~15) +
                16 * 4 + (size_t)epw * 64 * 4;
  return kv + rest;
}

// Tile geometry: one env per workgroup (the MFMA attention shares the K / V A-operand over the tile's query rows,
// so they must be one env's rows; envs per workgroup only ever shortened the round-1 VALU attention, and at the
// rollout shape one env per CU was already the fastest, 642 vs 690 us), RMAX = 16 rows per pass (stride mode).
// Returns EPW | (RMAX << 8), or 0 if the caches do not fit.
MDL_API int mdl_mat_decode_geometry(int NB, int L, int B) {
  (void)B;
  return mat_decode_lds_bytes(NB, 1, 16, L) <= 160 * 1024 ? 1 | (16 << 8) : 0;
}

MDL_API int mdl_mat_decode(const DecParams* p, int NB, hipStream_t st) {
  const int epw = p->epw;
  if (epw != 1 || p->act_dim > 64 || p->act_dim < 1) return -1;
  if (p->cont && (!p->wa || !p->ba || !p->lnd || p->n_disc != 0)) return -5;
  if (p->avail_cont && (!p->cont || p->act_dim < 3)) return -6;
  if (p->rmax < 1 || p->rmax * epw > 16) return -4;
  // one-row token passes (every stochastic rollout step) run on the one-wave kernel when it holds the configuration
  // (mat_decode_wave.hip; a null p->wfa keeps this 4-wave kernel: ops/mat_fused.WAVE_DECODE)
  {
    const int r = mdl_decode_wave(p, NB, st);
    if (r <= 0) return r;
  }
  size_t lds = mat_decode_lds_bytes(NB, epw, p->rmax, p->L);
  if (lds > 160 * 1024) return -2;
  const int grid = (p->B + epw - 1) / epw;
  // stage the per-row inputs in LDS when they fit next to the KV caches (MAT_DCML_DECODE_STAGE=0 disables)
  DecParams q = *p;
  static const bool stage_ok = [] { const char* e = getenv("MAT_DCML_DECODE_STAGE"); return !(e && e[0] == '0'); }();
  const size_t sb = mat_decode_stage_bytes(epw, p->L, p->act_dim, p->n_tok);
  q.stage = stage_ok && lds + sb <= 160 * 1024 && (p->rep != nullptr);
  if (q.stage) lds += sb;
  // precomputed cross-attention queries (MAT_DCML_DECODE_Q2PRE=0 disables) when they fit as well
  static const bool q2_ok = [] { const char* e = getenv("MAT_DCML_DECODE_Q2PRE"); return !(e && e[0] == '0'); }();
  const size_t q2b = (size_t)NB * (p->L + 16) * 64 * 2;
  q.q2pre = q2_ok && lds + q2b <= 160 * 1024 && p->rep != nullptr;
  if (q.q2pre) lds += q2b;
  p = &q;
#define MDL_DECODE_LAUNCH(NB_, STG_)                                                                            \
  hipFuncSetAttribute((const void*)mat_decode_kernel<NB_, STG_>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
  hipLaunchKernelGGL((mat_decode_kernel<NB_, STG_>), dim3(grid), dim3(256), lds, st, *p)
  switch (NB * 2 + (p->stage ? 1 : 0)) {
    case 2: MDL_DECODE_LAUNCH(1, false); break;
    case 3: MDL_DECODE_LAUNCH(1, true); break;
    case 4: MDL_DECODE_LAUNCH(2, false); break;
    case 5: MDL_DECODE_LAUNCH(2, true); break;
    case 6: MDL_DECODE_LAUNCH(3, false); break;
    case 7: MDL_DECODE_LAUNCH(3, true); break;
    default: return -3;
  }
#undef MDL_DECODE_LAUNCH
  MDL_CHECK_LAUNCH();
  return 0;
}
