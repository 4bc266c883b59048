// Round-2 fused MAT training tiles for gfx950: token-on-lane ("CT") register layout.
//
// Round 1 kept every activation in the MFMA C layout of Y = X·Wᵀ (rows = tokens in registers, one feature column
// per lane).  The next linear needs the token on the lane, so EVERY linear went through LDS: 16 ds_write_b16 +
// 16 cvt + 16 mask multiplies per lane, an lgkmcnt(0) drain, two ds_read_b128 — and LayerNorm needed 4 DPP
// steps per row.  At one wave per SIMD those drains were most of the kernels' 57 % s_waitcnt time and the
// conversion work most of their 27 VALU instructions per MFMA (profiles/r1_occupancy_ab.md).
//
// CT computes the transposed product Yᵀ = W·Xᵀ instead: A operand = weight rows, B operand = the activation with
// the TOKEN on the lane (lane&15) and 8 features per lane.  Its C layout (lane (g, c) holds features 16mt+4g+r of
// token c) is already the next product's B operand once two 16-row tiles are packed to bf16 — provided the weight
// fragment uses the same permuted k order perm(s, g, j) = 32s + 16(j>>2) + 4g + (j&3) (packed once per optimizer
// step, csrc/rl_ops.hip pack_weights "fa"/"ba").  So:
//  * linear → bias → GELU → linear → residual → LayerNorm chains never touch LDS (MLP forward: zero LDS ops);
//  * biases / residuals initialise the MFMA accumulators (no separate adds);
//  * per-token statistics (LayerNorm, softmax of the action head, value head) reduce 16 values in-lane and then
//    only across the 4 lanes of the token (v_permlane16/32_swap, no LDS);
//  * the operands of the attention (Q/K/V) and of the weight gradients (dY, X) go to the token-major swizzled LDS
//    tiles of round 1 with one ds_write_b64 per 4 features (was 4 ds_write_b16), so the round-1 MFMA attention and
//    the transposed-read weight-gradient GEMMs are reused unchanged;
//  * bias gradients come out of the weight-gradient MFMA loop (one extra MFMA against a ones fragment).
// Reference semantics: ma_transformer.py:24-230 (encoder / decoder blocks), transformer_act.py:103-129 (heads).
#pragma once
#include "mat_train_common.h"

// The backward kernels build in their own translation units (mat_enc_ct_bwd.hip / mat_dec_ct_bwd.hip: 8 waves per
// workgroup); per-TU exported names (the phase-profiler readers) carry this suffix.
#define MDL_CAT2(a, b) a##b
#define MDL_CAT(a, b) MDL_CAT2(a, b)
#ifdef MDL_CT_BWD_TU
#define MDL_CT_TU_SUFFIX _bwd
#else
#define MDL_CT_TU_SUFFIX
#endif

namespace {

// Phase profiler (-DMDL_CT_PROF): thread 0 of EVERY workgroup accumulates s_memtime cycles between marks (placed
// after workgroup barriers, so a phase = the slowest wave's span) in LDS and adds them to g_ctprof once per launch
// (no global traffic inside the kernel: the round-1 marks' read-modify-writes distorted the vmcnt waits).
#ifdef MDL_CT_PROF
__device__ unsigned long long g_ctprof[64];
__shared__ unsigned long long cp_acc[64];
#define CP_BEGIN() do { if (threadIdx.x < 64) cp_acc[threadIdx.x] = 0; __syncthreads(); \
  if (threadIdx.x == 0) cp_acc[63] = __builtin_amdgcn_s_memtime(); } while (0)
#define CP_MARK(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
  cp_acc[k] += t_ - cp_acc[63]; cp_acc[63] = t_; } } while (0)
#define CP_END() do { __syncthreads(); if (threadIdx.x < 63) atomicAdd(&g_ctprof[threadIdx.x], cp_acc[threadIdx.x]); } while (0)
#else
#define CP_BEGIN() do { } while (0)
#define CP_MARK(k) do { } while (0)
#define CP_END() do { } while (0)
#endif

// Forward kernels keep only Q / K / V in LDS (3 of the 6 token-major buffers): 74 KB at 192 rows, so TWO
// workgroups fit per CU (8 waves, 2 per SIMD: one workgroup's load / barrier stalls overlap the other's compute).
#ifndef MDL_FWD_WGPC
#define MDL_FWD_WGPC 2
#endif
constexpr int FWD_WGPC = MDL_FWD_WGPC;
__host__ __device__ inline size_t ct_fwd_lds_bytes(int NRP) { return (size_t)NRP * 64 * 2 * 3; }

template <typename K, typename PT, typename... X>
static int launch_ct(K kern, const PT* p, bool fwd, hipStream_t st, X... extra) {
  if (p->SQ <= 0 || p->NRP <= 0 || (p->SQ * p->L + 15) / 16 > NW * MAXRT) return -4;   // geometry not valid here
  const size_t lds = fwd ? ct_fwd_lds_bytes(p->NRP) : mat_train_lds_bytes(p->NRP, p->SQ, p->L);
  if (lds > (fwd ? LDS_BUDGET / FWD_WGPC : LDS_BUDGET)) return -2;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  const int tiles = (p->Bs + p->SQ - 1) / p->SQ;
  const int cap = n_cus() * (fwd ? FWD_WGPC : 1);
  const int grid = tiles < cap ? tiles : cap;
  // private gradient copies (GradMode): one copy per workgroup of THIS launch, and the fragment layout of the
  // 8-wave block mapping (grad_reduce_priv folds exactly `grid` copies)
  if (!fwd && p->g_copies > 0 && p->g_mode == 1 && (NW != 8 || grid > p->g_copies)) return -5;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), lds, st, *p, extra...);
  MDL_CHECK_LAUNCH();
  return 0;
}

struct CT { f32x4 v[4]; };          // v[mt][r] = feature 16mt + 4g + r of token (lane & 15) of a 16-token tile
struct CTr { uint2 q[4]; };         // the same as packed bf16: q[mt] = features 16mt+4g .. +3
struct AFr { bf16x8 f[4][2]; };     // A fragments of a 64x64 weight (rows 16mt + lane&15, k-step s, perm k order)

typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk2(float a, float b) {   // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
}
__device__ __forceinline__ bf16x8 mk8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(bf16x8, (u32x4v){a, b, c, d});
}
__device__ __forceinline__ float blo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bhi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

__device__ __forceinline__ void ct_zero(CT& t) {
#pragma unroll
  for (int i = 0; i < 4; ++i) t.v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
}
__device__ __forceinline__ CT ct_add(const CT& a, const CT& b) {
  CT o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o.v[i] = a.v[i] + b.v[i];
  return o;
}
__device__ __forceinline__ CTr ct_pack(const CT& x) {
  CTr r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.q[i] = make_uint2(pk2(x.v[i][0], x.v[i][1]), pk2(x.v[i][2], x.v[i][3]));
  return r;
}
__device__ __forceinline__ CT ct_unpack(const CTr& r) {
  CT x;
#pragma unroll
  for (int i = 0; i < 4; ++i) x.v[i] = f32x4{blo(r.q[i].x), bhi(r.q[i].x), blo(r.q[i].y), bhi(r.q[i].y)};
  return x;
}
__device__ __forceinline__ CTr ct_zero_r() {
  CTr r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.q[i] = make_uint2(0u, 0u);
  return r;
}
// k-step s of the B operand (features perm(s, g, j))
__device__ __forceinline__ bf16x8 rb(const CTr& r, int s) {
  return mk8(r.q[2 * s].x, r.q[2 * s].y, r.q[2 * s + 1].x, r.q[2 * s + 1].y);
}
// x ≈ hi + lo, both bf16 (≈16 significant bits) for the few products that need fp32-like accuracy
__device__ __forceinline__ void ct_split(const CT& x, CTr& hi, CTr& lo) {
  hi = ct_pack(x);
  const CT h = ct_unpack(hi);
  CT d;
#pragma unroll
  for (int i = 0; i < 4; ++i) d.v[i] = x.v[i] - h.v[i];
  lo = ct_pack(d);
}

__device__ __forceinline__ void loadA(AFr& W, const bf16_t* pk, int lane) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int s = 0; s < 2; ++s) W.f[mt][s] = *(const bf16x8*)(pk + ((size_t)((mt * 2 + s) * 64 + lane)) * 8);
}

// acc += W · x  (acc initialised by the caller: zero, bias, bias + residual)
__device__ __forceinline__ void mm(CT& acc, const AFr& W, const CTr& x) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 b = rb(x, s);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc.v[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W.f[mt][s], b, acc.v[mt], 0, 0, 0);
  }
}

// 64-float parameter vector as a CT (16-byte aligned: parameters are padded to 16 floats, ops/ppo_fused.PAD)
__device__ __forceinline__ CT ld_vec(const float* p, int lane) {
  const int g = lane >> 4;
  CT x;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) x.v[mt] = *(const f32x4*)(p + 16 * mt + 4 * g);
  return x;
}

__device__ __forceinline__ void gelu_ct(CT& t) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) t.v[i][r] = gelu_erf(t.v[i][r]);
}
// t <- GELU(t), gp <- GELU'(t) (one erf per element)
__device__ __forceinline__ void gelu_ct_both(CT& t, CT& gp) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float d;
      t.v[i][r] = gelu_erf_both(t.v[i][r], d);
      gp.v[i][r] = d;
    }
}

__device__ __forceinline__ float cross_row_max(float x) {
  float a, b;
  swap16(x, a, b);
  x = fmaxf(a, b);
  swap32(x, a, b);
  return fmaxf(a, b);
}

__device__ __forceinline__ bool tok_ok(int rt, const Ctx& c) { return rt * 16 + (c.lane & 15) < c.NR; }

// ------------------------------------------------------------------------------------------ LDS / global moves
// token-major swizzled LDS rows (tile.h tmo): piece mt of lane (g, c) = 8 bytes at column 16mt + 4g of row c
__device__ __forceinline__ void st_lds(bf16_t* buf, int rt, const CTr& x, bool ok, int lane) {
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) *(uint2*)(buf + tmo(row, 16 * mt + 4 * g)) = ok ? x.q[mt] : make_uint2(0u, 0u);
}
__device__ __forceinline__ CTr ld_lds(const bf16_t* buf, int rt, int lane) {
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
  CTr x;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) x.q[mt] = *(const uint2*)(buf + tmo(row, 16 * mt + 4 * g));
  return x;
}
// Saved activations (written by the forward, read only by the backward): one 128-byte record per token in the
// token-on-lane order — feature 16mt + 4g + r at element 16g + 4mt + r — so lane (g, c) owns 32 contiguous bytes of
// token c (two 16-byte accesses; a [tok][64] row-major record took four scattered 8-byte pieces per lane, and the
// forward's saves were store-issue bound).  Rows >= NR read as zero / are not written.
// A/B ablation (-DMDL_ABLATE_LDG): every chunk reads the saved rows of chunk 0 (L2-resident) instead of its own —
// wrong values, but it prices the HBM latency / bandwidth of the saved-activation loads.  Never in a shipped build.
#ifdef MDL_ABLATE_LDG
#define LDG_TOK0(t) 0
#else
#define LDG_TOK0(t) (t)
#endif
__device__ __forceinline__ CTr ld_g(const bf16_t* src, int tok0, int rt, int NR, int lane) {
  tok0 = LDG_TOK0(tok0);
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
  const bool ok = row < NR;
  const uint4* base = (const uint4*)(src + (size_t)(tok0 + (ok ? row : 0)) * 64 + 16 * g);
  const uint4 a = base[0], b = base[1];
  CTr x;
  x.q[0] = ok ? make_uint2(a.x, a.y) : make_uint2(0u, 0u);
  x.q[1] = ok ? make_uint2(a.z, a.w) : make_uint2(0u, 0u);
  x.q[2] = ok ? make_uint2(b.x, b.y) : make_uint2(0u, 0u);
  x.q[3] = ok ? make_uint2(b.z, b.w) : make_uint2(0u, 0u);
  return x;
}
// A/B ablation (-DMDL_ABLATE_SAVES, forward TUs): the saved-activation stores are skipped (a runtime-false predicate)
// — prices the forward's store traffic and the vmcnt waits of the loads queued behind it.  Never shipped.
#ifdef MDL_ABLATE_SAVES
#define SAVE_ON(row, NR) ((row) < (NR) && (NR) < 0)
#else
#define SAVE_ON(row, NR) ((row) < (NR))
#endif
// The saved-activation records leave as NONTEMPORAL stores (global_store ... nt): measured in the bench (rocprofv3),
// dec_fwd 189.8 -> 171.3 us and dec_bwd 483 -> 460 us per minibatch — the ~580 MB of records per minibatch no longer
// churn the L2 the forward's weight / rep loads and the backward's streams run through.  -DMDL_NT_SAVES=0: plain.
#ifndef MDL_NT_SAVES
#define MDL_NT_SAVES 1
#endif
#ifndef MDL_NT_SCALARS
#define MDL_NT_SCALARS 0   // A/B: the per-token f32 records (rstd, log-sum-exp) as nontemporal stores too
#endif
// MDL_SAVE_OLO=0 (A/B): the attention output is saved as bf16 only (its lo half — used only by the backward's
// delta = rowsum(dO O) — is not stored / loaded: 128 B per token and attention less in both directions)
#ifndef MDL_SAVE_OLO
#define MDL_SAVE_OLO 1
#endif
#ifndef MDL_SAVE_OLO2   // the same for the decoder's cross attention
#define MDL_SAVE_OLO2 MDL_SAVE_OLO
#endif
__device__ __forceinline__ void st_g(bf16_t* dst, int tok0, int rt, int NR, const CTr& x, int lane) {
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
  if (SAVE_ON(row, NR)) {
    u32x4v* base = (u32x4v*)(dst + (size_t)(tok0 + row) * 64 + 16 * g);
    const u32x4v a = {x.q[0].x, x.q[0].y, x.q[1].x, x.q[1].y}, b = {x.q[2].x, x.q[2].y, x.q[3].x, x.q[3].y};
#if MDL_NT_SAVES
    __builtin_nontemporal_store(a, base);
    __builtin_nontemporal_store(b, base + 1);
#else
    base[0] = a;
    base[1] = b;
#endif
  }
}
// plain global [tok][64] f32
__device__ __forceinline__ CT ld_gf(const float* src, int tok0, int rt, int NR, int lane) {
  tok0 = LDG_TOK0(tok0);
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
  const bool ok = row < NR;
  const float* base = src + (size_t)(tok0 + (ok ? row : 0)) * 64 + 4 * g;
  CT x;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const f32x4 v = *(const f32x4*)(base + 16 * mt);
    x.v[mt] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  return x;
}
__device__ __forceinline__ void st_gf(float* dst, int tok0, int rt, int NR, const CT& x, int lane) {
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
  if (row < NR) {
    float* base = dst + (size_t)(tok0 + row) * 64 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) *(f32x4*)(base + 16 * mt) = x.v[mt];
  }
}

// per-token f32 scalars ([tok]): LayerNorm rstd saved by the forward for the backward (lanes g = 0 write 16
// consecutive tokens)
__device__ __forceinline__ void st_tokf(float* dst, int rt, float v, const Ctx& c) {
  const int row = rt * 16 + (c.lane & 15);
  if ((c.lane >> 4) == 0 && SAVE_ON(row, c.NR)) {
#if MDL_NT_SCALARS
    __builtin_nontemporal_store(v, dst + (size_t)(c.tok0 + row));
#else
    dst[(size_t)(c.tok0 + row)] = v;
#endif
  }
}
__device__ __forceinline__ float ld_tokf(const float* src, int rt, const Ctx& c) {
  const int row = rt * 16 + (c.lane & 15);
  return row < c.NR ? src[(size_t)(LDG_TOK0(c.tok0) + row)] : 0.f;   // padded rows: rstd 0 -> zero gradient
}

// ------------------------------------------------------------------------------------------ LayerNorm (per token)
__device__ __forceinline__ float tok_sum(const CT& x) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += (x.v[i][0] + x.v[i][1]) + (x.v[i][2] + x.v[i][3]);
  return cross_row_sum(s);
}
#ifdef MDL_LN_ONEPASS   // the decoder translation units (measured: dec bwd -45 us, enc bwd +60 us with it)
// y = LN(x) * gamma + beta; returns rstd, xh = normalised x.  One pass: Σx and Σx² of the token reduce side by side
// (one cross-row exchange chain instead of two dependent ones), elementwise work on packed fp32 pairs.
__device__ __forceinline__ float ln_fwd_ct(const CT& x, CT& xh, CT& y, const CT& gam, const CT& bet) {
  f32x4 s4 = (x.v[0] + x.v[1]) + (x.v[2] + x.v[3]);
  f32x4 q4 = x.v[0] * x.v[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) q4 = x.v[i] * x.v[i] + q4;
  float s = (s4[0] + s4[1]) + (s4[2] + s4[3]), q = (q4[0] + q4[1]) + (q4[2] + q4[3]);
  float a0, b0, a1, b1;
  swap16(s, a0, b0);
  swap16(q, a1, b1);
  s = a0 + b0;
  q = a1 + b1;
  swap32(s, a0, b0);
  swap32(q, a1, b1);
  const float mean = (a0 + b0) * (1.f / 64.f);
  const float rstd = rsqrtf(fmaxf((a1 + b1) * (1.f / 64.f) - mean * mean, 0.f) + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xh.v[i] = (x.v[i] - mean) * rstd;
    y.v[i] = xh.v[i] * gam.v[i] + bet.v[i];
  }
  return rstd;
}
#else
// y = LN(x) * gamma + beta; returns rstd, xh = normalised x
__device__ __forceinline__ float ln_fwd_ct(const CT& x, CT& xh, CT& y, const CT& gam, const CT& bet) {
  const float mean = tok_sum(x) * (1.f / 64.f);
  const f32x4 m4 = {mean, mean, mean, mean};
#pragma unroll
  for (int i = 0; i < 4; ++i) xh.v[i] = x.v[i] - m4;
  f32x4 q4 = xh.v[0] * xh.v[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) q4 = xh.v[i] * xh.v[i] + q4;
  const float rstd = rsqrtf(cross_row_sum((q4[0] + q4[1]) + (q4[2] + q4[3])) * (1.f / 64.f) + 1e-5f);
  const f32x4 r4 = {rstd, rstd, rstd, rstd};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xh.v[i] *= r4;
    y.v[i] = xh.v[i] * gam.v[i] + bet.v[i];
  }
  return rstd;
}
#endif
// dx from dy; per-lane gamma / beta gradient partials in dg / db.  Padded token rows (row >= NR) need no mask here:
// every backward input is zero on them (the loss gradients, the saved activations and every LDS operand are
// stored masked, and xh of a padded row is the finite LN of its bias), so they contribute exactly zero.
// dx = rstd (gy - mean(gy) - xh mean(gy xh)) as two FMAs per element.
// Packed fp32 pairs throughout (f32x4 vector ops -> v_pk_*), the two row sums as trees, and their cross-row
// exchanges side by side (one swap chain for both).
__device__ __forceinline__ void ln_bwd_ct(const CT& dy, const CT& xh, float rstd, const CT& gam, bool /*ok*/, CT& dx,
                                          CT& dg, CT& db) {
  CT gy;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    gy.v[i] = dy.v[i] * gam.v[i];
    dg.v[i] = dy.v[i] * xh.v[i] + dg.v[i];
    db.v[i] += dy.v[i];
  }
  const f32x4 a4 = (gy.v[0] + gy.v[1]) + (gy.v[2] + gy.v[3]);
  f32x4 b4 = gy.v[0] * xh.v[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) b4 = gy.v[i] * xh.v[i] + b4;
  float a = (a4[0] + a4[1]) + (a4[2] + a4[3]), b = (b4[0] + b4[1]) + (b4[2] + b4[3]);
  float a0, a1, b0, b1;
  swap16(a, a0, a1);
  swap16(b, b0, b1);
  a = a0 + a1;
  b = b0 + b1;
  swap32(a, a0, a1);
  swap32(b, b0, b1);
  const float sc = rstd * (1.f / 64.f);
  const float A = (a0 + a1) * sc, B = (b0 + b1) * sc;
  const f32x4 r4 = {rstd, rstd, rstd, rstd}, mA = {-A, -A, -A, -A}, mB = {-B, -B, -B, -B};
#pragma unroll
  for (int i = 0; i < 4; ++i) dx.v[i] = xh.v[i] * mB + (gy.v[i] * r4 + mA);
}

// per-lane feature partials (summed over the tokens the lane saw) -> one atomic per feature: reduce over the 16
// token lanes of each row (DPP), then lane (g, c) adds feature 16(c>>2) + 4g + (c&3)
// Σ over the 16 tokens (lanes) of a row of 16 per-lane values, reduce-scattered: lane c ends with the sum of value c.
// Four butterfly steps (row mirror, half-row mirror, xor 2, xor 1) each halve the values a lane carries — 15 DPP
// adds instead of 16 full 16-lane reductions (64).
__device__ __forceinline__ float row_reduce_scatter16(const float (&v)[16], int lane) {
  const int c = lane & 15;
  float a[8], b[4], d[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool hi = c & 8;
    a[k] = (hi ? v[8 + k] : v[k]) + dppf<DPP_ROW_MIRROR>(hi ? v[k] : v[8 + k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool hi = c & 4;
    b[k] = (hi ? a[4 + k] : a[k]) + dppf<DPP_ROW_HALF_MIRROR>(hi ? a[k] : a[4 + k]);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool hi = c & 2;
    d[k] = (hi ? b[2 + k] : b[k]) + dppf<DPP_XOR2>(hi ? b[k] : b[2 + k]);
  }
  const bool hi = c & 1;
  return (hi ? d[1] : d[0]) + dppf<DPP_XOR1>(hi ? d[0] : d[1]);
}

// column sums of a CT accumulator (Σ over the 16 tokens of the lane row, then the 4 rows by the atomics) -> dst[64]
// (into the workgroup's LDS accumulator of parameter vector `slot`, global destination dst; vacc_add)
__device__ __forceinline__ void flush_vec(const CT& acc, float* dst, int slot, const Ctx& cx) {
  if (!dst) return;
  const int lane = cx.lane, c = lane & 15, g = lane >> 4;
  float v[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[4 * i + r] = acc.v[i][r];
  vacc_add(dst, slot, 16 * (c >> 2) + 4 * g + (c & 3), row_reduce_scatter16(v, lane), cx);
}

// ------------------------------------------------------------------------------------------ weight gradients
// A/B ablation (-DMDL_ABLATE_WATOM): the weight-gradient GEMMs run, but their fp32 atomics are skipped (a runtime-false
// predicate the compiler cannot fold) — measures what the atomic traffic costs.  Never in a shipped build.
#ifdef MDL_ABLATE_WATOM
#define WATOM(ptr, v) do { const float v_ = (v); if (v_ == 1.17549435e-38f) atomicAdd((ptr), v_); } while (0)
#else
#define WATOM(ptr, v) atomicAdd((ptr), (v))
#endif
// Weight-gradient blocks per wave (8-wave backward): wave w owns row block w & 3 and the two ADJACENT column tiles
// 2 (w >> 2), 2 (w >> 2) + 1, i.e. 16 rows x 32 contiguous columns of a 64 x 64 gradient.  The MFMA C layout puts
// lane (g, c) on rows 4g + r of one column tile — a per-register atomic would cover 4 rows x 64 B; one
// v_permlane16_swap + one v_permlane32_swap per register pair regroup the two tiles so that every fp32 atomic
// wave-instruction covers 2 rows x 128 contiguous bytes (the rate the memory-side atomic unit is measured at).
#ifndef MDL_WATOM_ROWS
#define MDL_WATOM_ROWS 1
#endif
constexpr bool WG_ROWS2 = MDL_WATOM_ROWS && NW == 8;
__device__ __forceinline__ int wg_ct(int wave, int j) { return WG_ROWS2 ? 2 * (wave >> 2) + j : (wave + NW * j) >> 2; }
__device__ __forceinline__ bool wg_has(int wave, int j) { return WG_ROWS2 ? true : wave + NW * j < 16; }
// flush a wave's 16 x 32 block (acc0 = column tile ct0, acc1 = ct0 + 1; rows 16 rb + 4g + r) of a 64-wide gradient
__device__ __forceinline__ void flush_rows2(const f32x4& acc0, const f32x4& acc1, float* dW, int rb, int ct0, int lane) {
  const int s = lane >> 5, col = 16 * ct0 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x0 = acc0[r], x1 = acc1[r];   // scalars first: never bit_cast a subscripted vector element
    const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x0), __builtin_bit_cast(unsigned, x1),
                                                    false, false);   // [a0 b0 a2 b2], [a1 b1 a3 b3] (16-lane rows)
    const auto q = __builtin_amdgcn_permlane32_swap((unsigned)p[0], (unsigned)p[1], false, false);   // [a0 b0 a1 b1], [a2 b2 a3 b3]
    WATOM(dW + (16 * rb + 4 * s + r) * 64 + col, __builtin_bit_cast(float, (unsigned)q[0]));
    WATOM(dW + (16 * rb + 8 + 4 * s + r) * 64 + col, __builtin_bit_cast(float, (unsigned)q[1]));
  }
}
// Private-copy flush variants (A/B, MDL_PRIV_FLUSH): 0 = plain load + add + store after the first chunk; 1 = the same
// with nontemporal loads / stores (the copies do not churn the L2 the saved activations stream through); 2 = the
// first chunk stores (nontemporal), later chunks add with fp32 atomics — one writer per address and program order,
// so still deterministic, and no load latency in the wave.
#ifndef MDL_PRIV_FLUSH
#define MDL_PRIV_FLUSH 0
#endif
__device__ __forceinline__ f32x4 priv_ld4(const f32x4* p) {
  if constexpr (MDL_PRIV_FLUSH == 1) return __builtin_nontemporal_load(p);
  return *p;
}
__device__ __forceinline__ float priv_ld1(const float* p) {
  if constexpr (MDL_PRIV_FLUSH == 1) return __builtin_nontemporal_load(p);
  return *p;
}
// v = this chunk's partial; old = the earlier chunks' (loaded, variants 0 / 1)
__device__ __forceinline__ void priv_st4(f32x4* p, f32x4 v, f32x4 old, bool first) {
  if constexpr (MDL_PRIV_FLUSH == 2) {
    if (first) {
      __builtin_nontemporal_store(v, p);
    } else {
      float* q = reinterpret_cast<float*>(p);
      const float v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
      atomicAdd(q, v0);
      atomicAdd(q + 1, v1);
      atomicAdd(q + 2, v2);
      atomicAdd(q + 3, v3);
    }
  } else if constexpr (MDL_PRIV_FLUSH == 1) {
    __builtin_nontemporal_store(v + old, p);
  } else {
    *p = v + old;
  }
}
__device__ __forceinline__ void priv_st1(float* p, float v, float old, bool first) {
  if constexpr (MDL_PRIV_FLUSH == 2) {
    if (first) __builtin_nontemporal_store(v, p);
    else atomicAdd(p, v);
  } else if constexpr (MDL_PRIV_FLUSH == 1) {
    __builtin_nontemporal_store(v + old, p);
  } else {
    *p = v + old;
  }
}
constexpr bool PRIV_LOADS = MDL_PRIV_FLUSH != 2;   // variants that read the earlier chunks' partials

// Private-copy position of a lane's accumulator j (an f32x4 over r) of a 64 x 64 weight gradient: FRAGMENT order
// (wave, lane, j, r) with the 8-wave block mapping above (row 16 (w & 3) + 4 g + r, column 16 (2 (w >> 2) + j) + c);
// csrc/ppo.hip grad_reduce_priv folds the copies and writes each element to its row-major place.
__device__ __forceinline__ f32x4* frag_slot(float* dW, int wave, int lane, int j) {
  return reinterpret_cast<f32x4*>(dW + wave * 512 + lane * 8 + 4 * j);
}

// dW[n][k] (row stride ld) += Σ_t Y[t][n] X[t][k] for n < nrows, k < ncols, and db[n] += Σ_t Y[t][n], from
// token-major swizzled LDS tiles of KP rows (KP % 32 == 0, padded rows zero).  The 16 output blocks (row block
// j & 3, column tile j >> 2) are dealt round robin, j = wave + NW i: a wave's blocks share one row block (NW % 4 == 0)
// and so one Y fragment per k-step.  The bias gradient is one extra MFMA per k-step against a ones fragment (the
// waves holding column tile 0).  Shared workspace copies: fp32 atomics; private copies (GradMode): row-major
// stores, or load + add + store after the workgroup's first chunk (loads issued before the MFMA loop).
// Y2 (optional): a second dY tile added in the same pass (the lo half of a hi / lo split dY) — one flush instead of
// two, so a private copy is read-modified-written once per chunk (two passes made the second pass's loads wait for
// the first pass's stores to the same addresses: ~6 us per chunk in the decoder's embedding backward)
__device__ __forceinline__ void wgrad_g(const bf16_t* Y, const bf16_t* X, int KP, float* dW, int ld, int nrows, int ncols,
                                        float* db, int wave, int lane, GradMode gm, const bf16_t* Y2 = nullptr) {
  static_assert(NW % 4 == 0, "row block per wave");
  constexpr int NCT = (16 + NW - 1) / NW;           // column tiles per wave (at most)
  const int rb = wave & 3;
  if (wave >= 4) db = nullptr;
  const int nct = dW ? (ncols + 15) >> 4 : 0;
  if ((!db && wg_ct(wave, 0) >= nct) || 16 * rb >= nrows) return;
  const int g = lane >> 4, c16 = lane & 15;
  gm.priv = gm.priv && !MDL_NO_PRIV;
  const bool rmw = PRIV_LOADS && gm.priv && !gm.first;
  f32x4 old[NCT];
  float oldb = 0.f;
#pragma unroll
  for (int j = 0; j < NCT; ++j) {
    const int ct = wg_ct(wave, j);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * rb + 4 * g + r, k = 16 * ct + c16;
      const bool ok = rmw && dW && wg_has(wave, j) && ct < nct && n < nrows && k < ncols;
      old[j][r] = ok ? priv_ld1(dW + n * ld + k) : 0.f;
    }
  }
  if (rmw && db && c16 < 4 && 16 * rb + 4 * g + c16 < nrows) oldb = priv_ld1(db + 16 * rb + 4 * g + c16);
  f32x4 acc[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  for (int k0 = 0; k0 < KP; k0 += 32) {
    const bf16x8 a = ld_frag_T(Y, k0, 16 * rb, lane);
    bf16x8 a2;
    if (Y2) a2 = ld_frag_T(Y2, k0, 16 * rb, lane);
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int ct = wg_ct(wave, j);
      if (wg_has(wave, j) && ct < nct) {
        const bf16x8 b = ld_frag_T(X, k0, 16 * ct, lane);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
        if (Y2) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b, acc[j], 0, 0, 0);
      }
    }
    if (db) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ones, accb, 0, 0, 0);
  }
  if (dW && gm.priv) {
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int ct = wg_ct(wave, j);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * rb + 4 * g + r, k = 16 * ct + c16;
        if (wg_has(wave, j) && ct < nct && n < nrows && k < ncols) priv_st1(dW + n * ld + k, acc[j][r], old[j][r], gm.first);
      }
    }
  } else if (dW && WG_ROWS2 && ld == 64 && nrows == 64 && ncols == 64) {
    if constexpr (WG_ROWS2) flush_rows2(acc[0], acc[1], dW, rb, wg_ct(wave, 0), lane);
  } else if (dW) {
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int ct = wg_ct(wave, j);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * rb + 4 * g + r, k = 16 * ct + c16;
        const bool ok = wg_has(wave, j) && ct < nct && n < nrows && k < ncols;
        if (ok) WATOM(dW + n * ld + k, acc[j][r]);
      }
    }
  }
  if (db && c16 < 4) {
    const float v = c16 == 0 ? accb[0] : c16 == 1 ? accb[1] : c16 == 2 ? accb[2] : accb[3];
    const int n = 16 * rb + 4 * g + c16;
    if (n < nrows) {
      if (gm.priv) priv_st1(db + n, v, oldb, gm.first);
      else atomicAdd(db + n, v);
    }
  }
}

// The same product for a SMALL gradient (nrows x ld <= 64 (slot_end - slot0) floats: the decoder's action embedding
// 64 x (A+1) and action head A x 64 for A <= 2), accumulated in the workgroup's LDS vector slots (vacc_add: 2^-32
// fixed point, order-free) across all of its chunks and flushed once per launch (vacc_end): no global traffic per
// chunk.  A private copy's per-chunk read-modify-write here stalled the decoder backward: the loads wait for the
// previous chunk's stores in the in-order vector-memory counter (head + embedding backward 22 % of dec_bwd vs 14 % with
// atomics).  dW rows are ld floats apart (ld >= ncols, row-major, contiguous: slot s = element e / 64); the bias
// gradient db (nrows floats) takes slot bslot.
__device__ __forceinline__ void wgrad_g_vacc(const bf16_t* Y, const bf16_t* X, int KP, float* dW, int ld, int nrows,
                                             int ncols, float* db, int slot0, int bslot, const Ctx& c,
                                             const bf16_t* Y2 = nullptr) {
  constexpr int NCT = (16 + NW - 1) / NW;
  const int wave = c.wave, lane = c.lane, rb = wave & 3;
  if (wave >= 4) db = nullptr;
  const int nct = dW ? (ncols + 15) >> 4 : 0;
  if ((!db && wg_ct(wave, 0) >= nct) || 16 * rb >= nrows) return;
  const int g = lane >> 4, c16 = lane & 15;
  f32x4 acc[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  for (int k0 = 0; k0 < KP; k0 += 32) {
    const bf16x8 a = ld_frag_T(Y, k0, 16 * rb, lane);
    bf16x8 a2;
    if (Y2) a2 = ld_frag_T(Y2, k0, 16 * rb, lane);
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int ct = wg_ct(wave, j);
      if (wg_has(wave, j) && ct < nct) {
        const bf16x8 b = ld_frag_T(X, k0, 16 * ct, lane);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
        if (Y2) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b, acc[j], 0, 0, 0);
      }
    }
    if (db) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ones, accb, 0, 0, 0);
  }
  const int total = nrows * ld;
  if (dW) {
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int ct = wg_ct(wave, j);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * rb + 4 * g + r, k = 16 * ct + c16, e = n * ld + k;
        if (wg_has(wave, j) && ct < nct && n < nrows && k < ncols) {
          const int s = e >> 6, len = total - 64 * s;
          vacc_add(dW + 64 * s, slot0 + s, e & 63, acc[j][r], c, len < 64 ? len : 64);
        }
      }
    }
  }
  if (db && c16 < 4) {
    const float v = c16 == 0 ? accb[0] : c16 == 1 ? accb[1] : c16 == 2 ? accb[2] : accb[3];
    const int n = 16 * rb + 4 * g + c16;
    if (n < nrows) vacc_add(db, bslot, n, v, c, nrows);
  }
}

// The weight gradients of ONE, TWO or THREE 64x64 matrices that share their input X (dW_q / dW_k / dW_v of an
// attention, dW_k / dW_v of the cross attention): one pass over the token axis reads each X fragment once for all
// of them (a pass per matrix re-read X: 6 transposed LDS reads per 2 MFMAs; here 2 + 2 NM per 2 NM).  Private copies:
// fragment-order 16-byte stores (frag_slot), the earlier chunks' partials loaded before the MFMA loop.
template <int NM>
__device__ __forceinline__ void wgrad64_shared_x(const bf16_t* const (&Y)[NM], const bf16_t* X, const Mat* const (&m)[NM],
                                                 const Ctx& c) {
  static_assert(NW % 4 == 0, "row block per wave");
  constexpr int NCT = (16 + NW - 1) / NW;
  const int wave = c.wave, lane = c.lane, KP = c.KP;
  const int rb = wave & 3;
  const bool bias = wave < 4;
  const int g = lane >> 4, c16 = lane & 15;
  // private copies need the 8-wave block mapping of frag_slot (the host refuses the mode otherwise)
  const bool priv = !MDL_NO_PRIV && NW == 8 && c.gm.priv, rmw = PRIV_LOADS && priv && !c.gm.first;
  f32x4 old[NM][NCT];
  float oldb[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    float* dW = c.g(m[i]->dW);
    float* db = c.g(m[i]->db);
#pragma unroll
    for (int j = 0; j < NCT; ++j) old[i][j] = (rmw && dW) ? priv_ld4(frag_slot(dW, wave, lane, j)) : f32x4{0.f, 0.f, 0.f, 0.f};
    oldb[i] = (rmw && bias && db && c16 < 4) ? priv_ld1(db + 16 * rb + 4 * g + c16) : 0.f;
  }
  f32x4 acc[NM][NCT], accb[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  for (int k0 = 0; k0 < KP; k0 += 32) {
    bf16x8 xb[NCT];
#pragma unroll
    for (int j = 0; j < NCT; ++j)
      if (wg_has(wave, j)) xb[j] = ld_frag_T(X, k0, 16 * wg_ct(wave, j), lane);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const bf16x8 a = ld_frag_T(Y[i], k0, 16 * rb, lane);
#pragma unroll
      for (int j = 0; j < NCT; ++j)
        if (wg_has(wave, j)) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xb[j], acc[i][j], 0, 0, 0);
      if (bias) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ones, accb[i], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    float* dW = c.g(m[i]->dW);
    float* db = c.g(m[i]->db);
    if (dW) {
      if (priv) {
#pragma unroll
        for (int j = 0; j < NCT; ++j) priv_st4(frag_slot(dW, wave, lane, j), acc[i][j], old[i][j], c.gm.first);
      } else if constexpr (WG_ROWS2) {
        flush_rows2(acc[i][0], acc[i][1], dW, rb, wg_ct(wave, 0), lane);
      } else {
#pragma unroll
        for (int j = 0; j < NCT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (wg_has(wave, j)) WATOM(dW + (16 * rb + 4 * g + r) * 64 + 16 * wg_ct(wave, j) + c16, acc[i][j][r]);
      }
    }
    if (bias && db && c16 < 4) {
      const float v = c16 == 0 ? accb[i][0] : c16 == 1 ? accb[i][1] : c16 == 2 ? accb[i][2] : accb[i][3];
      if (priv) priv_st1(db + 16 * rb + 4 * g + c16, v, oldb[i], c.gm.first);
      else atomicAdd(db + 16 * rb + 4 * g + c16, v);
    }
  }
}
__device__ __forceinline__ void wgrad64(const bf16_t* Y, const bf16_t* X, const Mat& m, const Ctx& c) {
  const bf16_t* const ys[1] = {Y};
  const Mat* const ms[1] = {&m};
  wgrad64_shared_x<1>(ys, X, ms, c);
}

// q / k / v projections of the packed tiles xp (one weight matrix live at a time) -> QB / KB / VB; m0 = index of
// the query matrix (0: self attention; the cross attention has its own q input)
// sv_save (forward): the input tiles are saved right after the FIRST weight load is issued (not before the phase's
// barrier: a store ahead of the weight loads would make them wait for it in the wave's in-order vmcnt)
__device__ __forceinline__ void proj3(const Mat* m, int m0, const CTr* xp, const Ctx& c, bf16_t* sv_save = nullptr) {
  bf16_t* outs[3] = {c.QB, c.KB, c.VB};
#pragma unroll
  for (int mi = 0; mi < 3; ++mi) {
    AFr W;
    loadA(W, m[m0 + mi].fa, c.lane);
    const CT b = ld_vec(m[m0 + mi].b, c.lane);
    if (mi == 0 && sv_save) {
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) st_g(sv_save, c.tok0, rt, c.NR, xp[k], c.lane);
      }
    }
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        CT t = b;
        mm(t, W, xp[k]);
        st_lds(outs[mi], rt, ct_pack(t), tok_ok(rt, c), c.lane);
      }
    }
  }
}

// dx[k] (+)= Σ_i W_iᵀ · (tile k of LDS buffer src_i) for the three projection matrices m[m0 .. m0+2]
__device__ __forceinline__ void proj3_bwd(const Mat* m, int m0, const bf16_t* s0, const bf16_t* s1, const bf16_t* s2,
                                          CT* d0, CT* d12, const Ctx& c) {
  const bf16_t* srcs[3] = {s0, s1, s2};
#pragma unroll
  for (int mi = 0; mi < 3; ++mi) {
    AFr W;
    loadA(W, m[m0 + mi].ba, c.lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) mm(mi == 0 ? d0[k] : d12[k], W, ld_lds(srcs[mi], rt, c.lane));
    }
  }
}

// ------------------------------------------------------------------------------------------ attention (CT)
// Sequence-block-diagonal attention over the workgroup's packed rows, per (16-row tile, head), keys / queries visited
// in 32-row chunks.  Round-1 MFMA attention (mat_train_common.h) with the operands turned around so that every
// product's output lands in the token-on-lane layout:
//  * scores: Sᵀ = K·Qᵀ (round 1): lane (g, c) holds S[query c][keys kb + 8g + j] — already the B operand (k = keys,
//    n = query) of Oᵀ = Vᵀ·Pᵀ, whose A operand Vᵀ comes from ds_read_b64_tr_b16 of the token-major V;
//  * so O (and dQ, dK, dV in the backward) come out as CT tiles — O feeds the output projection from registers;
//  * forward: ONE pass with an online max (round 1 took two: max/sum, then P·V), scores in log2 units so that
//    p = exp2(s - m) is a subtract + v_exp; P and dS enter their MFMAs as hi/lo bf16 pairs (dS rows sum to zero and
//    feed bias gradients; a single-bf16 P left the cross-attention query-bias gradient at 2.6x the bf16 yardstick);
//  * log-sum-exp is saved in log2 units ([tok][2], consumed only by these kernels).
constexpr float ATT_L2 = 0.17677669529663687f * 1.4426950408889634f;   // 1/sqrt(32) * log2(e)

struct QSpan { int qs, qe; };   // keys [qs, qe) visible to a query (empty for padded rows)
__device__ __forceinline__ QSpan qspan(int q, bool causal, const Ctx& c) {
  QSpan s;
  s.qs = (q / c.L) * c.L;
  s.qe = q >= c.NR ? s.qs : (causal ? q + 1 : min(s.qs + c.L, c.NR));
  return s;
}

// key j of this lane's chunk slots is visible iff qs <= base + j < qe: ONE unsigned compare of (base - qs + j)
// against the span (was two signed compares and a mask AND per key)
__device__ __forceinline__ bool key_vis(int d0, unsigned span, int j) { return (unsigned)(d0 + j) < span; }

// raw scores of one chunk for this lane's query (unscaled), invisible keys -inf; the 1/sqrt(d) log2(e) scale is
// applied by the consumer inside its exp2 argument (one FMA)
__device__ __forceinline__ void chunk_scores(const bf16_t* K, int kb, int h, const bf16x8& qB, const QSpan& qs,
                                             float* sc, int lane) {
  score_chunk_T(K, kb, h, qB, sc, lane);
  const int d0 = kb + 8 * (lane >> 4) - qs.qs;
  const unsigned span = (unsigned)(qs.qe - qs.qs);
#pragma unroll
  for (int j = 0; j < 8; ++j) sc[j] = key_vis(d0, span, j) ? sc[j] : -INFINITY;
}

__device__ __forceinline__ bf16x8 pack8v(const float* x) {
  return mk8(pk2(x[0], x[1]), pk2(x[2], x[3]), pk2(x[4], x[5]), pk2(x[6], x[7]));
}
__device__ __forceinline__ void split8v(const float* x, bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = pk2(x[2 * i], x[2 * i + 1]);
    l[i] = pk2(x[2 * i] - blo(h[i]), x[2 * i + 1] - bhi(h[i]));
  }
  hi = mk8(h[0], h[1], h[2], h[3]);
  lo = mk8(l[0], l[1], l[2], l[3]);
}

// forward: O (CT, the wave's query tiles rt = wave + NW k, both heads) = softmax(scale Q Kᵀ) V
// lse (optional): this lane's log-sum-exp per (tile, head), stored by the CALLER (lse_store_fwd) once it has issued
// the next phase's weight loads — a store issued before them would sit ahead of them in the wave's in-order vmcnt
__device__ __forceinline__ void attn_fwd_ct(const bf16_t* Q, const bf16_t* K, const bf16_t* V, bool causal, float* lse_g,
                                            CT* O, const Ctx& c, float (*lse)[2] = nullptr) {
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      const int q = rt * 16 + c16;
      const QSpan qs = qspan(q, causal, c);
      const SeqSpan sp = tile_span(rt, c, causal);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bf16x8 qB = lda_tm(Q, q, 4 * h + g);
        float m = -INFINITY, l = 0.f;
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
        for (int kb = sp.lo; kb < sp.hi; kb += 32) {
          float sc[8];
          chunk_scores(K, kb, h, qB, qs, sc, lane);
          float cm = sc[0];
#pragma unroll
          for (int j = 1; j < 8; ++j) cm = fmaxf(cm, sc[j]);
          const float nm = fmaxf(m, cross_row_max(cm) * ATT_L2);   // running max in log2 units
          const float mr = nm == -INFINITY ? 0.f : nm;
          const float alpha = fast_exp2(m - mr);
          float ps = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            sc[j] = fast_exp2(fmaf(sc[j], ATT_L2, -mr));
            ps += sc[j];
          }
          l = l * alpha + ps;
          o0 *= alpha;
          o1 *= alpha;
          bf16x8 ph, pl;
          split8v(sc, ph, pl);
          const bf16x8 va = ld_frag_T(V, kb, 32 * h, lane), vb = ld_frag_T(V, kb, 32 * h + 16, lane);
          o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, ph, o0, 0, 0, 0);
          o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pl, o0, 0, 0, 0);
          o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb, ph, o1, 0, 0, 0);
          o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb, pl, o1, 0, 0, 0);
          m = nm;
        }
        l = cross_row_sum(l);
        const float il = l > 0.f ? 1.f / l : 0.f;
        O[k].v[2 * h] = o0 * il;
        O[k].v[2 * h + 1] = o1 * il;
        if (lse) {
          lse[k][h] = l > 0.f ? m + __log2f(l) : 0.f;
        } else if (lse_g && g == 0 && q < c.NR) {
          const float lv = l > 0.f ? m + __log2f(l) : 0.f;
#if MDL_NT_SCALARS
          __builtin_nontemporal_store(lv, lse_g + (size_t)(c.tok0 + q) * 2 + h);
#else
          lse_g[(size_t)(c.tok0 + q) * 2 + h] = lv;
#endif
        }
      }
    }
  }
}

__device__ __forceinline__ void lse_store_fwd(float* lse_g, const float (*lse)[2], const Ctx& c) {
  const int g = c.lane >> 4;
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k, q = rt * 16 + (c.lane & 15);
    if (rt < c.NT && g == 0 && q < c.NR) {
#pragma unroll
      for (int h = 0; h < 2; ++h) lse_g[(size_t)(c.tok0 + q) * 2 + h] = lse[k][h];
    }
  }
}

// CT pieces mt0, mt0+1 (features 16mt0 .. 16mt0+31 = one head) of row tile rt -> token-major LDS
__device__ __forceinline__ void st_lds_head(bf16_t* buf, int rt, int h, f32x4 a, f32x4 b, bool ok, int lane) {
  const int g = lane >> 4, row = rt * 16 + (lane & 15);
  const uint2 ua = ok ? make_uint2(pk2(a[0], a[1]), pk2(a[2], a[3])) : make_uint2(0u, 0u);
  const uint2 ub = ok ? make_uint2(pk2(b[0], b[1]), pk2(b[2], b[3])) : make_uint2(0u, 0u);
  *(uint2*)(buf + tmo(row, 32 * h + 4 * g)) = ua;
  *(uint2*)(buf + tmo(row, 32 * h + 16 + 4 * g)) = ub;
}

// delta_q = Σ_k P_qk dP_qk = Σ_d dO_qd O_qd per (query, head) (dP = dO Vᵀ, O = P V): from the saved forward output
// O and dO in registers (CT layout, both heads) -> DEL [head][row] in LDS.  Replaces a full extra sweep over the keys
// (scores, exp2 and dP MFMAs) in the query pass.
// O = hi + lo (saved bf16 pair); dO as stored in DA (bf16), the same values the dP MFMAs see.
__device__ __forceinline__ void attn_delta_ct(const CTr& ohi, const CTr& olo, const CTr& dOr, int rt, bool ok,
                                              const Ctx& c) {
  const CT oh = ct_unpack(ohi), ol = ct_unpack(olo), dO = ct_unpack(dOr);
  float d[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // packed pairs, a tree per head
    const f32x4 t = (oh.v[2 * h] + ol.v[2 * h]) * dO.v[2 * h] + (oh.v[2 * h + 1] + ol.v[2 * h + 1]) * dO.v[2 * h + 1];
    d[h] = (t[0] + t[1]) + (t[2] + t[3]);
  }
  float a0, a1, b0, b1;   // both heads' cross-row sums side by side
  swap16(d[0], a0, a1);
  swap16(d[1], b0, b1);
  d[0] = a0 + a1;
  d[1] = b0 + b1;
  swap32(d[0], a0, a1);
  swap32(d[1], b0, b1);
  d[0] = a0 + a1;
  d[1] = b0 + b1;
  if ((c.lane >> 4) == 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) c.DEL[h * c.NRP + rt * 16 + (c.lane & 15)] = ok ? d[h] : 0.f;
  }
}

// backward, by (query tile, head) item: dQ = scale Σ_k dS K (-> DQ, token-major), dS = P (dP - delta) with delta from
// DEL (attn_delta_ct); LSE in log2 units.  Items are dealt round robin (a runtime loop: the per-wave tile loop of the
// forward blew up the backward kernels' code and register pressure).
__device__ __forceinline__ void attn_bwd_q_ct(const bf16_t* Q, const bf16_t* K, const bf16_t* V, const bf16_t* DA,
                                              bf16_t* DQ, bool causal, const Ctx& c) {
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  for (int item = c.wave; item < 2 * c.NT; item += NW) {
    const int rt = item >> 1, h = item & 1;
    const int q = rt * 16 + c16;
    const QSpan qs = qspan(q, causal, c);
    const SeqSpan sp = tile_span(rt, c, causal);
    const bf16x8 qB = lda_tm(Q, q, 4 * h + g), dB = lda_tm(DA, q, 4 * h + g);
    const float lse = c.LSE[h * c.NRP + q];
    const float delta = c.DEL[h * c.NRP + q];
    f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
    for (int kb = sp.lo; kb < sp.hi; kb += 32) {
      float sc[8], dp[8];
      chunk_scores(K, kb, h, qB, qs, sc, lane);
      score_chunk_T(V, kb, h, dB, dp, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[j] = fast_exp2(fmaf(sc[j], ATT_L2, -lse)) * (dp[j] - delta);
      bf16x8 dsh, dsl;
      split8v(sc, dsh, dsl);
      const bf16x8 k0 = ld_frag_T(K, kb, 32 * h, lane), k1 = ld_frag_T(K, kb, 32 * h + 16, lane);
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, dsh, d0, 0, 0, 0);
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, dsl, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, dsh, d1, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, dsl, d1, 0, 0, 0);
    }
    st_lds_head(DQ, rt, h, d0 * ATT_SCALE, d1 * ATT_SCALE, q < c.NR, lane);
  }
}

// backward, by (key tile, head) item: dV = Pᵀ dO, dK = scale dSᵀ Q, written over the item's own K / V head columns
__device__ __forceinline__ void attn_bwd_kv_ct(const bf16_t* Q, bf16_t* K, bf16_t* V, const bf16_t* DA, bool causal,
                                               const Ctx& c) {
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  for (int item = c.wave; item < 2 * c.NT; item += NW) {
    const int rt = item >> 1, h = item & 1;
    const int kk = rt * 16 + c16;
    const bool kv = kk < c.NR;
    const int ks = (kk / c.L) * c.L, ke = min(ks + c.L, c.NR);
    const int qlo = causal ? kk : ks;
    const unsigned qspan_n = kv ? (unsigned)(ke - qlo) : 0u;   // queries [qlo, ke) see this key
    SeqSpan sp = tile_span(rt, c, false);
    if (causal) sp.lo = (rt * 16) & ~31;
    const bf16x8 kB = lda_tm(K, kk, 4 * h + g), vB = lda_tm(V, kk, 4 * h + g);
    f32x4 k0a = {0.f, 0.f, 0.f, 0.f}, k1a = {0.f, 0.f, 0.f, 0.f}, v0a = {0.f, 0.f, 0.f, 0.f}, v1a = {0.f, 0.f, 0.f, 0.f};
    for (int qb = sp.lo; qb < sp.hi; qb += 32) {
      float sc[8], dp[8];
      score_chunk_T(Q, qb, h, kB, sc, lane);    // sc[j] = S[query qb + 8g + j][key kk]
      score_chunk_T(DA, qb, h, vB, dp, lane);   // dp[j] = dP[query][key kk]
      const float4* lp = (const float4*)(c.LSE + h * c.NRP + qb + 8 * g);
      const float4* dl = (const float4*)(c.DEL + h * c.NRP + qb + 8 * g);
      const float4 l0 = lp[0], l1 = lp[1], e0 = dl[0], e1 = dl[1];
      const float lsev[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
      const float delv[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
      float pv[8], ds[8];
      const int d0 = qb + 8 * g - qlo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pv[j] = fast_exp2(key_vis(d0, qspan_n, j) ? fmaf(sc[j], ATT_L2, -lsev[j]) : -INFINITY);
        ds[j] = pv[j] * (dp[j] - delv[j]);
      }
      bf16x8 ph, pl, dsh, dsl;
      split8v(pv, ph, pl);
      split8v(ds, dsh, dsl);
      const bf16x8 o0 = ld_frag_T(DA, qb, 32 * h, lane), o1 = ld_frag_T(DA, qb, 32 * h + 16, lane);
      v0a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o0, ph, v0a, 0, 0, 0);
      v0a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o0, pl, v0a, 0, 0, 0);
      v1a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o1, ph, v1a, 0, 0, 0);
      v1a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o1, pl, v1a, 0, 0, 0);
      const bf16x8 q0 = ld_frag_T(Q, qb, 32 * h, lane), q1 = ld_frag_T(Q, qb, 32 * h + 16, lane);
      k0a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(q0, dsh, k0a, 0, 0, 0);
      k0a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(q0, dsl, k0a, 0, 0, 0);
      k1a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(q1, dsh, k1a, 0, 0, 0);
      k1a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(q1, dsl, k1a, 0, 0, 0);
    }
    st_lds_head(K, rt, h, k0a * ATT_SCALE, k1a * ATT_SCALE, kv, lane);
    st_lds_head(V, rt, h, v0a, v1a, kv, lane);
  }
}

// ------------------------------------------------------------------------------------------ sublayers (forward)
// self attention: x <- LN(x + proj(attn(q(x), k(x), v(x))))   (ma_transformer.py:89-92,112)
template <bool SAVE>
__device__ __forceinline__ void self_attn_fwd_ct(const Mat* m, const LNp& ln, CT* xr, bool causal, bf16_t* sv_xin,
                                                 bf16_t* sv_a, bf16_t* sv_alo, float* sv_lse, bf16_t* sv_xh,
                                                 float* sv_rs, const Ctx& c) {
  const int lane = c.lane;
  {
    CTr xp[MAXRT];
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) xp[k] = ct_pack(xr[k]);
    }
    __syncthreads();   // every wave done reading the previous attention's K / V (no barrier after an attention)
    proj3(m, 0, xp, c, SAVE ? sv_xin : nullptr);
  }
  __syncthreads();
  CP_MARK(20);
  CT O[MAXRT];
  float lse[MAXRT][2];
  attn_fwd_ct(c.QB, c.KB, c.VB, causal, nullptr, O, c, lse);
  CP_MARK(21);
  AFr Wp;
  loadA(Wp, m[3].fa, lane);
  const CT bp = ld_vec(m[3].b, lane), gam = ld_vec(ln.g, lane), bet = ld_vec(ln.b, lane);
  if (SAVE) lse_store_fwd(sv_lse, lse, c);   // behind the proj weight loads
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      CTr a, alo;
      if (MDL_SAVE_OLO) ct_split(O[k], a, alo); else a = ct_pack(O[k]);
      if (SAVE) {
        st_g(sv_a, c.tok0, rt, c.NR, a, lane);
        if (MDL_SAVE_OLO) st_g(sv_alo, c.tok0, rt, c.NR, alo, lane);
      }
      CT t = ct_add(bp, xr[k]), xh;
      mm(t, Wp, a);
      const float rs = ln_fwd_ct(t, xh, xr[k], gam, bet);
      if (SAVE) {
        st_g(sv_xh, c.tok0, rt, c.NR, ct_pack(xh), lane);
        st_tokf(sv_rs, rt, rs, c);
      }
    }
  }  CP_MARK(22);
}

// MLP: x <- LN(x + W2 GELU(W1 x + b1) + b2)   (ma_transformer.py:84-86,91-92)
// MDL_SAVE_PREACT (A/B): the training forward saves the pre-activation h (bf16) instead of GELU(h) and GELU'(h) — 128 B
// per token and MLP less in both directions; the W2 operand is GELU(bf16(h)) in both passes (autocast's rounding
// point), and the backward re-derives GELU and GELU' from h with one erf
#ifndef MDL_SAVE_PREACT
#define MDL_SAVE_PREACT 0
#endif
template <bool SAVE>
__device__ __forceinline__ void mlp_fwd_ct(const Mat& m1, const Mat& m2, const LNp& ln, CT* xr, bf16_t* sv_x, bf16_t* sv_g,
                                           bf16_t* sv_gp, bf16_t* sv_xh, float* sv_rs, const Ctx& c) {
  const int lane = c.lane;
  AFr W1, W2;
  loadA(W1, m1.fa, lane);
  loadA(W2, m2.fa, lane);
  const CT b1 = ld_vec(m1.b, lane), b2 = ld_vec(m2.b, lane), gam = ld_vec(ln.g, lane), bet = ld_vec(ln.b, lane);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      const CTr x = ct_pack(xr[k]);
      if (SAVE) st_g(sv_x, c.tok0, rt, c.NR, x, lane);
      CT h = b1;
      mm(h, W1, x);
      CTr gr;
      if (SAVE && MDL_SAVE_PREACT) {   // h for the backward; GELU of its bf16 value as the W2 operand
        const CTr hb = ct_pack(h);
        st_g(sv_g, c.tok0, rt, c.NR, hb, lane);
        h = ct_unpack(hb);
        gelu_ct(h);
        gr = ct_pack(h);
      } else if (SAVE) {   // GELU(h) (the W2 operand) and GELU'(h) for the backward, from one erf
        CT gp;
        gelu_ct_both(h, gp);
        gr = ct_pack(h);
        st_g(sv_g, c.tok0, rt, c.NR, gr, lane);
        st_g(sv_gp, c.tok0, rt, c.NR, ct_pack(gp), lane);
      } else {
        gelu_ct(h);
        gr = ct_pack(h);
      }
      CT mo = ct_add(b2, xr[k]), xh;
      mm(mo, W2, gr);
      const float rs = ln_fwd_ct(mo, xh, xr[k], gam, bet);
      if (SAVE) {
        st_g(sv_xh, c.tok0, rt, c.NR, ct_pack(xh), lane);
        st_tokf(sv_rs, rt, rs, c);
      }
    }
  }
  CP_MARK(23);
}

// ------------------------------------------------------------------------------------------ sublayers (backward)
// Backward sublayers run in passes with ONE weight matrix live at a time (the 8-wave backward keeps every wave
// under 256 registers): each pass leaves its per-tile products in this wave's own LDS rows (read back by the same
// lanes, so no barrier between passes) or in dx.
__device__ __forceinline__ void mlp_bwd_ct(const Mat& m1, const Mat& m2, const LNp& ln, CT* dx, const bf16_t* sv_x,
                                           const bf16_t* sv_g, const bf16_t* sv_gp, const bf16_t* sv_xh,
                                           const float* sv_rs, const Ctx& c, int vslot) {
  const int lane = c.lane;
  CTr gps[MAXRT];   // MDL_SAVE_PREACT: GELU'(h) from pass 1 for pass 2
  {   // pass 1: LN backward from the saved x-hat / rstd -> ds (dx) ; DA = dY of W2, XB = X of W2 (GELU(h))
    CT dlg, dlb;
    ct_zero(dlg);
    ct_zero(dlb);
    const CT gam = ld_vec(ln.g, lane);
    CTr xs[MAXRT], hs[MAXRT], xhs[MAXRT];
    float rsv[MAXRT];
    if (MDL_SAVE_PREACT) (void)sv_gp;
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {   // every saved-activation load of the wave issued up front
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        xs[k] = ld_g(sv_x, c.tok0, rt, c.NR, lane);
        hs[k] = ld_g(sv_g, c.tok0, rt, c.NR, lane);
        xhs[k] = ld_g(sv_xh, c.tok0, rt, c.NR, lane);
        rsv[k] = ld_tokf(sv_rs, rt, c);
      }
    }
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const bool ok = tok_ok(rt, c);
        CTr glr = hs[k];   // GELU(h): the forward's own W2 operand
        if (MDL_SAVE_PREACT) {   // hs = h: GELU(h) -> XB, GELU'(h) kept (packed) for pass 2
          CT hv = ct_unpack(hs[k]), gp;
          gelu_ct_both(hv, gp);
          glr = ct_pack(hv);
          gps[k] = ct_pack(gp);
        }
        CT ds;
        ln_bwd_ct(dx[k], ct_unpack(xhs[k]), rsv[k], gam, ok, ds, dlg, dlb);
        st_lds(c.DA, rt, ct_pack(ds), ok, lane);   // dY of W2
        st_lds(c.XB, rt, glr, ok, lane);           // X of W2
        st_lds(c.QB, rt, xs[k], ok, lane);         // X of W1
        dx[k] = ds;                                // residual path
      }
    }
    flush_vec(dlg, c.g(ln.dg), vslot, c);
    flush_vec(dlb, c.g(ln.db), vslot + 1, c);
  }
  {   // pass 2 (W2ᵀ): dg = W2ᵀ ds * GELU'(h) -> KB (dY of W1)
    AFr W2b;
    loadA(W2b, m2.ba, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const bool ok = tok_ok(rt, c);
        const CT gp = ct_unpack(MDL_SAVE_PREACT ? gps[k] : ld_g(sv_gp, c.tok0, rt, c.NR, lane));   // GELU'(h)
        CT dg;
        ct_zero(dg);
        mm(dg, W2b, ld_lds(c.DA, rt, lane));
#pragma unroll
        for (int i = 0; i < 4; ++i) dg.v[i] *= gp.v[i];   // padded rows: GELU' reads as zero, ds is finite
        st_lds(c.KB, rt, ct_pack(dg), ok, lane);
      }
    }
  }
  {   // pass 3 (W1ᵀ): dx += W1ᵀ dg
    AFr W1b;
    loadA(W1b, m1.ba, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) mm(dx[k], W1b, ld_lds(c.KB, rt, lane));
    }
  }
  __syncthreads();
  CP_MARK(2);
  wgrad64(c.DA, c.XB, m2, c);
  wgrad64(c.KB, c.QB, m1, c);
  __syncthreads();
  CP_MARK(3);
}

// recompute + store q / k / v of the saved input, attention backward, weight gradients; returns through dx (+=) the
// input gradient of the q / k / v projections.  Self: q-input = kv-input = x (sv_xin).  The attention output
// gradient dO must already be in DA.
__device__ __forceinline__ void self_attn_bwd_ct(const Mat* m, const LNp& ln, CT* dx, const bf16_t* sv_xin,
                                                 const bf16_t* sv_a, const bf16_t* sv_alo, const float* sv_lse,
                                                 const bf16_t* sv_xh, const float* sv_rs, bool causal,
                                                 const Ctx& c, int vslot) {
  const int lane = c.lane;
  const LseR lse = lse_fetch(sv_lse, c);   // consumed after the recompute phase (latency hidden by passes 1-2)
  CTr xin[MAXRT];
  {
    CT dlg, dlb;
    ct_zero(dlg);
    ct_zero(dlb);
    {   // pass 1: LN backward from the saved x-hat / rstd -> ds (dx) ; DQ = dY of Wp, XB = X of Wp
      const CT gam = ld_vec(ln.g, lane);
      CTr as[MAXRT], xhs[MAXRT];
      float rsv[MAXRT];
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          as[k] = ld_g(sv_a, c.tok0, rt, c.NR, lane);
          xin[k] = ld_g(sv_xin, c.tok0, rt, c.NR, lane);
          xhs[k] = ld_g(sv_xh, c.tok0, rt, c.NR, lane);
          rsv[k] = ld_tokf(sv_rs, rt, c);
        }
      }
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          const bool ok = tok_ok(rt, c);
          CT ds;
          ln_bwd_ct(dx[k], ct_unpack(xhs[k]), rsv[k], gam, ok, ds, dlg, dlb);
          st_lds(c.DQ, rt, ct_pack(ds), ok, lane);   // dY of Wp
          st_lds(c.XB, rt, as[k], ok, lane);         // X of Wp
          dx[k] = ds;                                // residual path
        }
      }
      flush_vec(dlg, c.g(ln.dg), vslot, c);
      flush_vec(dlb, c.g(ln.db), vslot + 1, c);
    }
    {   // pass 2 (Wpᵀ): dO = Wpᵀ ds -> DA; delta = rowsum(dO O) -> DEL (O = X of Wp, in XB)
      AFr Wpb;
      loadA(Wpb, m[3].ba, lane);
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          const CTr alo = MDL_SAVE_OLO ? ld_g(sv_alo, c.tok0, rt, c.NR, lane) : ct_zero_r();
          CT da;
          ct_zero(da);
          mm(da, Wpb, ld_lds(c.DQ, rt, lane));
          const bool ok = tok_ok(rt, c);
          const CTr dap = ct_pack(da);
          st_lds(c.DA, rt, dap, ok, lane);
          attn_delta_ct(ld_lds(c.XB, rt, lane), alo, dap, rt, ok, c);
        }
      }
    }
  }
  __syncthreads();
  CP_MARK(11);
  // q / k / v recompute first (global weight loads, LDS writes to QB / KB / VB only), then the Wp weight gradient
  // (reads DQ / XB): its fp32 atomics drain under the attention instead of stalling the next global loads behind
  // them (vmcnt counts them in order), and one barrier fewer.  XB takes x (the X of dWq/k/v) once every wave is past
  // dWp (after the query-pass barrier).
  proj3(m, 0, xin, c);
  wgrad64(c.DQ, c.XB, m[3], c);
  lse_store(lse, c);
  __syncthreads();
  CP_MARK(13);
  attn_bwd_q_ct(c.QB, c.KB, c.VB, c.DA, c.DQ, causal, c);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) st_lds(c.XB, rt, xin[k], tok_ok(rt, c), lane);   // X of dWq / dWk / dWv
  }
  __syncthreads();
  CP_MARK(14);
  attn_bwd_kv_ct(c.QB, c.KB, c.VB, c.DA, causal, c);
  __syncthreads();
  CP_MARK(15);
  proj3_bwd(m, 0, c.DQ, c.KB, c.VB, dx, dx, c);   // before the weight gradients: its weight loads do not queue
  CP_MARK(16);                                     // behind their atomics
  {
    const bf16_t* const ys[3] = {c.DQ, c.KB, c.VB};
    const Mat* const ms[3] = {&m[0], &m[1], &m[2]};
    wgrad64_shared_x<3>(ys, c.XB, ms, c);
  }
  __syncthreads();
  CP_MARK(17);
}

}  // namespace
