// Fused MAT training kernels for gfx950: whole-encoder forward / backward over tiles of whole sequences.
//
// Replaces the eager forward/backward of the reference's Encoder (mat_src/mat/algorithms/mat/algorithm/
// ma_transformer.py:72-92,119-154) used by TransformerPolicy.evaluate_actions / get_values
// (transformer_policy.py:158-217) inside MATTrainer.ppo_update (mat_trainer.py:96-156).
//
// One 256-thread workgroup owns SQ whole sequences (NR = SQ*L token rows, NT 16-row MFMA tiles; wave w owns tiles
// w, w+4, w+8).  Everything between two attention phases is wave-local: each wave computes full 64-column rows on
// v_mfma_f32_16x16x32_bf16 (weights streamed as pre-packed B fragments from L2), keeps the f32 residual stream in
// registers and runs bias / residual / LayerNorm / GELU on the accumulator layout (tile.h).  Attention over a
// sequence (L <= ~200 rows) runs on the VALU with packed bf16 dot products (v_dot2c_f32_bf16) and an online softmax.
// Only the attention phases and the weight-gradient GEMMs need workgroup barriers.
//
// Backward: activations saved by the forward (block inputs, attention outputs, MLP inputs / pre-GELU, per-row
// log-sum-exp) are reloaded; LayerNorm statistics, projections, q/k/v and P are recomputed.  Weight gradients
// dW = dYᵀ·X reduce over the token axis straight from token-major LDS tiles with ds_read_b64_tr_b16 transpose
// reads and are flushed with one fp32 atomic per element per workgroup.
#pragma once
#include "tile.h"
#include <cstdlib>

using namespace mdl;

namespace {

// Variant builds (mat_*_o2.hip) re-include the kernels with other tiling constants and a name suffix.
#ifndef MDL_VARIANT_SUFFIX
#define MDL_VARIANT_SUFFIX
#endif
#define MDL_CAT2(a, b) a##b
#define MDL_CAT(a, b) MDL_CAT2(a, b)
#define MDL_V(name) MDL_CAT(name, MDL_VARIANT_SUFFIX)
#ifndef MDL_MAXRT
#define MDL_MAXRT 3
#endif
#ifndef MDL_WGPC
#define MDL_WGPC 1   // resident workgroups per CU the kernels are sized for (LDS budget, register cap, grid)
#endif
// Optional section profiler (-DMDL_TRAIN_PROF): thread 0 of workgroup 0 accumulates core-clock cycles per code
// section into g_tprof (read back by mdl_*_prof_read); each mark costs one global read-modify-write.
#ifdef MDL_TRAIN_PROF
__device__ unsigned long long g_tprof[32];
#define TP_DECL() bool tp_on_ = blockIdx.x == 0 && threadIdx.x == 0; unsigned long long tp_t_ = clock64()
#define TP_MARK(k) do { if (tp_on_) { const unsigned long long t_ = clock64(); g_tprof[k] += t_ - tp_t_; tp_t_ = t_; } } while (0)
#else
#define TP_DECL() do { } while (0)
#define TP_MARK(k) do { } while (0)
#endif

#ifndef MDL_NW
#define MDL_NW 4     // waves per workgroup (the round-2 backward translation units build with 8)
#endif
constexpr int NW = MDL_NW;
constexpr int NTHR = 64 * NW;
constexpr int MAXRT = MDL_MAXRT;  // row tiles per wave (NT <= NW * MAXRT; wave w owns tiles w, w + NW, ...)
constexpr int WGPC = MDL_WGPC;
constexpr int LDS_BUDGET = 160 * 1024 / WGPC;

// fw / bw: B fragments of W / Wᵀ (row-layout tiles); fa / ba: A fragments of W / Wᵀ with the permuted k order of
// the token-on-lane tiles (mat_train_ct.h)
struct Mat { const bf16_t* fw; const bf16_t* bw; const float* b; float* dW; float* db; const bf16_t* fa; const bf16_t* ba; };
struct LNp { const float* g; const float* b; float* dg; float* db; };
struct Blk { Mat m[10]; LNp ln[3]; };
struct Sv { bf16_t* xin; bf16_t* a1; float* lse1; bf16_t* x1; bf16_t* a2; float* lse2; bf16_t* x2; bf16_t* h; };

struct EncP {
  int Bs, L, od, SQ, NRP, n_obj;
  const float* obs;
  const float *lno_g, *lno_b, *we, *be, *ln0_g, *ln0_b;
  float *d_lno_g, *d_lno_b, *d_we, *d_be, *d_ln0_g, *d_ln0_b;
  Blk blk[3];
  Mat h1;
  LNp lnh;
  const float* wh2;
  const float* bh2;
  float* d_wh2;
  float* rep;
  float* v;
  Sv sv[3];
  const float* drep;
  const float* dv;
  long long g_delta, g_stride;   // dW workspace: copy k of a gradient lives at grad + g_delta + k * g_stride
  int g_copies;                  // 0: atomics straight into the gradients
  float* d_bh2;                  // value-head bias gradient Σ dv (round-2 backward; null: summed by the caller)
};

struct DecP {
  int Bs, L, A, SQ, NRP, n_disc;
  const float* act;      // [tok] stored action (discrete index, or the continuous value for continuous agents)
  const float* ava;      // [tok][A] availability (or null)
  const float* wa;       // action_encoder weight [64][A+1]
  float* d_wa;
  const float *lnd_g, *lnd_b;
  float *d_lnd_g, *d_lnd_b;
  Blk blk[3];
  Mat h1;
  LNp lnh;
  const float* wh2;      // [A][64]
  const float* bh2;      // [A]
  float* d_wh2;
  float* d_bh2;
  const float* stdv;     // [A] sigmoid(log_std) * 0.5
  const float* log_std;  // [A]
  float* d_log_std;
  const float* rep;      // [tok][64] encoder output
  float* logp;           // [tok]
  float* ent;            // [tok]
  Sv sv[3];
  const float* dlogp;
  const float* dent;
  float* drep;           // [tok][64] accumulated (pre-zeroed)
  bf16_t* sv_head;       // [tok][64] head input (last block output)
  long long g_delta, g_stride;
  int g_copies;
  // continuous action type (MA-MuJoCo, transformer_act.py:192-232): act / logp / ent / dlogp / dent are
  // [tok][A], the action embedding is Linear(A, 64) with bias (wa = [64][A], ba = [64]) on the previous agent's action
  int cont;
  const float* ba;
  float* d_ba;
};

struct Ctx {
  int tid, lane, wave, L, nseq, NR, NT, NRP, tok0;
  ptrdiff_t gofs;   // gradient-copy offset (floats): this block's slice of the 8-way dW workspace, 0 = direct
  __device__ __forceinline__ float* g(float* p) const { return p ? p + gofs : p; }
  bf16_t *QB, *KB, *VB, *DA, *DQ, *XB;
  float *LSE, *DEL;
};

typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2v, a), __builtin_bit_cast(bf2v, b), c, false);
}
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

__device__ __forceinline__ void ld_head_u(const bf16_t* buf, int row, int h, uint32_t* o) {
#pragma unroll
  for (int lc = 0; lc < 4; ++lc) {
    const uint4 v = *(const uint4*)(buf + (row << 6) + ((((4 * h + lc) ^ ((row >> 1) & 7))) << 3));
    o[4 * lc + 0] = v.x; o[4 * lc + 1] = v.y; o[4 * lc + 2] = v.z; o[4 * lc + 3] = v.w;
  }
}
__device__ __forceinline__ void st_head_f(bf16_t* buf, int row, int h, const float* v) {
#pragma unroll
  for (int lc = 0; lc < 4; ++lc) {
    uint4 u;
    u.x = (uint32_t)f2bf(v[8 * lc + 0]) | ((uint32_t)f2bf(v[8 * lc + 1]) << 16);
    u.y = (uint32_t)f2bf(v[8 * lc + 2]) | ((uint32_t)f2bf(v[8 * lc + 3]) << 16);
    u.z = (uint32_t)f2bf(v[8 * lc + 4]) | ((uint32_t)f2bf(v[8 * lc + 5]) << 16);
    u.w = (uint32_t)f2bf(v[8 * lc + 6]) | ((uint32_t)f2bf(v[8 * lc + 7]) << 16);
    *(uint4*)(buf + (row << 6) + ((((4 * h + lc) ^ ((row >> 1) & 7))) << 3)) = u;
  }
}

constexpr float ATT_SCALE = 0.17677669529663687f;  // 1/sqrt(32)

#ifdef MDL_ATTN_VALU
#include "attn_valu.h"
#else
// ------------------------------------------------------------------------------------------ attention (MFMA)
// Sequence-block-diagonal attention over the workgroup's packed rows (rows of sequence s = [sL, sL+L)), on
// v_mfma_f32_16x16x32_bf16 with the head dimension (32) as one K step.  Work items = (16-row tile, head), one per
// wave at a time; keys / queries are visited in 32-row chunks aligned to 32 (always inside the NRP-row buffers)
// and masked to the item's sequences (+ causal).
//
// Layout trick: the score tile is computed TRANSPOSED (Sᵀ = K·Qᵀ, A operand = K rows in the permuted order
// pi_t(m) = 8(m>>2) + 4t + (m&3) for the two 16-key halves t of a chunk).  The C layout then leaves lane (g, c)
// holding S[query c][key kb + 8g + j] for j = 4t + r — exactly the A-operand layout of the following P·V MFMA,
// whose B operand (V, K along the token axis) comes from ds_read_b64_tr_b16 transposed reads (ld_frag_T).
// No LDS round trip for P / dS.  LSE / delta live in LDS as [head][row] (NRP rows per head).
__device__ __forceinline__ int pi_row(int t, int m) { return 8 * (m >> 2) + 4 * t + (m & 3); }

__device__ __forceinline__ bf16x8 pack8(const float* x) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (short)f2bf(x[j]);
  return f;
}

// x ≈ hi + lo with both halves bf16 (≈16 mantissa bits): dS has rows summing to zero and feeds bias gradients,
// where a single bf16 rounding of dS leaves a visible bias; two MFMAs (hi, lo) keep it at fp32-like accuracy.
__device__ __forceinline__ void pack8_split(const float* x, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint16_t h = f2bf(x[j]);
    hi[j] = (short)h;
    lo[j] = (short)f2bf(x[j] - bf2f(h));
  }
}

// scores of one 32-key chunk, transposed: out[j] = S[q][kb + 8g + j] (q = this lane's query column)
__device__ __forceinline__ void score_chunk_T(const bf16_t* K, int kb, int h, bf16x8 qB, float* out, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const bf16x8 a = lda_tm(K, kb + pi_row(t, c16), 4 * h + g);
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qB, z, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[4 * t + i] = r[i];
  }
}

struct SeqSpan { int lo, hi; };   // [lo, hi) rows of the sequences a 16-row tile touches, 32-aligned chunk bounds

__device__ __forceinline__ SeqSpan tile_span(int t16, const Ctx& c, bool causal_hi) {
  const int r0 = t16 * 16, r1 = min(r0 + 15, c.NR - 1);
  const int lo = (r0 / c.L) * c.L;
  const int hi = causal_hi ? r1 + 1 : min((r1 / c.L + 1) * c.L, c.NR);
  return SeqSpan{lo & ~31, (hi + 31) & ~31};
}

// forward: O (may alias Q) = softmax(scale Q Kᵀ) V per head; lse_g (global [tok][2]) written if non-null
__device__ __forceinline__ void attn_fwd(const bf16_t* Q, const bf16_t* K, const bf16_t* V, bf16_t* O, bool causal, float* lse_g,
                                         const Ctx& c) {
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  for (int item = c.wave; item < 2 * c.NT; item += NW) {
    const int qt = item >> 1, h = item & 1;
    const int q = qt * 16 + c16;
    const bool qv = q < c.NR;
    const int qs = (q / c.L) * c.L, qe = causal ? q + 1 : min(qs + c.L, c.NR);
    const SeqSpan sp = tile_span(qt, c, causal);
    const bf16x8 qB = lda_tm(Q, q, 4 * h + g);
    // pass 1: per-lane online max / sum over its 8 keys per chunk, then merge the 4 lane groups
    float m = -INFINITY, l = 0.f;
    for (int kb = sp.lo; kb < sp.hi; kb += 32) {
      float sc[8];
      score_chunk_T(K, kb, h, qB, sc, lane);
      float cm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kb + 8 * g + j;
        sc[j] = (qv && k >= qs && k < qe) ? sc[j] * ATT_SCALE : -INFINITY;
        cm = fmaxf(cm, sc[j]);
      }
      const float nm = fmaxf(m, cm);
      if (nm > -INFINITY) {
        float add = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) add += __expf(sc[j] - nm);
        l = l * __expf(m - nm) + add;
        m = nm;
      }
    }
#pragma unroll
    for (int x = 16; x <= 32; x <<= 1) {
      const float om = x == 16 ? xor16_partner(m) : xor32_partner(m);
      const float ol = x == 16 ? xor16_partner(l) : xor32_partner(l);
      const float nm = fmaxf(m, om);
      l = (nm > -INFINITY) ? l * __expf(m - nm) + ol * __expf(om - nm) : 0.f;
      m = nm;
    }
    const float lse = l > 0.f ? m + __logf(l) : 0.f;
    // pass 2: P = exp(S - lse) (already normalised) → O = P V on MFMA
    f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int kb = sp.lo; kb < sp.hi; kb += 32) {
      float sc[8];
      score_chunk_T(K, kb, h, qB, sc, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kb + 8 * g + j;
        sc[j] = (qv && k >= qs && k < qe) ? __expf(sc[j] * ATT_SCALE - lse) : 0.f;
      }
      bf16x8 pah, pal;
      pack8_split(sc, pah, pal);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const bf16x8 vf = ld_frag_T(V, kb, 32 * h + 16 * dt, lane);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pah, vf, o[dt], 0, 0, 0);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pal, vf, o[dt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = qt * 16 + 4 * g + r;
        O[tmo(row, 32 * h + 16 * dt + c16)] = f2bf(row < c.NR ? o[dt][r] : 0.f);
      }
    if (lse_g && g == 0 && qv) lse_g[(size_t)(c.tok0 + q) * 2 + h] = lse;
  }
}

// backward pass 1 (by query tile): delta_q = sum_k P dP, dS = P (dP - delta), dQ = scale dS K  (→ DQ)
__device__ __forceinline__ void attn_bwd_q(const bf16_t* Q, const bf16_t* K, const bf16_t* V, const bf16_t* DA, bf16_t* DQ,
                                           bool causal, const Ctx& c) {
#ifdef MDL_ABLATE_ATTN
  return;
#endif
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  for (int item = c.wave; item < 2 * c.NT; item += NW) {
    const int qt = item >> 1, h = item & 1;
    const int q = qt * 16 + c16;
    const bool qv = q < c.NR;
    const int qs = (q / c.L) * c.L, qe = causal ? q + 1 : min(qs + c.L, c.NR);
    const SeqSpan sp = tile_span(qt, c, causal);
    const bf16x8 qB = lda_tm(Q, q, 4 * h + g), dB = lda_tm(DA, q, 4 * h + g);
    const float lse = c.LSE[h * c.NRP + q];
    float delta = 0.f;
    for (int kb = sp.lo; kb < sp.hi; kb += 32) {
      float sc[8], dp[8];
      score_chunk_T(K, kb, h, qB, sc, lane);
      score_chunk_T(V, kb, h, dB, dp, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kb + 8 * g + j;
        if (qv && k >= qs && k < qe) delta += __expf(sc[j] * ATT_SCALE - lse) * dp[j];
      }
    }
    delta = cross_row_sum(delta);
    f32x4 dq[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int kb = sp.lo; kb < sp.hi; kb += 32) {
      float sc[8], dp[8];
      score_chunk_T(K, kb, h, qB, sc, lane);
      score_chunk_T(V, kb, h, dB, dp, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kb + 8 * g + j;
        sc[j] = (qv && k >= qs && k < qe) ? __expf(sc[j] * ATT_SCALE - lse) * (dp[j] - delta) : 0.f;
      }
      bf16x8 dah, dal;
      pack8_split(sc, dah, dal);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const bf16x8 kf = ld_frag_T(K, kb, 32 * h + 16 * dt, lane);
        dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dah, kf, dq[dt], 0, 0, 0);
        dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dal, kf, dq[dt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = qt * 16 + 4 * g + r;
        DQ[tmo(row, 32 * h + 16 * dt + c16)] = f2bf(row < c.NR ? dq[dt][r] * ATT_SCALE : 0.f);
      }
    if (g == 0) c.DEL[h * c.NRP + q] = qv ? delta : 0.f;
  }
}

// backward pass 2 (by key tile): dV = Pᵀ dO, dK = scale dSᵀ Q, written in place over K / V (head columns)
__device__ __forceinline__ void attn_bwd_kv(const bf16_t* Q, bf16_t* K, bf16_t* V, const bf16_t* DA, bool causal, const Ctx& c) {
#ifdef MDL_ABLATE_ATTN
  return;
#endif
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  for (int item = c.wave; item < 2 * c.NT; item += NW) {
    const int kt = item >> 1, h = item & 1;
    const int k = kt * 16 + c16;
    const bool kv = k < c.NR;
    const int ks = (k / c.L) * c.L, ke = min(ks + c.L, c.NR);
    const int qlo = causal ? k : ks;   // queries that see key k
    SeqSpan sp = tile_span(kt, c, false);
    if (causal) sp.lo = (kt * 16) & ~31;
    const bf16x8 kB = lda_tm(K, k, 4 * h + g), vB = lda_tm(V, k, 4 * h + g);
    f32x4 dk[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, dv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int qb = sp.lo; qb < sp.hi; qb += 32) {
      float sc[8], dp[8];
      score_chunk_T(Q, qb, h, kB, sc, lane);    // sc[j] = S[query qb + 8g + j][key k]
      score_chunk_T(DA, qb, h, vB, dp, lane);   // dp[j] = dP[query][key k]
      const float4* lp = (const float4*)(c.LSE + h * c.NRP + qb + 8 * g);
      const float4* dl = (const float4*)(c.DEL + h * c.NRP + qb + 8 * g);
      const float4 l0 = lp[0], l1 = lp[1], d0 = dl[0], d1 = dl[1];
      const float lsev[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
      const float delv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
      float p[8], ds[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qq = qb + 8 * g + j;
        const bool ok = kv && qq >= qlo && qq < ke;
        p[j] = ok ? __expf(sc[j] * ATT_SCALE - lsev[j]) : 0.f;
        ds[j] = ok ? p[j] * (dp[j] - delv[j]) : 0.f;
      }
      bf16x8 pah, pal, dsh, dsl;
      pack8_split(p, pah, pal);
      pack8_split(ds, dsh, dsl);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const bf16x8 of = ld_frag_T(DA, qb, 32 * h + 16 * dt, lane);
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pah, of, dv[dt], 0, 0, 0);
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pal, of, dv[dt], 0, 0, 0);
        const bf16x8 qf = ld_frag_T(Q, qb, 32 * h + 16 * dt, lane);
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsh, qf, dk[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsl, qf, dk[dt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = kt * 16 + 4 * g + r;
        const bool ok = row < c.NR;
        K[tmo(row, 32 * h + 16 * dt + c16)] = f2bf(ok ? dk[dt][r] * ATT_SCALE : 0.f);
        V[tmo(row, 32 * h + 16 * dt + c16)] = f2bf(ok ? dv[dt][r] : 0.f);
      }
  }
}

#endif  // MDL_ATTN_VALU

// saved per-row log-sum-exp ([tok][2] global) -> LDS [head][NRP]
__device__ __forceinline__ void load_lse(const float* sv_lse, const Ctx& c) {
  for (int i = c.tid; i < 2 * c.NRP; i += NTHR) {
    const int h = i / c.NRP, row = i - h * c.NRP;
    c.LSE[i] = row < c.NR ? sv_lse[(size_t)(c.tok0 + row) * 2 + h] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------ helpers
// copy the valid rows of row tile rt of a swizzled LDS buffer to a plain global [tok][64] bf16 tensor
__device__ __forceinline__ void tile2g(bf16_t* dst, const bf16_t* buf, int rt, const Ctx& c) {
  for (int i = c.lane; i < 16 * 8; i += 64) {
    const int row = rt * 16 + (i >> 3), lc = i & 7;
    if (row < c.NR)
      *(uint4*)(dst + (size_t)(c.tok0 + row) * 64 + lc * 8) =
          *(const uint4*)(buf + (row << 6) + ((lc ^ ((row >> 1) & 7)) << 3));
  }
}

__device__ __forceinline__ void g2tile(bf16_t* buf, const bf16_t* src, int rt, const Ctx& c) {
  for (int i = c.lane; i < 16 * 8; i += 64) {
    const int row = rt * 16 + (i >> 3), lc = i & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < c.NR) v = *(const uint4*)(src + (size_t)(c.tok0 + row) * 64 + lc * 8);
    *(uint4*)(buf + (row << 6) + ((lc ^ ((row >> 1) & 7)) << 3)) = v;
  }
}

// all of this wave's row tiles of one or two saved activations -> LDS, every global load issued before the first
// LDS store (one latency instead of one per tile); rows beyond NR are zero-filled.
__device__ __forceinline__ void g2tiles(bf16_t* buf0, const bf16_t* src0, bf16_t* buf1, const bf16_t* src1,
                                        const Ctx& c) {
  uint4 v0[MAXRT][2], v1[MAXRT][2];
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = c.lane + 64 * ii, row = rt * 16 + (i >> 3), lc = i & 7;
      const bool ok = rt < c.NT && row < c.NR;
      const size_t off = (size_t)(c.tok0 + row) * 64 + lc * 8;
      v0[k][ii] = ok ? *(const uint4*)(src0 + off) : make_uint4(0, 0, 0, 0);
      v1[k][ii] = (ok && src1) ? *(const uint4*)(src1 + off) : make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = c.lane + 64 * ii, row = rt * 16 + (i >> 3), lc = i & 7;
        const int o = (row << 6) + ((lc ^ ((row >> 1) & 7)) << 3);
        *(uint4*)(buf0 + o) = v0[k][ii];
        if (src1) *(uint4*)(buf1 + o) = v1[k][ii];
      }
    }
  }
  wave_lds_sync();
}

// load a saved bf16 activation tile as an RT via LDS staging (vector global loads; buf rows of tile rt are
// overwritten and keep the activation, usable as a GEMM / weight-gradient operand afterwards)
__device__ __forceinline__ void ld_saved(bf16_t* buf, const bf16_t* src, int rt, RT& t, const Ctx& c) {
  g2tile(buf, src, rt, c);
  wave_lds_sync();
  ld_tm(buf, rt, t, c.lane);
}

__device__ __forceinline__ void gelu_rt(RT& t) {
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) t.v[ct][r] = gelu_erf(t.v[ct][r]);
}

__device__ __forceinline__ void zero_lds(char* smem, size_t bytes, int tid) {
  for (size_t i = (size_t)tid * 16; i < bytes; i += NTHR * 16) *(uint4*)(smem + i) = make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ void flush_ln(f32x4 dg, f32x4 db, const LNp& ln, const Ctx& c) {
  flush_cols(dg, c.g(ln.dg), c.lane);
  flush_cols(db, c.g(ln.db), c.lane);
}

// ------------------------------------------------------------------------------------------ sublayers (forward)
template <bool SAVE>
__device__ __forceinline__ void attn_self_fwd(const Mat* m, const LNp& ln, RT* xr, const Sv& sv, bool causal, bf16_t* sv_xin,
                              bf16_t* sv_a, float* sv_lse, const Ctx& c) {
  const int lane = c.lane;
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      st_tm_m(c.XB, rt, xr[k], row_mask(rt, c.NR, lane), lane);
      if (SAVE) { wave_lds_sync(); tile2g(sv_xin, c.XB, rt, c); }
    }
  }
  wave_lds_sync();
  bf16_t* outs[3] = {c.QB, c.KB, c.VB};
#pragma unroll
  for (int mi = 0; mi < 3; ++mi) {
    BFr B;
    loadB(B, m[mi].fw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        RT t;
        gemm_rt(t, c.XB, rt, B, lane, false);
        add_bias(t, m[mi].b, lane);
        st_tm_m(outs[mi], rt, t, row_mask(rt, c.NR, lane), lane);
      }
    }
  }
  __syncthreads();
  attn_fwd(c.QB, c.KB, c.VB, c.QB, causal, SAVE ? sv_lse : nullptr, c);
  __syncthreads();
  BFr B;
  loadB(B, m[3].fw, lane);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      if (SAVE) tile2g(sv_a, c.QB, rt, c);
      RT t, xh, y;
      gemm_rt(t, c.QB, rt, B, lane, false);
      add_bias(t, m[3].b, lane);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) t.v[ct] += xr[k].v[ct];
      f32x4 mu, rs;
      ln_fwd(t, xh, y, mu, rs, ln.g, ln.b, lane);
      xr[k] = y;
    }
  }
}

template <bool SAVE>
__device__ __forceinline__ void mlp_fwd(const Mat& m1, const Mat& m2, const LNp& ln, RT* xr, bf16_t* sv_x, bf16_t* sv_h,
                        const Ctx& c) {
  const int lane = c.lane;
  BFr B1, B2;
  loadB(B1, m1.fw, lane);
  loadB(B2, m2.fw, lane);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      const f32x4 vm = row_mask(rt, c.NR, lane);
      st_tm_m(c.XB, rt, xr[k], vm, lane);
      wave_lds_sync();
      if (SAVE) tile2g(sv_x, c.XB, rt, c);
      RT h;
      gemm_rt(h, c.XB, rt, B1, lane, false);
      add_bias(h, m1.b, lane);
      if (SAVE) {
        st_tm_m(c.XB, rt, h, vm, lane);
        wave_lds_sync();
        tile2g(sv_h, c.XB, rt, c);
      }
      gelu_rt(h);
      st_tm_m(c.XB, rt, h, vm, lane);
      wave_lds_sync();
      RT mo, xh, y;
      gemm_rt(mo, c.XB, rt, B2, lane, false);
      add_bias(mo, m2.b, lane);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) mo.v[ct] += xr[k].v[ct];
      f32x4 mu, rs;
      ln_fwd(mo, xh, y, mu, rs, ln.g, ln.b, lane);
      xr[k] = y;
    }
  }
}

// obs embedding (VALU; obs_dim <= 16): x0 = LN0(GELU(W_e · LN_obs(obs) + b_e))  — ma_transformer.py:133-134,151
// The LN_obs rows of the wave's current tile are staged in a per-wave LDS scratch (16 rows x [oh(16) | ohat(16)]
// f32 = 2 KB, aliasing the QB buffer, which is free before the first / after the last attention) instead of
// registers: 4 rows x 32 floats per lane kept the encoder backward above 256 VGPRs (scratch spills).
constexpr int ES_FLOATS = 16 * 32;
__device__ __forceinline__ float* emb_scratch(const Ctx& c) { return (float*)c.QB + c.wave * ES_FLOATS; }

// lanes 0..15 each normalise one row of the tile (obs_dim <= 16) into the scratch; rows >= NR are zero
__device__ __forceinline__ void embed_stage(const EncP& p, int rt, float* ES, const Ctx& c) {
  const int lane = c.lane, od = p.od;
  if (lane < 16) {
    const int row = rt * 16 + lane;
    const bool valid = row < c.NR;
    const size_t tok = (size_t)(c.tok0 + (valid ? row : 0));
    // all od loads issued before any is used (clamped in-bounds indices, selected after): a per-k branch
    // serialised the HBM latency od times (the section profiler put this staging at 20 % of mat_enc_bwd)
    float o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = p.obs[tok * od + (k < od ? k : 0)];
    float mean = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) { o[k] = (valid && k < od) ? o[k] : 0.f; mean += o[k]; }
    mean /= (float)od;
    float var = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) if (k < od) { const float d = o[k] - mean; var += d * d; }
    const float rstd = rsqrtf(var / (float)od + 1e-5f);
    float* e = ES + lane * 32;
#pragma unroll
    for (int k = 0; k < 16; k += 4) {
      f32x4 oh, hat;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k + j;
        hat[j] = (valid && kk < od) ? (o[kk] - mean) * rstd : 0.f;
        oh[j] = (valid && kk < od) ? hat[j] * p.lno_g[kk] + p.lno_b[kk] : 0.f;
      }
      *(f32x4*)(e + k) = oh;
      *(f32x4*)(e + 16 + k) = hat;
    }
  }
  wave_lds_sync();
}

// pre = W_e · LN_obs(obs) + b_e for the tile (LN_obs rows read back from the scratch, broadcast per lane group)
__device__ __forceinline__ void embed_pre(const EncP& p, int rt, RT& pre, const float* ES, const Ctx& c) {
  const int g = c.lane >> 4, c16 = c.lane & 15;
  const int nk = (p.od + 3) >> 2;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int col = 16 * ct + c16;
#pragma unroll
    for (int r = 0; r < 4; ++r) pre.v[ct][r] = p.be[col];
  }
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) {
    if (k4 < nk) {
      f32x4 x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = *(const f32x4*)(ES + (4 * g + r) * 32 + 4 * k4);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int col = 16 * ct + c16;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = 4 * k4 + j;
          const float w = k < p.od ? p.we[col * p.od + k] : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) pre.v[ct][r] += w * x[r][j];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ sublayers (backward)
__device__ __forceinline__ void mlp_bwd(const Mat& m1, const Mat& m2, const LNp& ln, RT* dx, const bf16_t* sv_x, const bf16_t* sv_h,
                        const Ctx& c) {
  const int lane = c.lane;
  f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0}, db1 = {0, 0, 0, 0}, db2 = {0, 0, 0, 0};
  {
    BFr B2f, B2b, B1b;
    loadB(B2f, m2.fw, lane);
    loadB(B2b, m2.bw, lane);
    loadB(B1b, m1.bw, lane);
    g2tiles(c.QB, sv_x, c.XB, sv_h, c);     // QB rows = X of dW1, XB = pre-GELU h
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT x, h, gl;
        ld_tm(c.QB, rt, x, lane);
        ld_tm(c.XB, rt, h, lane);
        gl = h;
        gelu_rt(gl);
        st_tm_m(c.XB, rt, gl, vm, lane);   // X of dW2
        wave_lds_sync();
        RT mo, xh, y, ds;
        gemm_rt(mo, c.XB, rt, B2f, lane, false);
        add_bias(mo, m2.b, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) mo.v[ct] += x.v[ct];
        f32x4 mu, rs;
        ln_fwd(mo, xh, y, mu, rs, ln.g, ln.b, lane);
        ln_bwd(dx[k], xh, rs, ln.g, ds, dlg, dlb, vm, lane);
        colsum_acc(ds, db2, vm);
        st_tm_m(c.DA, rt, ds, vm, lane);   // dY of dW2
        wave_lds_sync();
        RT dg;
        gemm_rt(dg, c.DA, rt, B2b, lane, false);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) dg.v[ct][r] *= gelu_erf_grad(h.v[ct][r]) * vm[r];
        colsum_acc(dg, db1, vm);
        st_tm_m(c.KB, rt, dg, vm, lane);   // dY of dW1
        wave_lds_sync();
        RT t;
        gemm_rt(t, c.KB, rt, B1b, lane, false);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) dx[k].v[ct] = ds.v[ct] + t.v[ct];
      }
    }
  }
  flush_ln(dlg, dlb, ln, c);
  flush_cols(db1, c.g(m1.db), lane);
  flush_cols(db2, c.g(m2.db), lane);
  __syncthreads();
  wgrad_tm(c.DA, c.XB, c.NRP, c.g(m2.dW), c.wave, lane);
  wgrad_tm(c.KB, c.QB, c.NRP, c.g(m1.dW), c.wave, lane);
  __syncthreads();
}

// attention sublayer backward: out = LN(res + proj(attn(q(qin), k(kvin), v(kvin))))
// self: qin = kvin = res = saved block input (sv_xin);  grads w.r.t. the input accumulate into dx.
__device__ __forceinline__ void attn_self_bwd(const Mat* m, const LNp& ln, RT* dx, const bf16_t* sv_xin, const bf16_t* sv_a,
                              const float* sv_lse, bool causal, const Ctx& c) {
  const int lane = c.lane;
  TP_DECL();
  f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0}, dbp = {0, 0, 0, 0};
  {
    BFr Bpf, Bpb;
    loadB(Bpf, m[3].fw, lane);
    loadB(Bpb, m[3].bw, lane);
    g2tiles(c.XB, sv_a, c.DA, sv_xin, c);  // XB = attention output (X of dWp), DA = block input
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT a, xin;
        ld_tm(c.DA, rt, xin, lane);
        RT s, xh, y, ds;
        gemm_rt(s, c.XB, rt, Bpf, lane, false);
        add_bias(s, m[3].b, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) s.v[ct] += xin.v[ct];
        f32x4 mu, rs;
        ln_fwd(s, xh, y, mu, rs, ln.g, ln.b, lane);
        ln_bwd(dx[k], xh, rs, ln.g, ds, dlg, dlb, vm, lane);
        colsum_acc(ds, dbp, vm);
        st_tm_m(c.DQ, rt, ds, vm, lane);   // dY of dWp (= d proj output)
        wave_lds_sync();
        RT da;
        gemm_rt(da, c.DQ, rt, Bpb, lane, false);
        st_tm_m(c.DA, rt, da, vm, lane);
        dx[k] = ds;                          // residual path
      }
    }
  }
  flush_ln(dlg, dlb, ln, c);
  flush_cols(dbp, c.g(m[3].db), lane);
  __syncthreads();
  TP_MARK(0);
  wgrad_tm(c.DQ, c.XB, c.NRP, c.g(m[3].dW), c.wave, lane);
  __syncthreads();
  TP_MARK(1);
  // recompute q, k, v from the saved input (whole tile, cooperative copy)
  g2lds_rows(c.XB, sv_xin, c.tok0, c.NR, c.NT * 16, c.tid);
  load_lse(sv_lse, c);
  __syncthreads();
  {
    bf16_t* outs[3] = {c.QB, c.KB, c.VB};
#pragma unroll
    for (int mi = 0; mi < 3; ++mi) {
      BFr B;
      loadB(B, m[mi].fw, lane);
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          RT t;
          gemm_rt(t, c.XB, rt, B, lane, false);
          add_bias(t, m[mi].b, lane);
          st_tm_m(outs[mi], rt, t, row_mask(rt, c.NR, lane), lane);
        }
      }
    }
  }
  __syncthreads();
  TP_MARK(2);
  attn_bwd_q(c.QB, c.KB, c.VB, c.DA, c.DQ, causal, c);
  __syncthreads();
  TP_MARK(3);
  attn_bwd_kv(c.QB, c.KB, c.VB, c.DA, causal, c);
  __syncthreads();
  TP_MARK(4);
  wgrad_tm(c.DQ, c.XB, c.NRP, c.g(m[0].dW), c.wave, lane);
  wgrad_tm(c.KB, c.XB, c.NRP, c.g(m[1].dW), c.wave, lane);
  wgrad_tm(c.VB, c.XB, c.NRP, c.g(m[2].dW), c.wave, lane);
  TP_MARK(5);
  const bf16_t* dsrc[3] = {c.DQ, c.KB, c.VB};
#pragma unroll
  for (int mi = 0; mi < 3; ++mi) {
    BFr B;
    loadB(B, m[mi].bw, lane);
    f32x4 dbb = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT g, t;
        ld_tm(dsrc[mi], rt, g, lane);
        colsum_acc(g, dbb, vm);
        gemm_rt(t, dsrc[mi], rt, B, lane, false);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) dx[k].v[ct] += t.v[ct];
      }
    }
    flush_cols(dbb, c.g(m[mi].db), lane);
  }
  __syncthreads();
  TP_MARK(6);
}

// ------------------------------------------------------------------------------------------ context
template <typename PT>
__device__ __forceinline__ Ctx make_ctx(const PT& p, char* smem, int seq0, int nseq) {
  Ctx c;
  c.tid = threadIdx.x;
  asm volatile("" : "+v"(c.tid));   // opaque per tile: lane-derived addresses are not hoisted out of the tile loop
  c.lane = c.tid & 63;
  c.wave = __builtin_amdgcn_readfirstlane(c.tid >> 6);
  c.L = p.L;
  c.nseq = nseq;
  c.NR = c.nseq * p.L;
  c.NT = (c.NR + 15) >> 4;
  c.NRP = p.NRP;
  c.tok0 = seq0 * p.L;
  // spread the fp32 weight-gradient atomics over g_copies copies (blockIdx % 8 ~ the XCD the block runs on):
  // 8x fewer adders per address than every workgroup hitting the same 16 KB matrix
  c.gofs = p.g_copies > 0 ? (ptrdiff_t)p.g_delta + (ptrdiff_t)(blockIdx.x % p.g_copies) * (ptrdiff_t)p.g_stride : 0;
  const size_t bs = (size_t)p.NRP * 64;
  bf16_t* base = (bf16_t*)smem;
  c.QB = base; c.KB = base + bs; c.VB = base + 2 * bs; c.DA = base + 3 * bs; c.DQ = base + 4 * bs; c.XB = base + 5 * bs;
  c.LSE = (float*)(base + 6 * bs);
  c.DEL = c.LSE + 2 * p.NRP;
  return c;
}

}  // namespace

__host__ __device__ inline size_t mat_train_lds_bytes(int NRP, int SQ, int L) {
  const size_t aux = (size_t)NRP * 2 * 4 * 2;   // LSE / delta [2][NRP] f32 (also the decoder's embedding-grad scratch)
  return (size_t)NRP * 64 * 2 * 6 + (aux < 9 * 64 * 4 ? 9 * 64 * 4 : aux);
}


// Persistent, balanced tiling: workgroup w owns the contiguous sequence range [Bs*w/G, Bs*(w+1)/G) and walks it in
// near-equal chunks of <= SQ sequences.  With G = #CUs the makespan is ceil(Bs/G) sequences per CU instead of
// ceil(Bs/SQ/G) full tiles (640 tiles of 5 on 256 CUs = 3 rounds of 5 -> 13 sequences per CU).
#define FOR_TILES(p, CALL)                                                                         \
  {                                                                                                \
    const long long G_ = gridDim.x, w_ = blockIdx.x;                                               \
    const int lo_ = (int)((long long)(p).Bs * w_ / G_), hi_ = (int)((long long)(p).Bs * (w_ + 1) / G_); \
    const int n_ = hi_ - lo_, nch_ = (n_ + (p).SQ - 1) / (p).SQ;                                   \
    for (int ch_ = 0; ch_ < nch_; ++ch_) {                                                         \
      const int s0 = lo_ + (int)((long long)n_ * ch_ / nch_);                                      \
      const int ns = lo_ + (int)((long long)n_ * (ch_ + 1) / nch_) - s0;                           \
      if (ch_) __syncthreads();                                                                    \
      CALL;                                                                                        \
    }                                                                                              \
  }

static int n_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    const char* e = getenv("MAT_DCML_PERSISTENT");
    if (e && e[0] == '0') n = 1 << 30;   // one tile per workgroup (non-persistent grid)
  }
  return n;
}

template <typename K, typename PT>
static int launch(K kern, const PT* p, hipStream_t st) {
  if (p->SQ <= 0 || p->NRP <= 0 || (p->SQ * p->L + 15) / 16 > NW * MAXRT) return -4;   // geometry not valid here
  const size_t lds = mat_train_lds_bytes(p->NRP, p->SQ, p->L);
  if (lds > LDS_BUDGET) return -2;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  const int tiles = (p->Bs + p->SQ - 1) / p->SQ;
  const int grid = tiles < n_cus() * WGPC ? tiles : n_cus() * WGPC;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), lds, st, *p);
  MDL_CHECK_LAUNCH();
  return 0;
}

