// Fused MAT decoder (teacher-forced) forward / backward, token-on-lane tiles (mat_train_ct.h).  Reference:
// ma_transformer.py:95-116 (DecodeBlock: causal self attention, causal cross attention on the encoder output, MLP),
// :157-230 (Decoder: action embedding, blocks, action head), transformer_act.py:103-129,176-189 (teacher-forced
// log-prob / entropy of the stored actions: masked Categorical, and the Normal ratio agent of Semi_Discrete).
//
// The action head's second linear (64 -> A, A <= 64) runs on MFMA in the transposed layout: the logits of a token
// are spread over its 4 lanes (a = 16ma + 4g + r), so the softmax statistics are in-lane + 2 permlane swaps.
// Logits use a hi/lo bf16 split of both operands (fp32-like: they feed exp(logp - old_logp)).
#define MDL_LN_ONEPASS
#include "mat_train_ct.h"

namespace {

// token of row i: 0 = start, 1 + a = one-hot of the previous agent's (discrete) action   (transformer_act.py:103-111)
__device__ __forceinline__ int dec_token_ct(const DecP& p, int tok, int i) {
  if (i == 0) return 0;
  int a = (int)p.act[src_tok(p.sidx, (size_t)tok, p.L) - 1];   // the previous agent of the same sequence
  a = a < 0 ? 0 : (a >= p.A ? p.A - 1 : a);
  return 1 + a;
}

// x0 pre-activation = W_a · onehot(token) — a column gather of W_a [64][A+1]; continuous action type:
// W_a · a_prev + b_a with a_prev the previous agent's action vector (zero for row 0)
template <bool CONT>
__device__ __forceinline__ CT dec_embed_pre_ct(const DecP& p, int rt, int& tokid, const Ctx& c) {
  const int lane = c.lane, g = lane >> 4;
  const int row = rt * 16 + (lane & 15);
  const bool ok = row < c.NR;
  CT pre;
  if (CONT) {
    tokid = -1;
    const bool first = !ok || row % c.L == 0;
    const float* prev = p.act + (first ? 0 : src_tok(p.sidx, (size_t)(c.tok0 + row), c.L) - 1) * p.A;
    pre = ld_vec(p.ba, lane);
    for (int k = 0; k < p.A; ++k) {
      const float x = first ? 0.f : prev[k];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) pre.v[mt][r] += p.wa[(16 * mt + 4 * g + r) * p.A + k] * x;
    }
    return pre;
  }
  tokid = ok ? dec_token_ct(p, c.tok0 + row, row % c.L) : 0;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) pre.v[mt][r] = p.wa[(16 * mt + 4 * g + r) * (p.A + 1) + tokid];
  return pre;
}

// Action-embedding table (discrete tokens): x0 = LN_dec(GELU(W_a[:, t])) depends only on the token id t in [0, A]
// (ma_transformer.py:194-195,224 on the one-hot shifted action), so its A + 1 rows — and for the backward x-hat,
// rstd and GELU' — are computed once per tile chunk, one wave per token row (lane = feature), instead of a W_a
// gather, an erf and a LayerNorm per token row.  fwd: X = x0; bwd: X = x-hat, GP = GELU'(pre), RS = rstd.
__device__ __forceinline__ void emb_table(const DecP& p, float* X, float* GP, float* RS, bool fwd, const Ctx& c) {
  const int f = c.lane;
  for (int t = c.wave; t <= p.A; t += NW) {
    float gp;
    const float e = gelu_erf_both(p.wa[f * (p.A + 1) + t], gp);
    const float mean = wave_sum(e) * (1.f / 64.f);
    const float d = e - mean;
    const float rstd = rsqrtf(wave_sum(d * d) * (1.f / 64.f) + 1e-5f);
    const float xh = d * rstd;
    if (fwd) {
      X[t * 64 + f] = fmaf(xh, p.lnd_g[f], p.lnd_b[f]);
    } else {
      X[t * 64 + f] = xh;
      GP[t * 64 + f] = gp;
      if (f == 0) RS[t] = rstd;
    }
  }
}
__device__ __forceinline__ CT emb_row(const float* T, int tok, int lane) {
  const int g = lane >> 4;
  CT x;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) x.v[mt] = *(const f32x4*)(T + tok * 64 + 16 * mt + 4 * g);
  return x;
}
// the tables fit the (free at that point) Q buffer (forward) / Q + K buffers (backward)
__device__ __forceinline__ bool emb_tab_fwd_ok(const DecP& p) { return (p.A + 1) * 64 * 4 <= p.NRP * 128; }
__device__ __forceinline__ bool emb_tab_bwd_ok(const DecP& p) { return (p.A + 1) * (2 * 64 + 1) * 4 <= 2 * p.NRP * 128; }

// ------------------------------------------------------------------------------------------ cross attention
// cross-attention projections: q = W_q rep (from global f32), k / v = W_k x1, W_v x1 (x1 = xr, or the saved x1 when
// xr is null) -> QB / KB / VB; x1 optionally saved (forward) or staged into XB (backward, X of dW_k / dW_v)
// (REG: x1 comes from the registers xr — a compile-time switch: a runtime `xr ? xr[k] : load` put the register
// array's address into a pointer select, which kept all of xr in scratch memory in the forward kernel)
template <bool REG>
__device__ __forceinline__ void cross_proj(const Mat* m, const CT* xr, const bf16_t* sv_x1_in, const float* rep,
                                           bf16_t* sv_x1_out, const Ctx& c, bool store_xb = true) {
  const int lane = c.lane;
  CTr xp[MAXRT], rp[MAXRT];
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      rp[k] = ct_pack(ld_gf(rep, c.tok0, rt, c.NR, lane));
      if constexpr (REG) xp[k] = ct_pack(xr[k]);
      else xp[k] = ld_g(sv_x1_in, c.tok0, rt, c.NR, lane);
      if constexpr (!REG) { if (store_xb) st_lds(c.XB, rt, xp[k], tok_ok(rt, c), lane); }
    }
  }
#pragma unroll
  for (int mi = 0; mi < 3; ++mi) {
    AFr W;
    loadA(W, m[4 + mi].fa, lane);
    const CT b = ld_vec(m[4 + mi].b, lane);
    if (mi == 0 && sv_x1_out) {   // saved x1 behind the first weight load (in-order vmcnt), not ahead of it
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) st_g(sv_x1_out, c.tok0, rt, c.NR, xp[k], lane);
      }
    }
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        CT t = b;
        mm(t, W, mi == 0 ? rp[k] : xp[k]);
        st_lds(mi == 0 ? c.QB : mi == 1 ? c.KB : c.VB, rt, ct_pack(t), tok_ok(rt, c), lane);
      }
    }
  }
}

// x <- LN(rep + proj(attn(q = W_q rep, k = W_k x, v = W_v x)))   (ma_transformer.py:114)
template <bool SAVE>
__device__ __forceinline__ void cross_attn_fwd_ct(const Mat* m, const LNp& ln, CT* xr, const float* rep, bf16_t* sv_x1,
                                                  bf16_t* sv_a, bf16_t* sv_alo, float* sv_lse, bf16_t* sv_xh,
                                                  float* sv_rs, const Ctx& c) {
  const int lane = c.lane;
  __syncthreads();   // every wave done reading the self-attention's K / V
  cross_proj<true>(m, xr, nullptr, rep, SAVE ? sv_x1 : nullptr, c);
  __syncthreads();
  CP_MARK(24);
  CT O[MAXRT];
  float lse[MAXRT][2];
  attn_fwd_ct(c.QB, c.KB, c.VB, true, nullptr, O, c, lse);
  CP_MARK(25);
  AFr Wp;
  loadA(Wp, m[7].fa, lane);
  const CT bp = ld_vec(m[7].b, lane), gam = ld_vec(ln.g, lane), bet = ld_vec(ln.b, lane);
  CT rp[MAXRT];
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) rp[k] = ld_gf(rep, c.tok0, rt, c.NR, lane);
  }
  if (SAVE) lse_store_fwd(sv_lse, lse, c);   // behind the proj weight / rep loads
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      CTr a, alo;
      if (MDL_SAVE_OLO2) ct_split(O[k], a, alo); else a = ct_pack(O[k]);
      if (SAVE) {
        st_g(sv_a, c.tok0, rt, c.NR, a, lane);
        if (MDL_SAVE_OLO2) st_g(sv_alo, c.tok0, rt, c.NR, alo, lane);
      }
      CT t = ct_add(bp, rp[k]), xh;
      mm(t, Wp, a);
      const float rs = ln_fwd_ct(t, xh, xr[k], gam, bet);
      if (SAVE) {
        st_g(sv_xh, c.tok0, rt, c.NR, ct_pack(xh), lane);
        st_tokf(sv_rs, rt, rs, c);
      }
    }
  }  CP_MARK(26);
}

// backward: dx (w.r.t. the sublayer output) -> d x1 (returned in dx); d rep accumulated into global drep
__device__ __forceinline__ void cross_attn_bwd_ct(const Mat* m, const LNp& ln, CT* dx, const float* rep, float* drep,
                                                  const bf16_t* sv_x1, const bf16_t* sv_a, const bf16_t* sv_alo,
                                                  const float* sv_lse, const bf16_t* sv_xh, const float* sv_rs,
                                                  bool first, const Ctx& c, int vslot) {
  const int lane = c.lane;
  const LseR lse = lse_fetch(sv_lse, c);   // consumed after the recompute phase (latency hidden by passes 1-2)
  CT dres[MAXRT];
  {
    CT dlg, dlb;
    ct_zero(dlg);
    ct_zero(dlb);
    {   // pass 1: LN backward from the saved x-hat / rstd -> ds ; DQ = dY of Wp, XB = X of Wp
      const CT gam = ld_vec(ln.g, lane);
      CTr as[MAXRT], xhs[MAXRT];
      float rsv[MAXRT];
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          as[k] = ld_g(sv_a, c.tok0, rt, c.NR, lane);
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
          dres[k] = ds;                              // residual path -> d rep
        }
      }
      flush_vec(dlg, c.g(ln.dg), vslot, c);
      flush_vec(dlb, c.g(ln.db), vslot + 1, c);
    }
    {   // pass 2 (Wpᵀ): dO = Wpᵀ ds -> DA; delta = rowsum(dO O) -> DEL (O = X of Wp, in XB)
      AFr Wpb;
      loadA(Wpb, m[7].ba, lane);
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          const CTr alo = MDL_SAVE_OLO2 ? ld_g(sv_alo, c.tok0, rt, c.NR, lane) : ct_zero_r();
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
  CP_MARK(4);
  // q / k / v recompute (writes QB / KB / VB only; x1 goes to XB later) before the Wp weight gradient (reads DQ / XB):
  // its atomics drain under the attention, one barrier fewer
  cross_proj<false>(m, nullptr, sv_x1, rep, nullptr, c, false);
  wgrad64(c.DQ, c.XB, m[7], c);
  lse_store(lse, c);
  __syncthreads();
  CP_MARK(6);
  attn_bwd_q_ct(c.QB, c.KB, c.VB, c.DA, c.DQ, true, c);
  __syncthreads();
  CP_MARK(7);
  attn_bwd_kv_ct(c.QB, c.KB, c.VB, c.DA, true, c);
  __syncthreads();
  CP_MARK(8);
  {
    CTr rq[MAXRT], xq[MAXRT];
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {   // q input (rep) into QB for dW_q, k / v input (x1) into XB for dW_k / dW_v
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        rq[k] = ct_pack(ld_gf(rep, c.tok0, rt, c.NR, lane));
        xq[k] = ld_g(sv_x1, c.tok0, rt, c.NR, lane);
      }
    }
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        st_lds(c.QB, rt, rq[k], tok_ok(rt, c), lane);
        st_lds(c.XB, rt, xq[k], tok_ok(rt, c), lane);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) ct_zero(dx[k]);
  }
  proj3_bwd(m, 4, c.DQ, c.KB, c.VB, dres, dx, c);   // reads DQ / KB / VB: before the barrier and the weight gradients
  {
    CT cur[MAXRT];
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {   // d rep read-modify-write (each row owned by exactly one wave of one workgroup);
      const int rt = c.wave + NW * k;   // the first block written (the last decoder block) overwrites: no zero fill
      if (rt < c.NT) {
        if (first) ct_zero(cur[k]);
        else cur[k] = ld_gf(drep, c.tok0, rt, c.NR, lane);
      }
    }
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) st_gf(drep, c.tok0, rt, c.NR, ct_add(cur[k], dres[k]), lane);
    }
  }
  __syncthreads();
  CP_MARK(9);
  wgrad64(c.DQ, c.QB, m[4], c);
  {
    const bf16_t* const ys[2] = {c.KB, c.VB};
    const Mat* const ms[2] = {&m[5], &m[6]};
    wgrad64_shared_x<2>(ys, c.XB, ms, c);
  }
  __syncthreads();
  CP_MARK(10);
}

// ------------------------------------------------------------------------------------------ action head
// logits = W_h2 · LN(GELU(W_h1 x + b)) + b_h2  (ma_transformer.py:202-203,228); MA = ceil(A / 16) logit tiles
template <int MA>
struct HeadW { bf16x8 hi[MA][2], lo[MA][2]; };

template <int MA>
__device__ __forceinline__ void head_w(const DecP& p, HeadW<MA>& W, int lane) {
  const int c16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ma = 0; ma < MA; ++ma)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int a = 16 * ma + c16, k = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
        const float w = a < p.A ? p.wh2[(a < p.A ? a : 0) * 64 + k] : 0.f;
        const uint16_t h = f2bf(w);
        W.hi[ma][s][j] = (short)h;
        W.lo[ma][s][j] = (short)f2bf(w - bf2f(h));
      }
}

template <int MA>
__device__ __forceinline__ void head_logits_ct(const DecP& p, const HeadW<MA>& W, const CT& n, f32x4* L, int lane) {
  const int g = lane >> 4;
  CTr nh, nl;
  ct_split(n, nh, nl);
#pragma unroll
  for (int ma = 0; ma < MA; ++ma) {
    f32x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 16 * ma + 4 * g + r;
      acc[r] = a < p.A ? p.bh2[a] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W.hi[ma][s], rb(nh, s), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W.hi[ma][s], rb(nl, s), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W.lo[ma][s], rb(nh, s), acc, 0, 0, 0);
    }
    L[ma] = acc;
  }
}

// availability bits of this lane's logit slots (a = 16ma + 4g + r): bit 4ma + r set = masked (tok: input row)
template <int MA>
__device__ __forceinline__ unsigned slot_mask(const DecP& p, size_t tok, int lane) {
  if (!p.ava) return 0u;
  const int g = lane >> 4;
  unsigned m = 0u;
#pragma unroll
  for (int ma = 0; ma < MA; ++ma)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 16 * ma + 4 * g + r;
      if (a < p.A && p.ava[tok * p.A + a] == 0.f) m |= 1u << (4 * ma + r);
    }
  return m;
}

// per-token softmax statistics of the masked logits (transformer_act.py:14-21: logit[ava == 0] = -1e10)
struct HeadStat { float lse, H, la, mean; };
template <int MA>
__device__ __forceinline__ HeadStat head_stats(const DecP& p, const f32x4* L, unsigned am, int act, bool disc, int lane) {
  const int g = lane >> 4;
  float mx = -INFINITY;
#pragma unroll
  for (int ma = 0; ma < MA; ++ma)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 16 * ma + 4 * g + r;
      const float l = ((am >> (4 * ma + r)) & 1u) ? -1e10f : L[ma][r];
      if (a < p.A) mx = fmaxf(mx, l);
    }
  mx = cross_row_max(mx);
  float se = 0.f, mean = 0.f;
#pragma unroll
  for (int ma = 0; ma < MA; ++ma)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 16 * ma + 4 * g + r;
      const float l = ((am >> (4 * ma + r)) & 1u) ? -1e10f : L[ma][r];
      se += a < p.A ? __expf(l - mx) : 0.f;
      mean += a == p.A - 1 ? L[ma][r] : 0.f;
    }
  HeadStat st;
  st.lse = mx + __logf(cross_row_sum(se));
  st.mean = cross_row_sum(mean);
  float H = 0.f, la = 0.f;
  if (disc) {
#pragma unroll
    for (int ma = 0; ma < MA; ++ma)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = 16 * ma + 4 * g + r;
        const float l = (((am >> (4 * ma + r)) & 1u) ? -1e10f : L[ma][r]) - st.lse;
        H -= a < p.A ? __expf(l) * l : 0.f;
        la += a == act ? l : 0.f;
      }
  }
  st.H = cross_row_sum(H);
  st.la = cross_row_sum(la);
  return st;
}

constexpr float HALF_LOG_2PI = 0.91893853320467274f;

// Normal-head std = sigmoid(log_std) * 0.5 (transformer_act.py:6, ma_transformer.py action std), from the parameter
// itself (round 1 read a per-minibatch torch copy: three launches per minibatch)
__device__ __forceinline__ float head_sd(const DecP& p, int a) { return 0.5f / (1.f + __expf(-p.log_std[a])); }

template <int MA, bool CONT>
__device__ __forceinline__ void head_fwd_ct(const DecP& p, const CT* xr, bool save, const Ctx& c) {
  const int lane = c.lane, g = lane >> 4;
  HeadW<MA> W;
  head_w<MA>(p, W, lane);
  AFr H;
  loadA(H, p.h1.fa, lane);
  const CT bh = ld_vec(p.h1.b, lane), gam = ld_vec(p.lnh.g, lane), bet = ld_vec(p.lnh.b, lane);
  CP_MARK(31);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      const int row = rt * 16 + (lane & 15);
      const bool ok = row < c.NR;
      const size_t tok = (size_t)(c.tok0 + (ok ? row : 0)), stok = src_tok(p.sidx, tok, c.L);
      const unsigned am = CONT ? 0u : slot_mask<MA>(p, stok, lane);
      const float actf = CONT ? 0.f : p.act[stok];
      const CTr x = ct_pack(xr[k]);
      if (save) st_g(p.sv_head, c.tok0, rt, c.NR, x, lane);
      CT hh = bh, xh, n;
      mm(hh, H, x);
      if (save && p.hs.xh) {   // x-hat, GELU'(h), rstd for the backward
        CT gp;
        gelu_ct_both(hh, gp);
        const float rs = ln_fwd_ct(hh, xh, n, gam, bet);
        st_g(p.hs.xh, c.tok0, rt, c.NR, ct_pack(xh), lane);
        st_g(p.hs.gp, c.tok0, rt, c.NR, ct_pack(gp), lane);
        st_tokf(p.hs.rs, rt, rs, c);
      } else {
        gelu_ct(hh);
        ln_fwd_ct(hh, xh, n, gam, bet);
      }
      CP_MARK(32);
      f32x4 L[MA];
      head_logits_ct<MA>(p, W, n, L, lane);
      CP_MARK(33);
      if (CONT) {   // per-dimension Normal(mean, std): this lane's dims a = 16ma + 4g + r
#pragma unroll
        for (int ma = 0; ma < MA; ++ma)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int a = 16 * ma + 4 * g + r;
            if (ok && a < p.A) {
              const float sd = head_sd(p, a), z = (p.act[stok * p.A + a] - L[ma][r]) / sd;
              p.logp[tok * p.A + a] = -0.5f * z * z - __logf(sd) - HALF_LOG_2PI;
              p.ent[tok * p.A + a] = 0.5f + HALF_LOG_2PI + __logf(sd);
            }
          }
        continue;
      }
      const bool disc = (row % c.L) < p.n_disc;
      const int act = min(max((int)actf, 0), p.A - 1);
      const HeadStat st = head_stats<MA>(p, L, am, act, disc, lane);
      float lp, en;
      if (disc) {
        lp = st.la;
        en = st.H;
      } else {
        const float sd = head_sd(p, p.A - 1), z = (actf - st.mean) / sd;
        lp = -0.5f * z * z - __logf(sd) - HALF_LOG_2PI;
        en = 0.5f + HALF_LOG_2PI + __logf(sd);
      }
      if (ok && g == 0) {
        p.logp[tok] = lp;
        p.ent[tok] = en;
      }
      CP_MARK(34);
    }
  }
}

// LDS vector slots of the small weight gradients (wgrad_g_vacc): d W_a (A+1 slots), d W_h2 (A slots), d b_h2 (1), after
// the 5 + 6 NB LayerNorm / log_std slots; -1 when they do not fit (A > 2 or NB = 3: per-chunk private / atomic flush)
#ifndef MDL_SMALL_WG_VACC
#define MDL_SMALL_WG_VACC 1
#endif
__device__ __forceinline__ int small_wg_slot0(const DecP& p, int NB) {
  const int s0 = 5 + 6 * NB;
  return (MDL_SMALL_WG_VACC && p.A <= 2 && s0 + 2 * p.A + 2 <= VSLOTS) ? s0 : -1;
}

template <int MA, bool CONT>
__device__ __forceinline__ void head_bwd_ct(const DecP& p, CT* dx, const Ctx& c, int vs0) {
  const int lane = c.lane, g = lane >> 4;
  constexpr int SB = (MA + 1) / 2;   // k-steps over the logit axis in dn = W_h2ᵀ dz
  CT dlg, dlb;
  ct_zero(dlg);
  ct_zero(dlb);
  float dls = 0.f;
  f32x4 dlsv[MA];   // continuous: per-dimension log_std partials of this lane's slots
#pragma unroll
  for (int ma = 0; ma < MA; ++ma) dlsv[ma] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    HeadW<MA> W;
    head_w<MA>(p, W, lane);
    // W_h2ᵀ as A fragments: rows = features 16mt + (lane&15), k = logit index perm(s, g, j)
    bf16x8 WT[4][SB];
    {
      const int c16 = lane & 15;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int s = 0; s < SB; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int a = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
            const float w = a < p.A ? p.wh2[(a < p.A ? a : 0) * 64 + 16 * mt + c16] : 0.f;
            WT[mt][s][j] = (short)f2bf(w);
          }
    }
    // the forward's x-hat, GELU'(h) and rstd of the head (no W_h1 product, GELU or LayerNorm forward here)
    CTr hxh[MAXRT], hgp[MAXRT];
    float hrs[MAXRT];
    {
      CTr xs[MAXRT];
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          xs[k] = ld_g(p.sv_head, c.tok0, rt, c.NR, lane);
          hxh[k] = ld_g(p.hs.xh, c.tok0, rt, c.NR, lane);
          hgp[k] = ld_g(p.hs.gp, c.tok0, rt, c.NR, lane);
          hrs[k] = ld_tokf(p.hs.rs, rt, c);
        }
      }
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) st_lds(c.KB, rt, xs[k], tok_ok(rt, c), lane);   // X of W_h1
      }
    }
    const CT gam = ld_vec(p.lnh.g, lane), bet = ld_vec(p.lnh.b, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const int row = rt * 16 + (lane & 15);
        const bool ok = row < c.NR;
        const size_t tok = (size_t)(c.tok0 + (ok ? row : 0)), stok = src_tok(p.sidx, tok, c.L);
        const unsigned am = CONT ? 0u : slot_mask<MA>(p, stok, lane);
        const float actf = CONT ? 0.f : p.act[stok];
        const float dlp = (ok && !CONT) ? p.dlogp[tok] : 0.f, den = (ok && !CONT) ? p.dent[tok] : 0.f;
        const CT xh = ct_unpack(hxh[k]), ggp = ct_unpack(hgp[k]);
        const float rs = hrs[k];
        CT n;
#pragma unroll
        for (int i = 0; i < 4; ++i) n.v[i] = xh.v[i] * gam.v[i] + bet.v[i];
        f32x4 L[MA];
        head_logits_ct<MA>(p, W, n, L, lane);
        const bool disc = !CONT && (row % c.L) < p.n_disc;
        const int act = min(max((int)actf, 0), p.A - 1);
        const HeadStat st = CONT ? HeadStat{0.f, 0.f, 0.f, 0.f} : head_stats<MA>(p, L, am, act, disc, lane);
        // d loss / d logits of this lane's slots
        f32x4 Z[2 * SB];
#pragma unroll
        for (int ma = 0; ma < 2 * SB; ++ma) Z[ma] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (CONT) {   // per-dimension Normal heads: d log p / d mean, and the log_std partials of this lane's dims
#pragma unroll
          for (int ma = 0; ma < MA; ++ma)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int a = 16 * ma + 4 * g + r;
              if (ok && a < p.A) {
                const float sd = head_sd(p, a), diff = p.act[stok * p.A + a] - L[ma][r];
                const float dl = p.dlogp[tok * p.A + a], de = p.dent[tok * p.A + a];
                Z[ma][r] = dl * diff / (sd * sd);
                const float dsd = dl * (diff * diff / (sd * sd * sd) - 1.f / sd) + de / sd;
                const float sg = 1.f / (1.f + __expf(-p.log_std[a]));
                dlsv[ma][r] += dsd * 0.5f * sg * (1.f - sg);
              }
            }
        } else if (disc) {
#pragma unroll
          for (int ma = 0; ma < MA; ++ma)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int a = 16 * ma + 4 * g + r;
              const float l = (((am >> (4 * ma + r)) & 1u) ? -1e10f : L[ma][r]) - st.lse;
              const float pr = __expf(l);
              const float z = dlp * ((a == act ? 1.f : 0.f) - pr) - den * pr * (l + st.H);
              Z[ma][r] = (ok && a < p.A) ? z : 0.f;
            }
        } else {
          const float sd = head_sd(p, p.A - 1), diff = actf - st.mean;
#pragma unroll
          for (int ma = 0; ma < MA; ++ma)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              Z[ma][r] = (ok && 16 * ma + 4 * g + r == p.A - 1) ? dlp * diff / (sd * sd) : 0.f;
          if (ok && g == 0) {
            const float dsd = dlp * (diff * diff / (sd * sd * sd) - 1.f / sd) + den / sd;
            const float sg = 1.f / (1.f + __expf(-p.log_std[p.A - 1]));
            dls += dsd * 0.5f * sg * (1.f - sg);
          }
        }
        // dn = W_h2ᵀ dz (hi / lo split of dz)
        CT dn;
        ct_zero(dn);
        CTr zh, zl;   // dz as a CT-shaped operand: piece ma = logits 16ma + 4g .. +3
        {
          CT zc;
#pragma unroll
          for (int ma = 0; ma < 4; ++ma) zc.v[ma] = ma < 2 * SB ? Z[ma < 2 * SB ? ma : 0] : f32x4{0.f, 0.f, 0.f, 0.f};
          ct_split(zc, zh, zl);
        }
#pragma unroll
        for (int s = 0; s < SB; ++s)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            dn.v[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WT[mt][s], rb(zh, s), dn.v[mt], 0, 0, 0);
            dn.v[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WT[mt][s], rb(zl, s), dn.v[mt], 0, 0, 0);
          }
        st_lds(c.DA, rt, zh, ok, lane);            // dY of W_h2 (logit axis in the feature slots)
        st_lds(c.XB, rt, ct_pack(n), ok, lane);    // X of W_h2
        CT dgg;
        ln_bwd_ct(dn, xh, rs, gam, ok, dgg, dlg, dlb);
#pragma unroll
        for (int i = 0; i < 4; ++i) dgg.v[i] *= ggp.v[i];   // padded rows: x-hat, GELU' and rstd are zero
        st_lds(c.DQ, rt, ct_pack(dgg), ok, lane);   // dY of W_h1
      }
    }
  }
  {   // second pass (W_h1ᵀ): dx = W_h1ᵀ dY
    AFr Hb;
    loadA(Hb, p.h1.ba, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        ct_zero(dx[k]);
        mm(dx[k], Hb, ld_lds(c.DQ, rt, lane));
      }
    }
  }
  flush_vec(dlg, c.g(p.lnh.dg), 0, c);
  flush_vec(dlb, c.g(p.lnh.db), 1, c);
  if (CONT) {
#pragma unroll
    for (int ma = 0; ma < MA; ++ma)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = group_sum<16>(dlsv[ma][r]);
        const int a = 16 * ma + 4 * g + r;
        if ((lane & 15) == 0 && a < p.A && p.d_log_std) vacc_add(c.g(p.d_log_std), 4, a, t, c, p.A);
      }
  } else {
    const float t = wave_sum(dls);
    if (lane == 0 && p.d_log_std && p.n_disc < p.L) vacc_add(c.g(p.d_log_std), 4, p.A - 1, t, c, p.A);
  }
  __syncthreads();
  CP_MARK(1);
  if (vs0 >= 0)   // slots vs0 + A + 1 .. (W_h2 rows), vs0 + 2A + 1 (bias)
    wgrad_g_vacc(c.DA, c.XB, c.KP, c.g(p.d_wh2), 64, p.A, 64, c.g(p.d_bh2), vs0 + p.A + 1, vs0 + 2 * p.A + 1, c);
  else
    wgrad_g(c.DA, c.XB, c.KP, c.g(p.d_wh2), 64, p.A, 64, c.g(p.d_bh2), c.wave, lane, c.gm);
  wgrad64(c.DQ, c.KB, p.h1, c);
  __syncthreads();
  CP_MARK(19);
}

// ============================================================================================== forward
template <int NB, bool SAVE, int MA, bool CONT>
__device__ __forceinline__ void dec_fwd_tile(const DecP& p, char* smem, int seq0, int nseq) {
  const Ctx c = make_ctx(p, smem, seq0, nseq);
  if (c.nseq <= 0) return;
  zero_pad_rows_fwd(c);
  __syncthreads();
  CP_MARK(0);
  const int lane = c.lane;
  CT xr[MAXRT];
  if (!CONT && emb_tab_fwd_ok(p)) {   // x0 rows from the per-token table (in QB until the first projection)
    float* X0 = (float*)c.QB;
    emb_table(p, X0, nullptr, nullptr, true, c);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const int row = rt * 16 + (lane & 15);
        const int tk = row < c.NR ? dec_token_ct(p, c.tok0 + row, row % c.L) : 0;
        xr[k] = emb_row(X0, tk, lane);
      }
    }
  } else {
    const CT gam = ld_vec(p.lnd_g, lane), bet = ld_vec(p.lnd_b, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        int tk;
        CT pre = dec_embed_pre_ct<CONT>(p, rt, tk, c), xh;
        gelu_ct(pre);
        ln_fwd_ct(pre, xh, xr[k], gam, bet);
      }
    }
  }
#pragma unroll 1
  for (int b = 0; b < NB; ++b) {
    const Blk& B = p.blk[b];
    Ctx cc = c;
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    self_attn_fwd_ct<SAVE>(B.m, B.ln[0], xr, true, p.sv[b].xin, p.sv[b].a1, p.sv[b].a1lo, p.sv[b].lse1,
                           p.sv[b].xh[0], p.sv[b].rs + 0 * (size_t)p.Bs * p.L, cc);
    cross_attn_fwd_ct<SAVE>(B.m, B.ln[1], xr, p.rep, p.sv[b].x1, p.sv[b].a2, p.sv[b].a2lo, p.sv[b].lse2,
                            p.sv[b].xh[1], p.sv[b].rs + 1 * (size_t)p.Bs * p.L, cc);
    mlp_fwd_ct<SAVE>(B.m[8], B.m[9], B.ln[2], xr, p.sv[b].x2, p.sv[b].g, p.sv[b].gp, p.sv[b].xh[2], p.sv[b].rs + 2 * (size_t)p.Bs * p.L, cc);
  }
  head_fwd_ct<MA, CONT>(p, xr, SAVE, c);
  CP_MARK(27);
}

#ifndef MDL_CT_BWD_TU
// MA = logit tiles of the action head: 1 (A <= 16: DCML, MPE), 3 (A <= 48: SMAC's 36 actions) or 4 (A <= 64)
template <int NB, bool SAVE, int MA, bool CONT>
__global__ __launch_bounds__(NTHR, FWD_WGPC) void mat_dec_fwd_ct(DecP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CP_BEGIN();
  FOR_TILES(p, (dec_fwd_tile<NB, SAVE, MA, CONT>(p, smem, s0, ns)));
  CP_END();
}

#endif  // !MDL_CT_BWD_TU

// ============================================================================================== backward
template <int NB, int MA, bool CONT>
__device__ __forceinline__ void dec_bwd_tile(const DecP& p, char* smem, int seq0, int nseq, bool first) {
  const Ctx c = make_ctx(p, smem, seq0, nseq, first);
  if (c.nseq <= 0) return;
  zero_pad_rows(c);
  __syncthreads();
  CP_MARK(0);
  const int lane = c.lane;
  CT dx[MAXRT];
  const int vs0 = small_wg_slot0(p, NB);
  head_bwd_ct<MA, CONT>(p, dx, c, vs0);
#pragma unroll 1
  for (int bb = NB - 1; bb >= 0; --bb) {
    const Blk& B = p.blk[bb];
    Ctx cc = c;
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    // parameter-vector slots (vacc): 0-1 head LayerNorm, 2-3 embedding LayerNorm, 4 log_std, 5 + 6 bb + 2 k the
    // block's k-th LayerNorm (gamma, beta); then the small weight gradients from vs0 (small_wg_slot0)
    mlp_bwd_ct(B.m[8], B.m[9], B.ln[2], dx, p.sv[bb].x2, p.sv[bb].g, p.sv[bb].gp, p.sv[bb].xh[2], p.sv[bb].rs + 2 * (size_t)p.Bs * p.L, cc,
               9 + 6 * bb);
    cross_attn_bwd_ct(B.m, B.ln[1], dx, p.rep, p.drep, p.sv[bb].x1, p.sv[bb].a2, p.sv[bb].a2lo, p.sv[bb].lse2,
                      p.sv[bb].xh[1], p.sv[bb].rs + 1 * (size_t)p.Bs * p.L, bb == NB - 1, cc, 7 + 6 * bb);
    self_attn_bwd_ct(B.m, B.ln[0], dx, p.sv[bb].xin, p.sv[bb].a1, p.sv[bb].a1lo, p.sv[bb].lse1, p.sv[bb].xh[0],
                     p.sv[bb].rs + 0 * (size_t)p.Bs * p.L, true, cc, 5 + 6 * bb);
  }
  // ---------------- embedding backward: dW_a[:, token] += d pre ; LN_dec params
  if (!CONT) {
    // discrete tokens: dW_a (64 x (A+1)) = Σ_rows d pre ⊗ onehot(token) — a weight-gradient GEMM on MFMA with the
    // one-hot rows as X (wgrad_g), d pre as a hi/lo bf16 pair; replaces per-element LDS atomics that collided on
    // the (A+1) token rows (16-way address conflicts per wave instruction)
    CT dlg, dlb;
    ct_zero(dlg);
    ct_zero(dlb);
    const CT gam = ld_vec(p.lnd_g, lane), bet = ld_vec(p.lnd_b, lane);
    const int g = lane >> 4;
    const bool tab = emb_tab_bwd_ok(p);   // x-hat / GELU' / rstd per token id in QB + KB (free after the blocks)
    float* XT = (float*)c.QB;
    float* GT = XT + (p.A + 1) * 64;
    float* RT = GT + (p.A + 1) * 64;
    if (tab) {
      emb_table(p, XT, GT, RT, false, c);
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const bool ok = tok_ok(rt, c);
        int tk;
        CT egp, xh, de;
        float rs;
        if (tab) {
          const int row = rt * 16 + (lane & 15);
          tk = row < c.NR ? dec_token_ct(p, c.tok0 + row, row % c.L) : 0;
          xh = emb_row(XT, tk, lane);
          egp = emb_row(GT, tk, lane);
          rs = RT[tk];
        } else {
          CT e = dec_embed_pre_ct<CONT>(p, rt, tk, c), yy;
          gelu_ct_both(e, egp);
          rs = ln_fwd_ct(e, xh, yy, gam, bet);
        }
        ln_bwd_ct(dx[k], xh, rs, gam, ok, de, dlg, dlb);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) de.v[mt][r] = ok ? de.v[mt][r] * egp.v[mt][r] : 0.f;
        CTr dh, dl, oh;
        ct_split(de, dh, dl);
        CT onehot;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) onehot.v[mt][r] = (ok && 16 * mt + 4 * g + r == tk) ? 1.f : 0.f;
        oh = ct_pack(onehot);
        st_lds(c.DA, rt, dh, ok, lane);   // dY (hi)
        st_lds(c.DQ, rt, dl, ok, lane);   // dY (lo)
        st_lds(c.XB, rt, oh, ok, lane);   // X = one-hot token rows
      }
    }
    flush_vec(dlg, c.g(p.d_lnd_g), 2, c);
    flush_vec(dlb, c.g(p.d_lnd_b), 3, c);
    __syncthreads();
    if (p.d_wa) {
      // hi and lo halves of d pre in one pass: one flush (LDS slots vs0 .. vs0 + A, or one read-modify-write of a
      // private copy per chunk)
      if (vs0 >= 0) wgrad_g_vacc(c.DA, c.XB, c.KP, c.g(p.d_wa), p.A + 1, 64, p.A + 1, nullptr, vs0, -1, c, c.DQ);
      else wgrad_g(c.DA, c.XB, c.KP, c.g(p.d_wa), p.A + 1, 64, p.A + 1, nullptr, c.wave, lane, c.gm, c.DQ);
    }
  } else {
    float* EMB = (float*)c.QB;   // [(A+1)][64] f32 accumulators (QB + KB: 2 NRP x 128 B >= 65 x 256 B)
    for (int i = c.tid; i < (p.A + 1) * 64; i += NTHR) EMB[i] = 0.f;
    __syncthreads();
    CT dlg, dlb;
    ct_zero(dlg);
    ct_zero(dlb);
    const CT gam = ld_vec(p.lnd_g, lane), bet = ld_vec(p.lnd_b, lane);
    const int g = lane >> 4;
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const bool ok = tok_ok(rt, c);
        int tk;
        CT e = dec_embed_pre_ct<CONT>(p, rt, tk, c), egp, xh, yy, de;
        gelu_ct_both(e, egp);
        const float rs = ln_fwd_ct(e, xh, yy, gam, bet);
        ln_bwd_ct(dx[k], xh, rs, gam, ok, de, dlg, dlb);
        if (ok) {   // EMB[k][f] += d pre_f * a_prev_k (k < A), EMB[A][f] += d pre_f (bias)
          const int row = rt * 16 + (lane & 15);
          const bool first = row % c.L == 0;
          const float* prev = p.act + (first ? 0 : src_tok(p.sidx, (size_t)(c.tok0 + row), c.L) - 1) * p.A;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float dp = de.v[mt][r] * egp.v[mt][r];
              const int f = 16 * mt + 4 * g + r;
              atomicAdd(EMB + p.A * 64 + f, dp);
              if (!first)
                for (int kk = 0; kk < p.A; ++kk) atomicAdd(EMB + kk * 64 + f, dp * prev[kk]);
            }
        }
      }
    }
    flush_vec(dlg, c.g(p.d_lnd_g), 2, c);
    flush_vec(dlb, c.g(p.d_lnd_b), 3, c);
    __syncthreads();
    for (int i = c.tid; i < (p.A + 1) * 64; i += NTHR) {   // W_a [64][A] and b_a
      const int t = i / 64, col = i % 64;
      float* d = t < p.A ? (p.d_wa ? c.g(p.d_wa) + col * p.A + t : nullptr) : (p.d_ba ? c.g(p.d_ba) + col : nullptr);
      if (!d) continue;
      if (c.gm.priv) priv_st1(d, EMB[i], (c.gm.first || !PRIV_LOADS) ? 0.f : priv_ld1(d), c.gm.first);   // owner thread
      else atomicAdd(d, EMB[i]);
    }
  }
  CP_MARK(30);
}

#ifdef MDL_CT_BWD_TU
template <int NB, int MA, bool CONT>
__global__ __launch_bounds__(NTHR, WGPC) void mat_dec_bwd_ct(DecP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CP_BEGIN();
  vacc_begin(p, smem);
  FOR_TILES(p, (dec_bwd_tile<NB, MA, CONT>(p, smem, s0, ns, it_ == 0)));
  vacc_end(p, smem);
  CP_END();
}

#endif  // MDL_CT_BWD_TU

}  // namespace

#ifndef MDL_CT_BWD_TU
template <int MA, bool CONT>
static int dec_fwd_ct(const DecP* p, int NB, int save, hipStream_t st) {
  if (NB == 1) return save ? launch_ct(mat_dec_fwd_ct<1, true, MA, CONT>, p, true, st) : launch_ct(mat_dec_fwd_ct<1, false, MA, CONT>, p, true, st);
  if (NB == 2) return save ? launch_ct(mat_dec_fwd_ct<2, true, MA, CONT>, p, true, st) : launch_ct(mat_dec_fwd_ct<2, false, MA, CONT>, p, true, st);
  if (NB == 3) return save ? launch_ct(mat_dec_fwd_ct<3, true, MA, CONT>, p, true, st) : launch_ct(mat_dec_fwd_ct<3, false, MA, CONT>, p, true, st);
  return -3;
}
// MA = logit tiles of the action head (1: A <= 16, 3: A <= 48 — SMAC's 36 actions, 4: A <= 64); the continuous
// action type is its own instantiation (its Normal-head / Linear-embedding code kept out of the discrete kernels'
// instruction stream)
MDL_API int mdl_mat_dec_fwd_ct(const DecP* p, int NB, int save, hipStream_t st) {
  if (p->A > 64 || p->A < 1) return -1;
  if (p->cont) return p->A <= 16 ? dec_fwd_ct<1, true>(p, NB, save, st) : dec_fwd_ct<4, true>(p, NB, save, st);
  if (p->A <= 16) return dec_fwd_ct<1, false>(p, NB, save, st);
  return p->A <= 48 ? dec_fwd_ct<3, false>(p, NB, save, st) : dec_fwd_ct<4, false>(p, NB, save, st);
}
#else
template <int MA, bool CONT>
static int dec_bwd_ct(const DecP* p, int NB, hipStream_t st) {
  if (NB == 1) return launch_ct(mat_dec_bwd_ct<1, MA, CONT>, p, false, st);
  if (NB == 2) return launch_ct(mat_dec_bwd_ct<2, MA, CONT>, p, false, st);
  if (NB == 3) return launch_ct(mat_dec_bwd_ct<3, MA, CONT>, p, false, st);
  return -3;
}

MDL_API int mdl_mat_dec_bwd_ct(const DecP* p, int NB, hipStream_t st) {
  if (p->A > 64 || p->A < 1 || 2 * p->NRP * 128 < (p->A + 1) * 256) return -1;
  if (p->cont) return p->A <= 16 ? dec_bwd_ct<1, true>(p, NB, st) : dec_bwd_ct<4, true>(p, NB, st);
  if (p->A <= 16) return dec_bwd_ct<1, false>(p, NB, st);
  return p->A <= 48 ? dec_bwd_ct<3, false>(p, NB, st) : dec_bwd_ct<4, false>(p, NB, st);
}
#endif  // MDL_CT_BWD_TU

#ifdef MDL_CT_PROF
MDL_API int MDL_CAT(mdl_ctprof_dec, MDL_CT_TU_SUFFIX)(unsigned long long* out, int reset) {
  if (reset) {
    unsigned long long z[64] = {0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ctprof), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ctprof), sizeof(unsigned long long) * 64, 0, hipMemcpyDeviceToHost);
}
#endif
