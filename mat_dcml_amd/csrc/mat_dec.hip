// Fused MAT decoder (teacher-forced) forward / backward kernels (see mat_train_common.h).
#include "mat_train_common.h"

// ============================================================================================== decoder pieces
// token of row i: 0 = start, 1 + a = one-hot of the previous agent's (discrete) action   (transformer_act.py:103-111)
__device__ __forceinline__ int dec_token(const DecP& p, int tok, int i) {
  if (i == 0) return 0;
  int a = (int)p.act[tok - 1];
  a = a < 0 ? 0 : (a >= p.A ? p.A - 1 : a);
  return 1 + a;
}

// x0 = LN_dec(GELU(W_a · onehot(token)))  (ma_transformer.py:194-195,224-225) — a column gather of W_a
__device__ __forceinline__ void dec_embed_pre(const DecP& p, int rt, RT& pre, int* tokr, const Ctx& c) {
  const int g = c.lane >> 4, c16 = c.lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rt * 16 + 4 * g + r;
    tokr[r] = row < c.NR ? dec_token(p, c.tok0 + row, row % c.L) : 0;
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) pre.v[ct][r] = p.wa[(16 * ct + c16) * (p.A + 1) + tokr[r]];
}

// cross attention sublayer: out = LN(rep + proj(attn(q = W_q rep, k = W_k x1, v = W_v x1)))  (ma_transformer.py:114)
template <bool SAVE>
__device__ __forceinline__ void attn_cross_fwd(const Mat* m, const LNp& ln, RT* xr, const float* rep, bf16_t* sv_x1, bf16_t* sv_a,
                               float* sv_lse, const Ctx& c) {
  const int lane = c.lane;
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      st_tm_m(c.XB, rt, xr[k], row_mask(rt, c.NR, lane), lane);
      if (SAVE) { wave_lds_sync(); tile2g(sv_x1, c.XB, rt, c); }
    }
  }
  wave_lds_sync();
  {
    bf16_t* outs[2] = {c.KB, c.VB};
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      BFr B;
      loadB(B, m[5 + mi].fw, lane);
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + 4 * k;
        if (rt < c.NT) {
          RT t;
          gemm_rt(t, c.XB, rt, B, lane, false);
          add_bias(t, m[5 + mi].b, lane);
          st_tm_m(outs[mi], rt, t, row_mask(rt, c.NR, lane), lane);
        }
      }
    }
    BFr B;
    loadB(B, m[4].fw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT r_;
        ld_g_f(rep, c.tok0, rt, c.NR, r_, lane);
        st_tm_m(c.XB, rt, r_, vm, lane);
        wave_lds_sync();
        RT t;
        gemm_rt(t, c.XB, rt, B, lane, false);
        add_bias(t, m[4].b, lane);
        st_tm_m(c.QB, rt, t, vm, lane);
      }
    }
  }
  __syncthreads();
  attn_fwd(c.QB, c.KB, c.VB, c.QB, true, SAVE ? sv_lse : nullptr, c);
  __syncthreads();
  BFr B;
  loadB(B, m[7].fw, lane);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      if (SAVE) tile2g(sv_a, c.QB, rt, c);
      RT t, r_, xh, y;
      gemm_rt(t, c.QB, rt, B, lane, false);
      add_bias(t, m[7].b, lane);
      ld_g_f(rep, c.tok0, rt, c.NR, r_, lane);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) t.v[ct] += r_.v[ct];
      f32x4 mu, rs;
      ln_fwd(t, xh, y, mu, rs, ln.g, ln.b, lane);
      xr[k] = y;
    }
  }
}

// cross attention backward: dx (w.r.t. the sublayer output) -> d x1 (returned in dx), d rep accumulated in global
__device__ __forceinline__ void attn_cross_bwd(const Mat* m, const LNp& ln, RT* dx, const float* rep, float* drep,
                                               const bf16_t* sv_x1, const bf16_t* sv_a, const float* sv_lse,
                                               const Ctx& c) {
  const int lane = c.lane;
  TP_DECL();
  f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0}, dbp = {0, 0, 0, 0};
  RT dres[MAXRT];
  {
    BFr Bpf, Bpb;
    loadB(Bpf, m[7].fw, lane);
    loadB(Bpb, m[7].bw, lane);
    g2tiles(c.XB, sv_a, nullptr, nullptr, c);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT r_;
        ld_g_f(rep, c.tok0, rt, c.NR, r_, lane);
        wave_lds_sync();
        RT s, xh, y, ds;
        gemm_rt(s, c.XB, rt, Bpf, lane, false);
        add_bias(s, m[7].b, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) s.v[ct] += r_.v[ct];
        f32x4 mu, rs;
        ln_fwd(s, xh, y, mu, rs, ln.g, ln.b, lane);
        ln_bwd(dx[k], xh, rs, ln.g, ds, dlg, dlb, vm, lane);
        colsum_acc(ds, dbp, vm);
        st_tm_m(c.DQ, rt, ds, vm, lane);
        wave_lds_sync();
        RT da;
        gemm_rt(da, c.DQ, rt, Bpb, lane, false);
        st_tm_m(c.DA, rt, da, vm, lane);
        dres[k] = ds;                  // residual path -> d rep
      }
    }
  }
  flush_ln(dlg, dlb, ln, c);
  flush_cols(dbp, c.g(m[7].db), lane);
  __syncthreads();
  TP_MARK(7);
  wgrad_tm(c.DQ, c.XB, c.NRP, c.g(m[7].dW), c.wave, lane);
  __syncthreads();
  TP_MARK(12);
  // recompute k, v (from x1) and q (from rep)
  g2lds_rows(c.XB, sv_x1, c.tok0, c.NR, c.NT * 16, c.tid);
  load_lse(sv_lse, c);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      RT r_;
      ld_g_f(rep, c.tok0, rt, c.NR, r_, lane);
      st_tm_m(c.DQ, rt, r_, row_mask(rt, c.NR, lane), lane);  // rep (bf16) as the q-projection input
    }
  }
  __syncthreads();
  {
    BFr B;
    loadB(B, m[5].fw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        RT t;
        gemm_rt(t, c.XB, rt, B, lane, false);
        add_bias(t, m[5].b, lane);
        st_tm_m(c.KB, rt, t, row_mask(rt, c.NR, lane), lane);
      }
    }
    loadB(B, m[6].fw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        RT t;
        gemm_rt(t, c.XB, rt, B, lane, false);
        add_bias(t, m[6].b, lane);
        st_tm_m(c.VB, rt, t, row_mask(rt, c.NR, lane), lane);
      }
    }
    loadB(B, m[4].fw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        RT t;
        gemm_rt(t, c.DQ, rt, B, lane, false);
        add_bias(t, m[4].b, lane);
        st_tm_m(c.QB, rt, t, row_mask(rt, c.NR, lane), lane);
      }
    }
  }
  __syncthreads();
  TP_MARK(13);
  attn_bwd_q(c.QB, c.KB, c.VB, c.DA, c.DQ, true, c);
  __syncthreads();
  TP_MARK(14);
  attn_bwd_kv(c.QB, c.KB, c.VB, c.DA, true, c);
  __syncthreads();
  TP_MARK(15);
  // q input (rep) back into QB for dW_q
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      RT r_;
      ld_g_f(rep, c.tok0, rt, c.NR, r_, lane);
      st_tm_m(c.QB, rt, r_, row_mask(rt, c.NR, lane), lane);
    }
  }
  __syncthreads();
  wgrad_tm(c.DQ, c.QB, c.NRP, c.g(m[4].dW), c.wave, lane);
  wgrad_tm(c.KB, c.XB, c.NRP, c.g(m[5].dW), c.wave, lane);
  wgrad_tm(c.VB, c.XB, c.NRP, c.g(m[6].dW), c.wave, lane);
  TP_MARK(17);
  // d x1 = dk Wk + dv Wv ;  d rep += ds + dq Wq
  const bf16_t* dsrc[3] = {c.DQ, c.KB, c.VB};
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) rt_zero(dx[k]);
  }
#pragma unroll
  for (int mi = 0; mi < 3; ++mi) {
    BFr B;
    loadB(B, m[4 + mi].bw, lane);
    f32x4 dbb = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT gr, t;
        ld_tm(dsrc[mi], rt, gr, lane);
        colsum_acc(gr, dbb, vm);
        gemm_rt(t, dsrc[mi], rt, B, lane, false);
        if (mi == 0) {
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) dres[k].v[ct] += t.v[ct];
        } else {
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) dx[k].v[ct] += t.v[ct];
        }
      }
    }
    flush_cols(dbb, c.g(m[4 + mi].db), lane);
  }
  // d rep read-modify-write (each row owned by exactly one wave of one workgroup)
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      RT cur;
      ld_g_f(drep, c.tok0, rt, c.NR, cur, lane);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) cur.v[ct] += dres[k].v[ct];
      st_g_f(drep, c.tok0, rt, c.NR, cur, lane);
    }
  }
  __syncthreads();
}

// action head: logits = W_h2 · LN(GELU(W_h1 x + b)) + b  (ma_transformer.py:202-203,228), then per-row log-prob /
// entropy of the stored action: masked Categorical for discrete agents, Normal(column A-1) for the ratio agent
// (transformer_act.py:103-129).  A <= 8.
struct HeadRow { float lg[8]; };

__device__ __forceinline__ void head_logits(const DecP& p, const RT& n, float lg[8][4], int lane) {
  const int c16 = lane & 15;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    if (a < p.A) {
      RT t;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const float w = p.wh2[a * 64 + 16 * ct + c16];
#pragma unroll
        for (int r = 0; r < 4; ++r) t.v[ct][r] = n.v[ct][r] * w;
      }
      const f32x4 s = rowsum(t);
#pragma unroll
      for (int r = 0; r < 4; ++r) lg[a][r] = s[r] + p.bh2[a];
    }
  }
}

__device__ __forceinline__ float mask_logit(const DecP& p, int tok, int a, float l) {
  return (p.ava && p.ava[(size_t)tok * p.A + a] == 0.f) ? -1e10f : l;
}

// Per-row head inputs of one row tile (this lane's 4 C-layout rows), loaded at the top of the tile iteration so
// their L2 / HBM latency hides behind the head GEMM, GELU and LayerNorm instead of stalling the softmax (the
// section profiler put the head at 17 % of the decoder backward): availability as a bitmask, the taken action,
// and (backward) the log-prob / entropy gradients.
struct HeadRows { float act[4], dlp[4], den[4]; unsigned am[4]; };
__device__ __forceinline__ void head_rows(const DecP& p, const Ctx& c, int rt, int g, bool grads, HeadRows& h) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rt * 16 + 4 * g + r;
    const bool ok = row < c.NR;
    const int tok = c.tok0 + (ok ? row : 0);
    h.act[r] = p.act[tok];
    h.dlp[r] = grads && ok ? p.dlogp[tok] : 0.f;
    h.den[r] = grads && ok ? p.dent[tok] : 0.f;
    unsigned am = 0;
    if (p.ava) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
        if (a < p.A && p.ava[(size_t)tok * p.A + a] == 0.f) am |= 1u << a;
    }
    h.am[r] = am;
  }
}
__device__ __forceinline__ float mask_logit_m(unsigned am, int a, float l) { return ((am >> a) & 1u) ? -1e10f : l; }

// ============================================================================================== decoder forward
template <int NB, bool SAVE>
__device__ __forceinline__ void mat_dec_fwd_tile(const DecP& p, char* smem, int seq0, int nseq) {
  const Ctx c = make_ctx(p, smem, seq0, nseq);
  if (c.nseq <= 0) return;
  zero_lds(smem, mat_train_lds_bytes(p.NRP, p.SQ, p.L), c.tid);
  __syncthreads();
  const int lane = c.lane, g = lane >> 4;
  RT xr[MAXRT];
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      RT pre, xh;
      int tk[4];
      dec_embed_pre(p, rt, pre, tk, c);
      gelu_rt(pre);
      f32x4 mu, rs;
      ln_fwd(pre, xh, xr[k], mu, rs, p.lnd_g, p.lnd_b, lane);
    }
  }
#pragma unroll 1
  for (int b = 0; b < NB; ++b) {
    const Blk& B = p.blk[b];
    Ctx cc = c;
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    attn_self_fwd<SAVE>(B.m, B.ln[0], xr, p.sv[b], true, p.sv[b].xin, p.sv[b].a1, p.sv[b].lse1, cc);
    attn_cross_fwd<SAVE>(B.m, B.ln[1], xr, p.rep, p.sv[b].x1, p.sv[b].a2, p.sv[b].lse2, cc);
    mlp_fwd<SAVE>(B.m[8], B.m[9], B.ln[2], xr, p.sv[b].x2, p.sv[b].h, cc);
  }
  BFr Bh;
  loadB(Bh, p.h1.fw, lane);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      HeadRows hr;
      head_rows(p, c, rt, g, false, hr);
      st_tm_m(c.XB, rt, xr[k], row_mask(rt, c.NR, lane), lane);
      if (SAVE) { wave_lds_sync(); tile2g(p.sv_head, c.XB, rt, c); }
      wave_lds_sync();
      RT hh, xh, n;
      gemm_rt(hh, c.XB, rt, Bh, lane, false);
      add_bias(hh, p.h1.b, lane);
      gelu_rt(hh);
      f32x4 mu, rs;
      ln_fwd(hh, xh, n, mu, rs, p.lnh.g, p.lnh.b, lane);
      float lg[8][4];
      head_logits(p, n, lg, lane);
      if ((lane & 15) == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rt * 16 + 4 * g + r;
          if (row >= c.NR) continue;
          const int tok = c.tok0 + row, i = row % c.L;
          float lp, en;
          if (i < p.n_disc) {
            float mx = -INFINITY;
#pragma unroll
            for (int a = 0; a < 8; ++a) if (a < p.A) mx = fmaxf(mx, mask_logit_m(hr.am[r], a, lg[a][r]));
            float se = 0.f;
#pragma unroll
            for (int a = 0; a < 8; ++a) if (a < p.A) se += __expf(mask_logit_m(hr.am[r], a, lg[a][r]) - mx);
            const float lse = mx + __logf(se);
            const int act = min(max((int)hr.act[r], 0), p.A - 1);
            float H = 0.f, la = 0.f;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
              if (a < p.A) {
                const float l = mask_logit_m(hr.am[r], a, lg[a][r]) - lse;
                const float pr = __expf(l);
                H -= pr * l;
                if (a == act) la = l;
              }
            }
            lp = la;
            en = H;
          } else {
            const int a = p.A - 1;
            float mean = 0.f;
#pragma unroll
            for (int aa = 0; aa < 8; ++aa) if (aa == a) mean = lg[aa][r];
            const float sd = p.stdv[a], z = (hr.act[r] - mean) / sd;
            lp = -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
            en = 0.5f + 0.91893853320467274f + __logf(sd);
          }
          p.logp[tok] = lp;
          p.ent[tok] = en;
        }
      }
    }
  }
}

template <int NB, bool SAVE>
__global__ __launch_bounds__(256, WGPC) void MDL_V(mat_dec_fwd)(DecP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FOR_TILES(p, (mat_dec_fwd_tile<NB, SAVE>(p, smem, s0, ns)));
}

// ============================================================================================== decoder backward
template <int NB>
__device__ __forceinline__ void mat_dec_bwd_tile(const DecP& p, char* smem, int seq0, int nseq) {
  const Ctx c = make_ctx(p, smem, seq0, nseq);
  if (c.nseq <= 0) return;
  TP_DECL();
  zero_lds(smem, mat_train_lds_bytes(p.NRP, p.SQ, p.L), c.tid);
  __syncthreads();
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  RT dx[MAXRT];
  // ---------------- head backward (head input = last block output, saved in sv[NB-1].xin by the forward)
  {
    f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0}, dbh = {0, 0, 0, 0};
    f32x4 dwh2[8];
    float dbh2[8], dls = 0.f;
#pragma unroll
    for (int a = 0; a < 8; ++a) { dwh2[a] = f32x4{0, 0, 0, 0}; dbh2[a] = 0.f; }
    BFr Bf, Bb;
    loadB(Bf, p.h1.fw, lane);
    loadB(Bb, p.h1.bw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        HeadRows hr;
        head_rows(p, c, rt, g, true, hr);
        const f32x4 vm = row_mask(rt, c.NR, lane);
        g2tile(c.XB, p.sv_head, rt, c);
        wave_lds_sync();
        RT hh, gl, xh, n, dn, dgg;
        gemm_rt(hh, c.XB, rt, Bf, lane, false);
        add_bias(hh, p.h1.b, lane);
        gl = hh;
        gelu_rt(gl);
        f32x4 mu, rs;
        ln_fwd(gl, xh, n, mu, rs, p.lnh.g, p.lnh.b, lane);
        float lg[8][4];
        head_logits(p, n, lg, lane);
        float dz[8][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rt * 16 + 4 * g + r;
          const bool ok = row < c.NR;
          const int tok = c.tok0 + (ok ? row : 0), i = row % c.L;
          const float dlp = hr.dlp[r], den = hr.den[r];
#pragma unroll
          for (int a = 0; a < 8; ++a) dz[a][r] = 0.f;
          if (!ok) continue;
          if (i < p.n_disc) {
            float mx = -INFINITY;
#pragma unroll
            for (int a = 0; a < 8; ++a) if (a < p.A) mx = fmaxf(mx, mask_logit_m(hr.am[r], a, lg[a][r]));
            float se = 0.f;
#pragma unroll
            for (int a = 0; a < 8; ++a) if (a < p.A) se += __expf(mask_logit_m(hr.am[r], a, lg[a][r]) - mx);
            const float lse = mx + __logf(se);
            const int act = min(max((int)hr.act[r], 0), p.A - 1);
            float H = 0.f;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
              if (a < p.A) {
                const float l = mask_logit_m(hr.am[r], a, lg[a][r]) - lse;
                H -= __expf(l) * l;
              }
            }
#pragma unroll
            for (int a = 0; a < 8; ++a) {
              if (a < p.A) {
                const float l = mask_logit_m(hr.am[r], a, lg[a][r]) - lse;
                const float pr = __expf(l);
                dz[a][r] = dlp * ((a == act ? 1.f : 0.f) - pr) - den * pr * (l + H);
              }
            }
          } else {
            const int a = p.A - 1;
            float mean = 0.f;
#pragma unroll
            for (int aa = 0; aa < 8; ++aa) if (aa == a) mean = lg[aa][r];
            const float sd = p.stdv[a], diff = hr.act[r] - mean;
#pragma unroll
            for (int aa = 0; aa < 8; ++aa) if (aa == a) dz[aa][r] = dlp * diff / (sd * sd);
            if (c16 == 0) {
              const float dsd = dlp * (diff * diff / (sd * sd * sd) - 1.f / sd) + den / sd;
              const float sg = 1.f / (1.f + __expf(-p.log_std[a]));
              dls += dsd * 0.5f * sg * (1.f - sg);
            }
          }
        }
        rt_zero(dn);
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          if (a < p.A) {
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) {
              const float w = p.wh2[a * 64 + 16 * ct + c16];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                dn.v[ct][r] += dz[a][r] * w;
                dwh2[a][ct] += dz[a][r] * n.v[ct][r];
              }
            }
            if (c16 == 0) dbh2[a] += dz[a][0] + dz[a][1] + dz[a][2] + dz[a][3];
          }
        }
        ln_bwd(dn, xh, rs, p.lnh.g, dgg, dlg, dlb, vm, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) dgg.v[ct][r] *= gelu_erf_grad(hh.v[ct][r]) * vm[r];
        colsum_acc(dgg, dbh, vm);
        st_tm_m(c.DQ, rt, dgg, vm, lane);
        wave_lds_sync();
        gemm_rt(dx[k], c.DQ, rt, Bb, lane, false);
      }
    }
    flush_ln(dlg, dlb, p.lnh, c);
    flush_cols(dbh, c.g(p.h1.db), lane);
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (a < p.A) {
        flush_cols(dwh2[a], c.g(p.d_wh2 ? p.d_wh2 + a * 64 : nullptr), lane);
        float x = dbh2[a];
        x = cross_row_sum(x);
        if (lane == 0 && p.d_bh2) atomicAdd(c.g(p.d_bh2) + a, x);
      }
    }
    {
      float x = dls;
      x = cross_row_sum(x);
      if (lane == 0 && p.d_log_std) atomicAdd(c.g(p.d_log_std) + (p.A - 1), x);
    }
    __syncthreads();
    wgrad_tm(c.DQ, c.XB, c.NRP, c.g(p.h1.dW), c.wave, lane);
    __syncthreads();
  }
  TP_MARK(11);
  // ---------------- blocks in reverse
#pragma unroll 1
  for (int bb = NB - 1; bb >= 0; --bb) {
    const Blk& B = p.blk[bb];
    Ctx cc = c;
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    TP_DECL();
    mlp_bwd(B.m[8], B.m[9], B.ln[2], dx, p.sv[bb].x2, p.sv[bb].h, cc);
    TP_MARK(8);
    attn_cross_bwd(B.m, B.ln[1], dx, p.rep, p.drep, p.sv[bb].x1, p.sv[bb].a2, p.sv[bb].lse2, cc);
    TP_MARK(9);
    attn_self_bwd(B.m, B.ln[0], dx, p.sv[bb].xin, p.sv[bb].a1, p.sv[bb].lse1, true, cc);
    TP_MARK(10);
  }
  // ---------------- embedding backward: dW_a[:, token] += dpre ; LN_dec params
  {
    float* EMB = c.LSE;  // reuse: [(A+1)][64] f32 accumulators (A+1 <= 9 -> 2.3 KB <= LSE/DEL space)
    for (int i = c.tid; i < (p.A + 1) * 64; i += 256) EMB[i] = 0.f;
    __syncthreads();
    f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT pre, e, xh, y, de;
        int tk[4];
        dec_embed_pre(p, rt, pre, tk, c);
        e = pre;
        gelu_rt(e);
        f32x4 mu, rs;
        ln_fwd(e, xh, y, mu, rs, p.lnd_g, p.lnd_b, lane);
        ln_bwd(dx[k], xh, rs, p.lnd_g, de, dlg, dlb, vm, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = de.v[ct][r] * gelu_erf_grad(pre.v[ct][r]) * vm[r];
            if (vm[r] != 0.f) atomicAdd(EMB + tk[r] * 64 + 16 * ct + c16, v);
          }
      }
    }
    flush_ln(dlg, dlb, LNp{nullptr, nullptr, p.d_lnd_g, p.d_lnd_b}, c);
    __syncthreads();
    if (p.d_wa)
      for (int i = c.tid; i < (p.A + 1) * 64; i += 256) {
        const int t = i / 64, col = i % 64;
        atomicAdd(c.g(p.d_wa) + col * (p.A + 1) + t, EMB[i]);
      }
  }
}

template <int NB>
__global__ __launch_bounds__(256, WGPC) void MDL_V(mat_dec_bwd)(DecP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FOR_TILES(p, (mat_dec_bwd_tile<NB>(p, smem, s0, ns)));
}


MDL_API int MDL_V(mdl_mat_dec_fwd)(const DecP* p, int NB, int save, hipStream_t st) {
  if (p->A > 8 || p->A < 1) return -1;
  if (NB == 1) return save ? launch(MDL_V(mat_dec_fwd)<1, true>, p, st) : launch(MDL_V(mat_dec_fwd)<1, false>, p, st);
  if (NB == 2) return save ? launch(MDL_V(mat_dec_fwd)<2, true>, p, st) : launch(MDL_V(mat_dec_fwd)<2, false>, p, st);
  if (NB == 3) return save ? launch(MDL_V(mat_dec_fwd)<3, true>, p, st) : launch(MDL_V(mat_dec_fwd)<3, false>, p, st);
  return -3;
}

MDL_API int MDL_V(mdl_mat_dec_bwd)(const DecP* p, int NB, hipStream_t st) {
  if (p->A > 8 || p->A < 1) return -1;
  if (NB == 1) return launch(MDL_V(mat_dec_bwd)<1>, p, st);
  if (NB == 2) return launch(MDL_V(mat_dec_bwd)<2>, p, st);
  if (NB == 3) return launch(MDL_V(mat_dec_bwd)<3>, p, st);
  return -3;
}

#ifdef MDL_TRAIN_PROF
MDL_API int mdl_dec_prof_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tprof), sizeof(unsigned long long) * 32, 0, hipMemcpyDeviceToHost);
}
#endif
