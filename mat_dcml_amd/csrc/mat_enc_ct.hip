// Fused MAT encoder forward / backward, token-on-lane tiles (mat_train_ct.h).  Reference: ma_transformer.py:72-92
// (EncodeBlock), :119-154 (Encoder: obs_encoder = LN(obs_dim) -> Linear -> GELU, ln, blocks, value head).
//
// Observation embedding: obs_dim <= 16 runs in-kernel (LN_obs per lane, W_e on MFMA with a hi/lo split of the
// LN output); larger observations (SMAC: 1288) come in as the embedding pre-activation `pre_in` computed by the
// obs-embedding GEMM kernels (obs_embed.hip), and the backward hands d pre back through `dpre_out`.
#include "mat_train_ct.h"

namespace {

struct EncX {   // EncP extension of the round-2 kernels (passed next to EncP)
  const float* pre_in;   // [tok][64] embedding pre-activation (null: embed obs in-kernel, obs_dim <= 16)
  float* dpre_out;       // [tok][64] gradient w.r.t. pre_in (backward, when pre_in is used)
};

// LN_obs of this lane's token: lane (g, c) loads and normalises only its 4 dims 4g .. 4g+3 (od <= 16), the token's
// mean / variance reduce across the 4 lane rows (two-pass, as torch's LayerNorm); -> this lane's 4 dims of the LN
// output and x-hat.  Padded rows read zeros (finite x-hat 0, output = beta).
__device__ __forceinline__ void obs_ln(const EncP& p, int rt, const Ctx& c, float oh[4], float hat[4]) {
  const int lane = c.lane, g = lane >> 4, od = p.od;
  const int row = rt * 16 + (lane & 15);
  const bool ok = row < c.NR;
  const float* src = p.obs + src_tok(p.sidx, (size_t)(c.tok0 + (ok ? row : 0)), c.L) * od;
  float o[4];
  bool in[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kk = 4 * g + j;
    in[j] = kk < od;
    o[j] = (ok && in[j]) ? src[kk] : 0.f;
  }
  const float mean = cross_row_sum((o[0] + o[1]) + (o[2] + o[3])) / (float)od;
  float d[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) d[j] = in[j] ? o[j] - mean : 0.f;
  const float var = cross_row_sum((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]));
  const float rstd = rsqrtf(var / (float)od + 1e-5f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ks = in[j] ? 4 * g + j : 0;
    hat[j] = d[j] * rstd;
    oh[j] = in[j] ? hat[j] * p.lno_g[ks] + p.lno_b[ks] : 0.f;
  }
}

// W_e (64 x od, fp32) as A fragments: rows 16mt + (lane&15), k = obs dim 4g + j (j < 4; j >= 4 -> dims >= 16: 0)
__device__ __forceinline__ void we_frags(const EncP& p, bf16x8 W[4], int lane) {
  const int c16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 4 * g + j;
      const bool in = j < 4 && kk < p.od;
      const float w = p.we[(16 * mt + c16) * p.od + (in ? kk : 0)];
      W[mt][j] = (short)f2bf(in ? w : 0.f);
    }
}
// W_eᵀ as A fragments for d(LN_obs out) = W_eᵀ d pre: rows = obs dim (lane&15), k = features perm(s, g, j)
__device__ __forceinline__ void weT_frags(const EncP& p, bf16x8 W[2], int lane) {
  const int c16 = lane & 15, g = lane >> 4;
  const bool in = c16 < p.od;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
      const float w = p.we[f * p.od + (in ? c16 : 0)];
      W[s][j] = (short)f2bf(in ? w : 0.f);
    }
}

__device__ __forceinline__ CT embed_pre(const EncP& p, const EncX& x, int rt, const bf16x8 W[4], float oh[4], float hat[4],
                                        const Ctx& c) {
  if (x.pre_in) return ld_gf(x.pre_in, c.tok0, rt, c.NR, c.lane);
  obs_ln(p, rt, c, oh, hat);
  const uint32_t h01 = pk2(oh[0], oh[1]), h23 = pk2(oh[2], oh[3]);
  const uint32_t l01 = pk2(oh[0] - blo(h01), oh[1] - bhi(h01)), l23 = pk2(oh[2] - blo(h23), oh[3] - bhi(h23));
  const bf16x8 bh = mk8(h01, h23, 0u, 0u), bl = mk8(l01, l23, 0u, 0u);
  CT pre = ld_vec(p.be, c.lane);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    pre.v[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W[mt], bh, pre.v[mt], 0, 0, 0);
    pre.v[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W[mt], bl, pre.v[mt], 0, 0, 0);
  }
  return pre;
}

// ============================================================================================== forward
template <int NB, bool SAVE>
__device__ __forceinline__ void enc_fwd_tile(const EncP& p, const EncX& ex, char* smem, int seq0, int nseq) {
  const Ctx c = make_ctx(p, smem, seq0, nseq);
  if (c.nseq <= 0) return;
  zero_pad_rows_fwd(c);
  __syncthreads();
  CP_MARK(0);
  const int lane = c.lane, g = lane >> 4;
  CT xr[MAXRT];
  {
    bf16x8 W[4];
    if (!ex.pre_in) we_frags(p, W, lane);
    const CT gam = ld_vec(p.ln0_g, lane), bet = ld_vec(p.ln0_b, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        float oh[4], hat[4];
        CT pre = embed_pre(p, ex, rt, W, oh, hat, c), xh;
        if (SAVE) {   // x-hat, GELU'(pre), rstd for the backward (which recomputes none of the embedding forward)
          CT gp;
          gelu_ct_both(pre, gp);
          const float rs = ln_fwd_ct(pre, xh, xr[k], gam, bet);
          st_g(p.es.xh, c.tok0, rt, c.NR, ct_pack(xh), lane);
          st_g(p.es.gp, c.tok0, rt, c.NR, ct_pack(gp), lane);
          st_tokf(p.es.rs, rt, rs, c);
        } else {
          gelu_ct(pre);
          ln_fwd_ct(pre, xh, xr[k], gam, bet);
        }
      }
    }
  }
  CP_MARK(28);
#pragma unroll 1
  for (int b = 0; b < NB; ++b) {
    const Blk& B = p.blk[b];
    Ctx cc = c;   // opaque per-iteration lane id: keeps hipcc from hoisting (and spilling) every LDS address
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    self_attn_fwd_ct<SAVE>(B.m, B.ln[0], xr, false, p.sv[b].xin, p.sv[b].a1, p.sv[b].a1lo, p.sv[b].lse1,
                           p.sv[b].xh[0], p.sv[b].rs + 0 * (size_t)p.Bs * p.L, cc);
    mlp_fwd_ct<SAVE>(B.m[8], B.m[9], B.ln[1], xr, p.sv[b].x1, p.sv[b].g, p.sv[b].gp, p.sv[b].xh[1], p.sv[b].rs + 1 * (size_t)p.Bs * p.L, cc);
  }
  // value head: v = W_v2 · LN(GELU(W_v1 · rep + b)) + b   (ma_transformer.py:138-139,152)
  AFr H;
  loadA(H, p.h1.fa, lane);
  const CT bh = ld_vec(p.h1.b, lane), gam = ld_vec(p.lnh.g, lane), bet = ld_vec(p.lnh.b, lane);
  const CT w0 = ld_vec(p.wh2, lane);
  CT w1;
  if (p.n_obj > 1) w1 = ld_vec(p.wh2 + 64, lane); else ct_zero(w1);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + NW * k;
    if (rt < c.NT) {
      const bool ok = tok_ok(rt, c);
      if (p.rep) st_gf(p.rep, c.tok0, rt, c.NR, xr[k], lane);
      CT hh = bh, xh, n;
      mm(hh, H, ct_pack(xr[k]));
      if (SAVE) {   // x-hat, GELU'(h), rstd for the backward
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
      f32x4 t0 = n.v[0] * w0.v[0], t1 = n.v[0] * w1.v[0];   // packed pairs, then both row sums side by side
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        t0 = n.v[i] * w0.v[i] + t0;
        t1 = n.v[i] * w1.v[i] + t1;
      }
      float s0 = (t0[0] + t0[1]) + (t0[2] + t0[3]), s1 = (t1[0] + t1[1]) + (t1[2] + t1[3]);
      {
        float a0, a1, b0, b1;
        swap16(s0, a0, a1);
        swap16(s1, b0, b1);
        s0 = a0 + a1;
        s1 = b0 + b1;
        swap32(s0, a0, a1);
        swap32(s1, b0, b1);
        s0 = a0 + a1;
        s1 = b0 + b1;
      }
      if (ok && g == 0) {
        const size_t tok = (size_t)(c.tok0 + rt * 16 + (lane & 15));
        p.v[tok * p.n_obj] = s0 + p.bh2[0];
        if (p.n_obj > 1) p.v[tok * p.n_obj + 1] = s1 + p.bh2[1];
      }
    }
  }
  CP_MARK(27);
}

#ifndef MDL_CT_BWD_TU
template <int NB, bool SAVE>
__global__ __launch_bounds__(NTHR, FWD_WGPC) void mat_enc_fwd_ct(EncP p, EncX ex) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CP_BEGIN();
  FOR_TILES(p, (enc_fwd_tile<NB, SAVE>(p, ex, smem, s0, ns)));
  CP_END();
}

#endif  // !MDL_CT_BWD_TU

// ============================================================================================== backward
template <int NB>
__device__ __forceinline__ void enc_bwd_tile(const EncP& p, const EncX& ex, char* smem, int seq0, int nseq, bool first) {
  const Ctx c = make_ctx(p, smem, seq0, nseq, first);
  if (c.nseq <= 0) return;
  zero_pad_rows(c);
  __syncthreads();
  CP_MARK(0);
  const int lane = c.lane;
  CT dx[MAXRT];
  // ---------------- value head backward (+ incoming d rep from the decoder)
  {
    CT dlg, dlb, dw0, dw1;
    ct_zero(dlg);
    ct_zero(dlb);
    ct_zero(dw0);
    ct_zero(dw1);
    // the forward's x-hat, GELU'(h) and rstd of the head (no W_h1 product, GELU or LayerNorm forward here); every
    // tile's loads requested up front (one latency, not three)
    CTr hxh[MAXRT], hgp[MAXRT];
    float hrs[MAXRT], dv0s[MAXRT], dv1s[MAXRT];
    {
      CT reps[MAXRT];
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          reps[k] = ld_gf(p.rep, c.tok0, rt, c.NR, lane);
          hxh[k] = ld_g(p.hs.xh, c.tok0, rt, c.NR, lane);
          hgp[k] = ld_g(p.hs.gp, c.tok0, rt, c.NR, lane);
          hrs[k] = ld_tokf(p.hs.rs, rt, c);
          const bool ok = tok_ok(rt, c);
          const size_t tok = (size_t)(c.tok0 + (ok ? rt * 16 + (lane & 15) : 0));
          dv0s[k] = ok ? p.dv[tok * p.n_obj] : 0.f;
          dv1s[k] = (ok && p.n_obj > 1) ? p.dv[tok * p.n_obj + 1] : 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) st_lds(c.XB, rt, ct_pack(reps[k]), tok_ok(rt, c), lane);   // X of W_h1
      }
    }
    const CT gam = ld_vec(p.lnh.g, lane), bet = ld_vec(p.lnh.b, lane);
    const CT w0 = ld_vec(p.wh2, lane);
    CT w1;
    if (p.n_obj > 1) w1 = ld_vec(p.wh2 + 64, lane); else ct_zero(w1);
    float sdv0 = 0.f, sdv1 = 0.f;   // Σ dv of this lane's tokens (value-head bias gradient)
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const bool ok = tok_ok(rt, c);
        const float dv0 = dv0s[k], dv1 = dv1s[k];
        sdv0 += dv0;
        sdv1 += dv1;
        const CT xh = ct_unpack(hxh[k]), ggp = ct_unpack(hgp[k]);
        CT n, dn, dg;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          n.v[i] = xh.v[i] * gam.v[i] + bet.v[i];
          dn.v[i] = dv0 * w0.v[i] + dv1 * w1.v[i];
          dw0.v[i] += dv0 * n.v[i];
          dw1.v[i] += dv1 * n.v[i];
        }
        ln_bwd_ct(dn, xh, hrs[k], gam, ok, dg, dlg, dlb);
#pragma unroll
        for (int i = 0; i < 4; ++i) dg.v[i] *= ggp.v[i];   // padded rows: x-hat, GELU' and rstd are zero
        st_lds(c.DQ, rt, ct_pack(dg), ok, lane);   // dY of W_h1
      }
    }
    {   // second pass (W_h1ᵀ): dx = d rep (from the decoder) + W_h1ᵀ dY
      AFr Hb;
      loadA(Hb, p.h1.ba, lane);
#pragma unroll
      for (int k = 0; k < MAXRT; ++k) {
        const int rt = c.wave + NW * k;
        if (rt < c.NT) {
          CT t = ld_gf(p.drep, c.tok0, rt, c.NR, lane);
          mm(t, Hb, ld_lds(c.DQ, rt, lane));
          dx[k] = t;
        }
      }
    }
    // parameter-vector slots (vacc): 0-1 head LayerNorm, 2-3 value-head rows, 4 value-head bias, 5-6 embedding
    // LayerNorm, 7 embedding bias, 8-9 observation LayerNorm, 10 + 4 bb + 2 k the block's k-th LayerNorm
    flush_vec(dlg, c.g(p.lnh.dg), 0, c);
    flush_vec(dlb, c.g(p.lnh.db), 1, c);
    flush_vec(dw0, c.g(p.d_wh2), 2, c);
    if (p.n_obj > 1) flush_vec(dw1, c.g(p.d_wh2 ? p.d_wh2 + 64 : nullptr), 3, c);
    if (p.d_bh2) {   // lanes g = 0 carry each token once
      const float s0 = group_sum<16>(sdv0), s1 = group_sum<16>(sdv1);
      if (lane == 0) {
        vacc_add(c.g(p.d_bh2), 4, 0, s0, c, p.n_obj);
        if (p.n_obj > 1) vacc_add(c.g(p.d_bh2), 4, 1, s1, c, p.n_obj);
      }
    }
    __syncthreads();
    wgrad64(c.DQ, c.XB, p.h1, c);
    __syncthreads();
    CP_MARK(1);
  }
  // ---------------- blocks in reverse
#pragma unroll 1
  for (int bb = NB - 1; bb >= 0; --bb) {
    const Blk& B = p.blk[bb];
    Ctx cc = c;
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    mlp_bwd_ct(B.m[8], B.m[9], B.ln[1], dx, p.sv[bb].x1, p.sv[bb].g, p.sv[bb].gp, p.sv[bb].xh[1], p.sv[bb].rs + 1 * (size_t)p.Bs * p.L, cc,
               12 + 4 * bb);
    self_attn_bwd_ct(B.m, B.ln[0], dx, p.sv[bb].xin, p.sv[bb].a1, p.sv[bb].a1lo, p.sv[bb].lse1, p.sv[bb].xh[0],
                     p.sv[bb].rs + 0 * (size_t)p.Bs * p.L, false, cc, 10 + 4 * bb);
  }
  // ---------------- embedding backward: x0 = LN0(GELU(pre)), pre = W_e · LN_obs(obs) + b_e
  {
    CT dlg, dlb, dbe;
    ct_zero(dlg);
    ct_zero(dlb);
    ct_zero(dbe);
    f32x4 dog = {0.f, 0.f, 0.f, 0.f}, dob = {0.f, 0.f, 0.f, 0.f};
    bf16x8 WT[2];
    if (!ex.pre_in) weT_frags(p, WT, lane);
    const CT gam = ld_vec(p.ln0_g, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + NW * k;
      if (rt < c.NT) {
        const bool ok = tok_ok(rt, c);
        float oh[4] = {0.f, 0.f, 0.f, 0.f}, hat[4] = {0.f, 0.f, 0.f, 0.f};
        if (!ex.pre_in) obs_ln(p, rt, c, oh, hat);   // X of W_e and the LN_obs backward (od <= 16 dims in-lane)
        // the forward's x-hat, GELU'(pre) and rstd (no embedding product, GELU or LayerNorm forward here)
        const CT xh = ct_unpack(ld_g(p.es.xh, c.tok0, rt, c.NR, lane)), egp = ct_unpack(ld_g(p.es.gp, c.tok0, rt, c.NR, lane));
        CT de;
        ln_bwd_ct(dx[k], xh, ld_tokf(p.es.rs, rt, c), gam, ok, de, dlg, dlb);
#pragma unroll
        for (int i = 0; i < 4; ++i) de.v[i] *= egp.v[i];   // padded rows: zero
        if (ex.pre_in) {
          st_gf(ex.dpre_out, c.tok0, rt, c.NR, de, lane);
          continue;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dbe.v[i] += de.v[i];
        CTr dh, dl;
        ct_split(de, dh, dl);
        st_lds(c.DA, rt, dh, ok, lane);   // dY of W_e
        CTr xo = ct_zero_r();
        xo.q[0] = make_uint2(pk2(oh[0], oh[1]), pk2(oh[2], oh[3]));
        st_lds(c.XB, rt, xo, ok, lane);   // X of W_e (obs dims 0..15 = features 0..15 of the LDS row)
        // d(LN_obs output)[dim 4g + r] of this lane's token
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WT[s], rb(dh, s), d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(WT[s], rb(dl, s), d, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dog[r] += ok ? d[r] * hat[r] : 0.f;
          dob[r] += ok ? d[r] : 0.f;
        }
      }
    }
    flush_vec(dlg, c.g(p.d_ln0_g), 5, c);
    flush_vec(dlb, c.g(p.d_ln0_b), 6, c);
    if (!ex.pre_in) {
      flush_vec(dbe, c.g(p.d_be), 7, c);
      const int c16 = lane & 15, g = lane >> 4;
      float og = 0.f, ob = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = group_sum<16>(dog[r]), b = group_sum<16>(dob[r]);
        og = c16 == r ? a : og;
        ob = c16 == r ? b : ob;
      }
      const int dim = 4 * g + c16;
      if (c16 < 4 && dim < p.od) {
        if (p.d_lno_g) vacc_add(c.g(p.d_lno_g), 8, dim, og, c, p.od);
        if (p.d_lno_b) vacc_add(c.g(p.d_lno_b), 9, dim, ob, c, p.od);
      }
      __syncthreads();
      wgrad_g(c.DA, c.XB, c.KP, c.g(p.d_we), p.od, 64, p.od, nullptr, c.wave, lane, c.gm);
    }
  }
  CP_MARK(30);
}

#ifdef MDL_CT_BWD_TU
template <int NB>
__global__ __launch_bounds__(NTHR, WGPC) void mat_enc_bwd_ct(EncP p, EncX ex) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CP_BEGIN();
  vacc_begin(p, smem);
  FOR_TILES(p, (enc_bwd_tile<NB>(p, ex, smem, s0, ns, it_ == 0)));
  vacc_end(p, smem);
  CP_END();
}

#endif  // MDL_CT_BWD_TU

}  // namespace

// ============================================================================================== host API
#ifndef MDL_CT_BWD_TU
MDL_API int mdl_mat_train_geometry_ct(int L) {
  const int MAXROWS = 16 * NW * MAXRT;   // row tiles of one round of the forward's waves
  int SQ = MAXROWS / L;
  if (SQ < 1) return 0;
  int NRP = ((SQ * L + 31) / 32) * 32;
  if (NRP < 64) NRP = 64;
  while (SQ > 1 && (NRP > MAXROWS || mat_train_lds_bytes(NRP, SQ, L) > LDS_BUDGET)) {
    --SQ;
    NRP = ((SQ * L + 31) / 32) * 32;
    if (NRP < 64) NRP = 64;
  }
  if (mat_train_lds_bytes(NRP, SQ, L) > LDS_BUDGET || (SQ * L + 15) / 16 > 4 * MAXRT) return 0;
  return SQ | (NRP << 16);
}

// workgroups of a backward launch over Bs sequences in tiles of SQ (= the private gradient copies it writes)
MDL_API int mdl_ct_bwd_grid(int Bs, int SQ) {
  const int tiles = (Bs + SQ - 1) / SQ, cap = n_cus();
  return tiles < cap ? tiles : cap;
}

MDL_API int mdl_mat_enc_fwd_ct(const EncP* p, const float* pre_in, int NB, int save, hipStream_t st) {
  if ((!pre_in && (p->od > 16 || p->od < 1)) || p->n_obj > 2 || p->n_obj < 1) return -1;
  const EncX ex{pre_in, nullptr};
  if (NB == 1) return save ? launch_ct(mat_enc_fwd_ct<1, true>, p, true, st, ex) : launch_ct(mat_enc_fwd_ct<1, false>, p, true, st, ex);
  if (NB == 2) return save ? launch_ct(mat_enc_fwd_ct<2, true>, p, true, st, ex) : launch_ct(mat_enc_fwd_ct<2, false>, p, true, st, ex);
  if (NB == 3) return save ? launch_ct(mat_enc_fwd_ct<3, true>, p, true, st, ex) : launch_ct(mat_enc_fwd_ct<3, false>, p, true, st, ex);
  return -3;
}

#else
MDL_API int mdl_mat_enc_bwd_ct(const EncP* p, const float* pre_in, float* dpre_out, int NB, hipStream_t st) {
  if ((!pre_in && (p->od > 16 || p->od < 1)) || p->n_obj > 2 || p->n_obj < 1 || (pre_in && !dpre_out)) return -1;
  const EncX ex{pre_in, dpre_out};
  if (NB == 1) return launch_ct(mat_enc_bwd_ct<1>, p, false, st, ex);
  if (NB == 2) return launch_ct(mat_enc_bwd_ct<2>, p, false, st, ex);
  if (NB == 3) return launch_ct(mat_enc_bwd_ct<3>, p, false, st, ex);
  return -3;
}
#endif  // MDL_CT_BWD_TU

#ifdef MDL_CT_PROF
MDL_API int MDL_CAT(mdl_ctprof_enc, MDL_CT_TU_SUFFIX)(unsigned long long* out, int reset) {
  if (reset) {
    unsigned long long z[64] = {0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ctprof), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ctprof), sizeof(unsigned long long) * 64, 0, hipMemcpyDeviceToHost);
}
#endif
