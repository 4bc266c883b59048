// Fused MAT encoder forward / backward kernels (see mat_train_common.h for the design).
#include "mat_train_common.h"

// ============================================================================================== encoder forward
template <int NB, bool SAVE>
__device__ __forceinline__ void mat_enc_fwd_tile(const EncP& p, char* smem, int seq0, int nseq) {
  const Ctx c = make_ctx(p, smem, seq0, nseq);
  if (c.nseq <= 0) return;
  zero_lds(smem, mat_train_lds_bytes(p.NRP, p.SQ, p.L), c.tid);
  __syncthreads();
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  RT xr[MAXRT];
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      RT pre, xh;
      float* ES = emb_scratch(c);
      embed_stage(p, rt, ES, c);
      embed_pre(p, rt, pre, ES, c);
      gelu_rt(pre);
      f32x4 mu, rs;
      ln_fwd(pre, xh, xr[k], mu, rs, p.ln0_g, p.ln0_b, lane);
    }
  }
#pragma unroll 1
  for (int b = 0; b < NB; ++b) {
    const Blk& B = p.blk[b];
    Ctx cc = c;   // opaque per-iteration lane id: keeps hipcc from hoisting (and spilling) every LDS address
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    attn_self_fwd<SAVE>(B.m, B.ln[0], xr, p.sv[b], false, p.sv[b].xin, p.sv[b].a1, p.sv[b].lse1, cc);
    mlp_fwd<SAVE>(B.m[8], B.m[9], B.ln[1], xr, p.sv[b].x1, p.sv[b].h, cc);
  }
  // value head: v = W_v2 · LN(GELU(W_v1 · rep + b)) + b   (ma_transformer.py:138-139,152)
  BFr Bh;
  loadB(Bh, p.h1.fw, lane);
#pragma unroll
  for (int k = 0; k < MAXRT; ++k) {
    const int rt = c.wave + 4 * k;
    if (rt < c.NT) {
      st_tm_m(c.XB, rt, xr[k], row_mask(rt, c.NR, lane), lane);
      if (p.rep) st_g_f(p.rep, c.tok0, rt, c.NR, xr[k], lane);
      wave_lds_sync();
      RT hh, xh, n;
      gemm_rt(hh, c.XB, rt, Bh, lane, false);
      add_bias(hh, p.h1.b, lane);
      gelu_rt(hh);
      f32x4 mu, rs;
      ln_fwd(hh, xh, n, mu, rs, p.lnh.g, p.lnh.b, lane);
      for (int o = 0; o < p.n_obj; ++o) {
        RT t;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const float w = p.wh2[o * 64 + 16 * ct + c16];
#pragma unroll
          for (int r = 0; r < 4; ++r) t.v[ct][r] = n.v[ct][r] * w;
        }
        const f32x4 vs = rowsum(t);
        if (c16 == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rt * 16 + 4 * g + r;
            if (row < c.NR) p.v[(size_t)(c.tok0 + row) * p.n_obj + o] = vs[r] + p.bh2[o];
          }
        }
      }
    }
  }
}

template <int NB, bool SAVE>
__global__ __launch_bounds__(256, WGPC) void MDL_V(mat_enc_fwd)(EncP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FOR_TILES(p, (mat_enc_fwd_tile<NB, SAVE>(p, smem, s0, ns)));
}

// ============================================================================================== encoder backward
template <int NB>
__device__ __forceinline__ void mat_enc_bwd_tile(const EncP& p, char* smem, int seq0, int nseq) {
  const Ctx c = make_ctx(p, smem, seq0, nseq);
  if (c.nseq <= 0) return;
  zero_lds(smem, mat_train_lds_bytes(p.NRP, p.SQ, p.L), c.tid);
  __syncthreads();
  TP_DECL();
  const int lane = c.lane, g = lane >> 4, c16 = lane & 15;
  RT dx[MAXRT];
  // ---------------- value head backward (+ incoming d rep from the decoder)
  {
    f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0}, dbh = {0, 0, 0, 0}, dw2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    BFr Bf, Bb;
    loadB(Bf, p.h1.fw, lane);
    loadB(Bb, p.h1.bw, lane);
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT rep;
        ld_g_f(p.rep, c.tok0, rt, c.NR, rep, lane);
        st_tm_m(c.XB, rt, rep, vm, lane);   // X of dW_h1
        wave_lds_sync();
        RT hh, gl, xh, n, dn, dg;
        gemm_rt(hh, c.XB, rt, Bf, lane, false);
        add_bias(hh, p.h1.b, lane);
        gl = hh;
        gelu_rt(gl);
        f32x4 mu, rs;
        ln_fwd(gl, xh, n, mu, rs, p.lnh.g, p.lnh.b, lane);
        rt_zero(dn);
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          if (o >= p.n_obj) break;
          f32x4 dvv;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rt * 16 + 4 * g + r;
            dvv[r] = row < c.NR ? p.dv[(size_t)(c.tok0 + row) * p.n_obj + o] : 0.f;
          }
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) {
            const float w = p.wh2[o * 64 + 16 * ct + c16];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              dn.v[ct][r] += dvv[r] * w;
              dw2[o][ct] += dvv[r] * n.v[ct][r];
            }
          }
        }
        ln_bwd(dn, xh, rs, p.lnh.g, dg, dlg, dlb, vm, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) dg.v[ct][r] *= gelu_erf_grad(hh.v[ct][r]) * vm[r];
        colsum_acc(dg, dbh, vm);
        st_tm_m(c.DQ, rt, dg, vm, lane);    // dY of dW_h1
        wave_lds_sync();
        RT t, dr;
        gemm_rt(t, c.DQ, rt, Bb, lane, false);
        ld_g_f(p.drep, c.tok0, rt, c.NR, dr, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) dx[k].v[ct] = dr.v[ct] + t.v[ct];
      }
    }
    flush_ln(dlg, dlb, p.lnh, c);
    flush_cols(dbh, c.g(p.h1.db), lane);
    flush_cols(dw2[0], c.g(p.d_wh2), lane);
    if (p.n_obj > 1) flush_cols(dw2[1], c.g(p.d_wh2 ? p.d_wh2 + 64 : nullptr), lane);
    __syncthreads();
    wgrad_tm(c.DQ, c.XB, c.NRP, c.g(p.h1.dW), c.wave, lane);
    __syncthreads();
  TP_MARK(20);
  }
  // ---------------- blocks in reverse
#pragma unroll 1
  for (int bb = NB - 1; bb >= 0; --bb) {
    const Blk& B = p.blk[bb];
    Ctx cc = c;
    asm volatile("" : "+v"(cc.lane), "+v"(cc.tid));
    mlp_bwd(B.m[8], B.m[9], B.ln[1], dx, p.sv[bb].x1, p.sv[bb].h, cc);
    attn_self_bwd(B.m, B.ln[0], dx, p.sv[bb].xin, p.sv[bb].a1, p.sv[bb].lse1, false, cc);
  }
  TP_MARK(21);
  // ---------------- embedding backward: x0 = LN0(GELU(W_e · LN_obs(obs) + b_e))
  __syncthreads();   // QB becomes the per-wave LN_obs scratch
#ifndef MDL_ABLATE_EMB
  {
    f32x4 dlg = {0, 0, 0, 0}, dlb = {0, 0, 0, 0}, dbe = {0, 0, 0, 0};
    float dwe[4][16], dlog[16], dlob[16];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) dwe[ct][kk] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) { dlog[kk] = 0.f; dlob[kk] = 0.f; }
#ifndef MDL_ABLATE_DOH
    float wreg[4][16];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) wreg[ct][kk] = kk < p.od ? p.we[(16 * ct + c16) * p.od + kk] : 0.f;
#endif
#pragma unroll
    for (int k = 0; k < MAXRT; ++k) {
      const int rt = c.wave + 4 * k;
      if (rt < c.NT) {
        const f32x4 vm = row_mask(rt, c.NR, lane);
        RT pre, e, xh, y, de;
        const float* ES = emb_scratch(c);
        TP_MARK(29);
        embed_stage(p, rt, emb_scratch(c), c);
        TP_MARK(23);
        embed_pre(p, rt, pre, ES, c);
        TP_MARK(24);
        e = pre;
        gelu_rt(e);
        f32x4 mu, rs;
        ln_fwd(e, xh, y, mu, rs, p.ln0_g, p.ln0_b, lane);
        ln_bwd(dx[k], xh, rs, p.ln0_g, de, dlg, dlb, vm, lane);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) de.v[ct][r] *= gelu_erf_grad(pre.v[ct][r]) * vm[r];
        colsum_acc(de, dbe, vm);
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          if (4 * k4 < p.od) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const f32x4 oh = *(const f32x4*)(ES + (4 * g + r) * 32 + 4 * k4);
#pragma unroll
              for (int ct = 0; ct < 4; ++ct)
#pragma unroll
                for (int j = 0; j < 4; ++j) dwe[ct][4 * k4 + j] += de.v[ct][r] * oh[j];
            }
          }
        }
        TP_MARK(25);
        // d(LN_obs output)[row][kk] = sum_col dpre * W_e[col][kk]  -> LN_obs affine-parameter grads
#ifndef MDL_ABLATE_DOH
        // W_e columns of this lane in registers (loaded once per tile above), and the 16-lane reductions of
        // one row issued back to back — they were serialised behind per-(row, kk) global loads (24 % of
        // mat_enc_bwd in the section profile)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t[16];
#pragma unroll
          for (int kk = 0; kk < 16; ++kk) {
            t[kk] = 0.f;
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) t[kk] += de.v[ct][r] * wreg[ct][kk];
          }
#pragma unroll
          for (int kk = 0; kk < 16; ++kk)
            if (kk < p.od) t[kk] = group_sum<16>(t[kk]);
          if (c16 == 0) {
#pragma unroll
            for (int kk = 0; kk < 16; ++kk)
              if (kk < p.od) { dlog[kk] += t[kk] * ES[(4 * g + r) * 32 + 16 + kk]; dlob[kk] += t[kk]; }
          }
        }
#endif
        TP_MARK(26);
        wave_lds_sync();   // scratch reads done before the next tile's staging overwrites it
      }
    }
    TP_MARK(29);
    flush_ln(dlg, dlb, LNp{nullptr, nullptr, p.d_ln0_g, p.d_ln0_b}, c);
    flush_cols(dbe, c.g(p.d_be), lane);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        if (kk < p.od) {
          float x = dwe[ct][kk];
          x = cross_row_sum(x);
          if (g == 0 && p.d_we) atomicAdd(c.g(p.d_we) + (16 * ct + c16) * p.od + kk, x);
        }
      }
    TP_MARK(27);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      if (kk < p.od) {
        float a = dlog[kk], b2 = dlob[kk];
        a = cross_row_sum(a);
        b2 = cross_row_sum(b2);
        if (lane == 0) {
          if (p.d_lno_g) atomicAdd(c.g(p.d_lno_g) + kk, a);
          if (p.d_lno_b) atomicAdd(c.g(p.d_lno_b) + kk, b2);
        }
      }
    }
  }
#endif
  TP_MARK(22);
}

template <int NB>
__global__ __launch_bounds__(256, WGPC) void MDL_V(mat_enc_bwd)(EncP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FOR_TILES(p, (mat_enc_bwd_tile<NB>(p, smem, s0, ns)));
}



// ============================================================================================== host API
MDL_API int MDL_V(mdl_mat_train_geometry)(int L) {
  // sequences per tile: rows = SQ*L <= 4*MAXRT*16, LDS-padded rows a multiple of 32; returns SQ | NRP << 16
  const int MAXROWS = 64 * MAXRT;
  int SQ = MAXROWS / L;
  if (SQ < 1) return 0;
  int NRP = ((SQ * L + 31) / 32) * 32;
  if (NRP < 64) NRP = 64;   // QB doubles as the 4 x 2 KB LN_obs scratch of the embedding
  while (SQ > 1 && (NRP > MAXROWS || mat_train_lds_bytes(NRP, SQ, L) > LDS_BUDGET)) {
    --SQ;
    NRP = ((SQ * L + 31) / 32) * 32;
    if (NRP < 64) NRP = 64;
  }
  if (mat_train_lds_bytes(NRP, SQ, L) > LDS_BUDGET || (SQ * L + 15) / 16 > 4 * MAXRT) return 0;
  return SQ | (NRP << 16);
}

MDL_API int MDL_V(mdl_mat_enc_fwd)(const EncP* p, int NB, int save, hipStream_t st) {
  if (p->od > 16 || p->od < 1 || p->n_obj > 2) return -1;
  if (NB == 1) return save ? launch(MDL_V(mat_enc_fwd)<1, true>, p, st) : launch(MDL_V(mat_enc_fwd)<1, false>, p, st);
  if (NB == 2) return save ? launch(MDL_V(mat_enc_fwd)<2, true>, p, st) : launch(MDL_V(mat_enc_fwd)<2, false>, p, st);
  if (NB == 3) return save ? launch(MDL_V(mat_enc_fwd)<3, true>, p, st) : launch(MDL_V(mat_enc_fwd)<3, false>, p, st);
  return -3;
}

MDL_API int MDL_V(mdl_mat_enc_bwd)(const EncP* p, int NB, hipStream_t st) {
  if (p->od > 16 || p->od < 1 || p->n_obj > 2) return -1;
  if (NB == 1) return launch(MDL_V(mat_enc_bwd)<1>, p, st);
  if (NB == 2) return launch(MDL_V(mat_enc_bwd)<2>, p, st);
  if (NB == 3) return launch(MDL_V(mat_enc_bwd)<3>, p, st);
  return -3;
}


#ifdef MDL_TRAIN_PROF
MDL_API int mdl_enc_prof_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tprof), sizeof(unsigned long long) * 32, 0, hipMemcpyDeviceToHost);
}
#endif
