// Kernel arguments and sampling-noise helpers shared by the two rollout-decode kernels:
//   * mat_decode.hip      — 4 waves per env, every decode mode (stride blocks, continuous heads, long L);
//   * mat_decode_wave.hip — ONE wave per env for one-row token passes (the rollout hot path), no barriers.
// Reference semantics: mat_src/mat/algorithms/utils/transformer_act.py:76-99 (autoregressive sampling),
// 37-75 (stride "batch decision" blocks).
#pragma once
#include "common.h"

using mdl::bf16_t;

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
  int B, L, act_dim, n_disc, stride, deterministic, epw, rmax, n_tok, tok_start, tok_zero;   // epw must be 1
  int stage;             // 1: rep / ava / draws of the workgroup's envs are staged in LDS at kernel start
  int cont;              // 1: "Continuous" action type — every agent samples act_dim Gaussians and the next
                         //    row's input is LN(GELU(W_a · x + b_a)) of the sampled vector (not a token row)
  const float* wa;       // [64][act_dim] action-encoder weight (cont)
  const float* ba;       // [64] action-encoder bias (cont)
  const float* lnd;      // [2][64] decoder input LayerNorm (cont)
  int gen;               // 1: draw the sampling noise in-kernel (Philox4x32-10, key (rk0, rk1), counter (env, row,
  uint32_t rk0, rk1, rctr;   //    rctr, purpose)) instead of reading rnd_u / rnd_n — no per-step torch.rand launches
  int avail_cont;        // with cont: "Available_Continuous" (transformer_act.py:234-283) — a categorical over the
                         // first 2 logits (masked by ava[.., :2]) + Normals over the rest; the action vector
                         // [onehot(a), x] feeds the next row; log-probs [B][L][act_dim - 1] = [lp(a), lp(x)]
  const float* qkv0;     // [n_tok][3][64] block-0 q / k / v (bias included) of every action token, or null:
                         // with one row per pass (stride 1, token inputs) the head phase writes the NEXT row's
                         // block-0 query / K / V / residual straight from this table and block 0's projection
                         // phase (one MFMA GEMM + barrier per agent step) disappears
  int q2pre;             // 1: the cross-attention queries W_q2 rep_i + b of every row are precomputed into LDS
                         // before the agent loop (they depend only on the encoder output, ma_transformer.py:114)
  uint32_t genv0;        // global id of batch row 0: the noise of row b is keyed by env genv0 + b, so the rollout of a
                         // global env does not depend on how envs are split over ranks
  const float* hfold;    // [act_dim][64] W_h2 diag(gamma_h), then G[act_dim] = Σ_c W_h2 gamma_h, C[act_dim] = W_h2 beta_h
                         // + b_h2: the head LayerNorm folded into the logit GEMV (fused head of one-row passes)
  const bf16_t* wfa;     // [10*NB+1][4096] decoder weights as token-on-lane A fragments (the training kernels' "fa"
                         // pack, ops/mat_train.ModelPack): the one-wave decode (mat_decode_wave.hip); null: not used
};

// in-kernel sampling noise: one Philox block per (global env, row, call counter, purpose); purpose 0 = the categorical
// uniform (x) and the Normal draws of dims 0, 1 (Box-Muller of y, z); purpose 1 + k = dims 2 + 2k, 3 + 2k
__device__ __forceinline__ float draw_u(const DecParams& p, int env, int row) {
  const mdl::u4 r = mdl::philox4x32_10(p.genv0 + (uint32_t)env, (uint32_t)row, p.rctr, (uint32_t)mdl::P_POLICY, p.rk0, p.rk1);
  return mdl::u01_open_f(r.x);
}
__device__ __forceinline__ float draw_n(const DecParams& p, int env, int row, int a) {
  const int k = a >> 1;
  const mdl::u4 r = mdl::philox4x32_10(p.genv0 + (uint32_t)env, (uint32_t)row, p.rctr, (uint32_t)(mdl::P_POLICY + k),
                                       p.rk0, p.rk1);
  const uint32_t b0 = k == 0 ? r.y : r.x, b1 = k == 0 ? r.z : r.y;
  const float rad = sqrtf(-2.f * __logf(mdl::u01_open_f(b0))), th = 6.283185307179586f * mdl::u01_open_f(b1);
  return (a & 1) ? rad * __sinf(th) : rad * __cosf(th);
}

// One-wave decode (mat_decode_wave.hip): 0 = launched, 1 = this configuration is not on its path (the caller runs
// the 4-wave kernel), < 0 = launch error.
int mdl_decode_wave(const DecParams* p, int NB, hipStream_t st);
