// Token-tile MFMA toolkit shared by the fused MAT training kernels (gfx950).
//
// Conventions (D = 64 features everywhere):
//  * A workgroup owns a tile of whole sequences: rows = tokens, padded to 16-row MFMA row tiles ("rt").
//    Wave w owns row tiles rt = w, w+4, ...; a wave always computes FULL rows (all 64 output columns), so every
//    row-wise op (bias, residual, LayerNorm, GELU) runs in registers on the MFMA accumulator layout.
//  * RT = one 16x64 f32 register tile in the v_mfma_f32_16x16x32_bf16 C layout: v[ct][r] holds
//    (row 4*(lane>>4) + r, col 16*ct + (lane&15)).  Row reductions: in-lane over ct, then xor 1,2,4,8.
//  * Token-major LDS buffers: [rows][64] bf16, 16-byte chunk c of row r stored at chunk c ^ ((r>>1)&7) — the
//    16 rows read by one ds_read_b128 lane group land on 16 distinct 4-bank groups.
//  * Feature-major LDS buffers ([64][pitch] bf16, pitch = padded rows + 8) feed the weight-gradient GEMMs
//    dW = dYᵀ·X, whose reduction dimension is the token axis.
//  * Weights arrive pre-packed as MFMA B fragments ([4 col tiles][2 k-steps][64 lanes][8] bf16), for both W
//    (forward, Y = X·Wᵀ) and Wᵀ (backward, dX = dY·W).
#pragma once
#include "common.h"

namespace mdl {

struct RT { f32x4 v[4]; };
struct BFr { bf16x8 f[4][2]; };

__device__ __forceinline__ void rt_zero(RT& t) {
#pragma unroll
  for (int c = 0; c < 4; ++c) t.v[c] = f32x4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ int tmo(int row, int col) {
  return (row << 6) + ((((col >> 3) ^ ((row >> 1) & 7))) << 3) + (col & 7);
}

__device__ __forceinline__ bf16x8 lda_tm(const bf16_t* buf, int row, int lc) {
  return *(const bf16x8*)(buf + (row << 6) + ((lc ^ ((row >> 1) & 7)) << 3));
}

__device__ __forceinline__ void loadB(BFr& B, const bf16_t* pk, int lane) {
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) B.f[ct][ks] = *(const bf16x8*)(pk + ((size_t)((ct * 2 + ks) * 64 + lane)) * 8);
}

// acc (+)= A[rt rows] · B   (A token-major bf16 in LDS)
__device__ __forceinline__ void gemm_rt(RT& acc, const bf16_t* A, int rt, const BFr& B, int lane, bool accumulate) {
  const int row = rt * 16 + (lane & 15), g = lane >> 4;
  const bf16x8 a0 = lda_tm(A, row, g), a1 = lda_tm(A, row, g + 4);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    f32x4 c = accumulate ? acc.v[ct] : f32x4{0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, B.f[ct][0], c, 0, 0, 0);
    acc.v[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, B.f[ct][1], c, 0, 0, 0);
  }
}

__device__ __forceinline__ void add_bias(RT& t, const float* b, int lane) {
  const int c16 = lane & 15;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const float bb = b[16 * ct + c16];
#pragma unroll
    for (int r = 0; r < 4; ++r) t.v[ct][r] += bb;
  }
}

__device__ __forceinline__ f32x4 rowsum(const RT& t) {
  f32x4 s;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float x = t.v[0][r] + t.v[1][r] + t.v[2][r] + t.v[3][r];
    s[r] = group_sum<16>(x);
  }
  return s;
}

// LayerNorm over the 64 columns of each row; xhat/out in place semantics chosen by caller
__device__ __forceinline__ void ln_fwd(const RT& x, RT& xhat, RT& y, f32x4& mean, f32x4& rstd, const float* gam,
                                       const float* bet, int lane) {
  const int c16 = lane & 15;
  mean = rowsum(x);
#pragma unroll
  for (int r = 0; r < 4; ++r) mean[r] *= (1.f / 64.f);
  RT d;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) { const float t = x.v[ct][r] - mean[r]; d.v[ct][r] = t * t; }
  f32x4 var = rowsum(d);
#pragma unroll
  for (int r = 0; r < 4; ++r) rstd[r] = rsqrtf(var[r] * (1.f / 64.f) + 1e-5f);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const float gg = gam[16 * ct + c16], bb = bet[16 * ct + c16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float xh = (x.v[ct][r] - mean[r]) * rstd[r];
      xhat.v[ct][r] = xh;
      y.v[ct][r] = xh * gg + bb;
    }
  }
}

// LayerNorm backward: dx from dy, xhat, rstd; accumulates dgamma/dbeta partials (per lane, its column) in
// dgacc/dbacc (masked by row validity via vmask).
__device__ __forceinline__ void ln_bwd(const RT& dy, const RT& xhat, const f32x4& rstd, const float* gam, RT& dx,
                                       f32x4& dgacc, f32x4& dbacc, const f32x4& vmask, int lane) {
  const int c16 = lane & 15;
  RT gy, gyx;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const float gg = gam[16 * ct + c16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float dyv = dy.v[ct][r] * vmask[r];
      gy.v[ct][r] = dyv * gg;
      gyx.v[ct][r] = gy.v[ct][r] * xhat.v[ct][r];
      dgacc[ct] += dyv * xhat.v[ct][r];
      dbacc[ct] += dyv;
    }
  }
  f32x4 a = rowsum(gy), b = rowsum(gyx);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      dx.v[ct][r] = (gy.v[ct][r] - a[r] * (1.f / 64.f) - xhat.v[ct][r] * b[r] * (1.f / 64.f)) * rstd[r];
}

// column partial sums of a masked RT (for bias gradients)
__device__ __forceinline__ void colsum_acc(const RT& t, f32x4& acc, const f32x4& vmask) {
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[ct] += t.v[ct][r] * vmask[r];
}

// flush per-lane column partials: reduce over the 4 row groups (xor 16, 32), lanes with g == 0 add
__device__ __forceinline__ void flush_cols(f32x4 acc, float* dst, int lane) {
  if (!dst) return;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    float x = acc[ct];
    x = cross_row_sum(x);
    if ((lane >> 4) == 0) atomicAdd(dst + 16 * ct + (lane & 15), x);
  }
}

// RT -> token-major bf16 LDS (rows of row tile rt)
__device__ __forceinline__ void st_tm(bf16_t* buf, int rt, const RT& t, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) buf[tmo(rt * 16 + 4 * g + r, 16 * ct + c16)] = f2bf(t.v[ct][r]);
}

__device__ __forceinline__ void ld_tm(const bf16_t* buf, int rt, RT& t, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) t.v[ct][r] = bf2f(buf[tmo(rt * 16 + 4 * g + r, 16 * ct + c16)]);
}

// RT -> feature-major bf16 LDS [col][pitch] (4 consecutive rows per lane = one 8-byte store)
__device__ __forceinline__ void st_fm(bf16_t* buf, int pitch, int rt, const RT& t, const f32x4& vmask, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const uint32_t lo = (uint32_t)f2bf(t.v[ct][0] * vmask[0]) | ((uint32_t)f2bf(t.v[ct][1] * vmask[1]) << 16);
    const uint32_t hi = (uint32_t)f2bf(t.v[ct][2] * vmask[2]) | ((uint32_t)f2bf(t.v[ct][3] * vmask[3]) << 16);
    *(uint2*)(buf + (16 * ct + c16) * pitch + rt * 16 + 4 * g) = make_uint2(lo, hi);
  }
}

// dW[n][k] += sum_rows Yf[n][row] * Xf[k][row]   (both feature-major, KP rows, multiple of 32)
// wave w computes output rows n in [16w, 16w+16); atomics into the fp32 gradient
__device__ __forceinline__ void wgrad(const bf16_t* Yf, const bf16_t* Xf, int pitch, int KP, float* dW, int wave,
                                      int lane) {
  if (!dW) return;
  const int g = lane >> 4, c16 = lane & 15;
  RT acc;
  rt_zero(acc);
  const bf16_t* ya = Yf + (16 * wave + c16) * pitch + 8 * g;
  for (int k0 = 0; k0 < KP; k0 += 32) {
    const bf16x8 a = *(const bf16x8*)(ya + k0);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const bf16x8 b = *(const bf16x8*)(Xf + (16 * ct + c16) * pitch + k0 + 8 * g);
      acc.v[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc.v[ct], 0, 0, 0);
    }
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) atomicAdd(dW + (16 * wave + 4 * g + r) * 64 + 16 * ct + c16, acc.v[ct][r]);
}

__device__ __forceinline__ void wave_lds_sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// global (token-major, plain [tok][64] bf16) <-> RT
__device__ __forceinline__ void ld_g_bf(const bf16_t* src, int tok0, int rt, int NR, RT& t, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rt * 16 + 4 * g + r;
    const bool ok = row < NR;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) t.v[ct][r] = ok ? bf2f(src[(size_t)(tok0 + row) * 64 + 16 * ct + c16]) : 0.f;
  }
}
__device__ __forceinline__ void st_g_bf(bf16_t* dst, int tok0, int rt, int NR, const RT& t, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rt * 16 + 4 * g + r;
    if (row < NR) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) dst[(size_t)(tok0 + row) * 64 + 16 * ct + c16] = f2bf(t.v[ct][r]);
    }
  }
}
__device__ __forceinline__ void ld_g_f(const float* src, int tok0, int rt, int NR, RT& t, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rt * 16 + 4 * g + r;
    const bool ok = row < NR;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) t.v[ct][r] = ok ? src[(size_t)(tok0 + row) * 64 + 16 * ct + c16] : 0.f;
  }
}
__device__ __forceinline__ void st_g_f(float* dst, int tok0, int rt, int NR, const RT& t, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rt * 16 + 4 * g + r;
    if (row < NR) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) dst[(size_t)(tok0 + row) * 64 + 16 * ct + c16] = t.v[ct][r];
    }
  }
}

// copy token-major rows [tok0, tok0+NR) of a plain global bf16 [tok][64] tensor into a swizzled LDS buffer
// (zeros for the padded rows up to NRP); cooperative over the workgroup.
__device__ __forceinline__ void g2lds_rows(bf16_t* buf, const bf16_t* src, int tok0, int NR, int NRP, int tid) {
  for (int i = tid; i < NRP * 8; i += 256) {
    const int row = i >> 3, lc = i & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < NR) v = *(const uint4*)(src + (size_t)(tok0 + row) * 64 + lc * 8);
    *(uint4*)(buf + (row << 6) + ((lc ^ ((row >> 1) & 7)) << 3)) = v;
  }
}

__device__ __forceinline__ f32x4 row_mask(int rt, int NR, int lane) {
  const int g = lane >> 4;
  f32x4 m;
#pragma unroll
  for (int r = 0; r < 4; ++r) m[r] = (rt * 16 + 4 * g + r) < NR ? 1.f : 0.f;
  return m;
}

}  // namespace mdl

namespace mdl {
typedef short s16x4 __attribute__((ext_vector_type(4)));

// ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p supplies the address of row q, columns 4p..4p+3 of a
// 4x16 block; lane i receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ s16x4 ld_tr(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// Transposed fragment from a token-major swizzled buffer: lane (g, c) gets rows k0+8g..k0+8g+7 of column n0+c
// (the K-dim of the weight-gradient GEMM is the token axis).  EXEC must be full.
__device__ __forceinline__ bf16x8 ld_frag_T(const bf16_t* buf, int k0, int n0, int lane) {
  const int g = lane >> 4, c = lane & 15, q = c >> 2, p = c & 3;
  const int col = n0 + 4 * p;
  const int r0 = k0 + 8 * g + q, r1 = r0 + 4;
  const bf16_t* a0 = buf + (r0 << 6) + ((((col >> 3) ^ ((r0 >> 1) & 7))) << 3) + (col & 7);
  const bf16_t* a1 = buf + (r1 << 6) + ((((col >> 3) ^ ((r1 >> 1) & 7))) << 3) + (col & 7);
  const s16x4 lo = ld_tr(a0), hi = ld_tr(a1);
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// dW[n][k] += sum_rows Y[row][n] * X[row][k] with Y, X token-major swizzled LDS tiles of KP rows (KP % 32 == 0,
// padded rows zero).  Wave w produces dW rows n in [16w, 16w+16); fp32 atomics into the gradient.
__device__ __forceinline__ void wgrad_tm(const bf16_t* Y, const bf16_t* X, int KP, float* dW, int wave, int lane) {
  if (!dW) return;
#ifdef MDL_ABLATE_WGRAD
  return;
#endif
  const int g = lane >> 4, c16 = lane & 15;
  RT acc;
  rt_zero(acc);
  for (int k0 = 0; k0 < KP; k0 += 32) {
    const bf16x8 a = ld_frag_T(Y, k0, 16 * wave, lane);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const bf16x8 b = ld_frag_T(X, k0, 16 * ct, lane);
      acc.v[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc.v[ct], 0, 0, 0);
    }
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) atomicAdd(dW + (16 * wave + 4 * g + r) * 64 + 16 * ct + c16, acc.v[ct][r]);
}

// masked store of an RT into a token-major buffer (rows with vmask 0 written as 0)
__device__ __forceinline__ void st_tm_m(bf16_t* buf, int rt, const RT& t, const f32x4& vmask, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) buf[tmo(rt * 16 + 4 * g + r, 16 * ct + c16)] = f2bf(t.v[ct][r] * vmask[r]);
}
}  // namespace mdl
