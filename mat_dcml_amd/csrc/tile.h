// Token-tile MFMA helpers shared by the fused MAT kernels (gfx950): the token-major swizzled LDS layout and its
// transposed (ds_read_b64_tr_b16) fragment reads.
//
// Token-major LDS buffers: [rows][64] bf16, 16-byte chunk c of row r stored at chunk c ^ ((r>>1)&7) — the 16 rows
// read by one ds_read_b128 lane group land on 16 distinct 4-bank groups.
// RT = one 16x64 f32 register tile in the v_mfma_f32_16x16x32_bf16 C layout: v[ct][r] holds
// (row 4*(lane>>4) + r, col 16*ct + (lane&15)).
#pragma once
#include "common.h"

namespace mdl {

struct RT { f32x4 v[4]; };

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

}  // namespace mdl
