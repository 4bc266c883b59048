// VALU reference implementation of the training-kernel attention (packed bf16 dot products, online softmax).
// Kept as a numerics cross-check for the MFMA path: build with -DMDL_ATTN_VALU (MAT_DCML_EXTRA_FLAGS).
#pragma once
// ------------------------------------------------------------------------------------------ attention (VALU)
// items (s, h, i): online softmax over the keys of sequence s; O may alias Q (each item reads only its own q row)
__device__ __forceinline__ void attn_fwd(const bf16_t* Q, const bf16_t* K, const bf16_t* V, bf16_t* O, bool causal, float* lse_g,
                         const Ctx& c) {
  const int L = c.L, n_items = c.nseq * 2 * L;
  for (int it = c.tid; it < n_items; it += 256) {
    const int s = it / (2 * L), rem = it - s * 2 * L, h = rem / L, i = rem - h * L;
    const int row = s * L + i;
    uint32_t q[16];
    ld_head_u(Q, row, h, q);
    float m = -1e30f, l = 0.f, acc[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) acc[d] = 0.f;
    const int jn = causal ? i + 1 : L;
    for (int j = 0; j < jn; ++j) {
      const int kr = s * L + j;
      uint32_t k[16];
      ld_head_u(K, kr, h, k);
      float d = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) d = dot2(q[t], k[t], d);
      d *= ATT_SCALE;
      if (d > m + 8.f) {  // lazy rescale: exp(d - m) stays <= e^8 between rescales
        const float cf = __expf(m - d);
        l *= cf;
#pragma unroll
        for (int e = 0; e < 32; ++e) acc[e] *= cf;
        m = d;
      }
      const float pj = __expf(d - m);
      l += pj;
      uint32_t v[16];
      ld_head_u(V, kr, h, v);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        acc[2 * t] += pj * lo_bf(v[t]);
        acc[2 * t + 1] += pj * hi_bf(v[t]);
      }
    }
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < 32; ++d) acc[d] *= inv;
    st_head_f(O, row, h, acc);
    if (lse_g) lse_g[(size_t)(c.tok0 + row) * 2 + h] = m + __logf(l);
  }
}

// backward pass 1 (by query row): recompute P from the saved log-sum-exp, delta_i = dO_i·O_i, dq_i
__device__ __forceinline__ void attn_bwd_q(const bf16_t* Q, const bf16_t* K, const bf16_t* V, const bf16_t* DA, bf16_t* DQ,
                           bool causal, const Ctx& c) {
#ifdef MDL_ABLATE_ATTN
  return;
#endif
  const int L = c.L, n_items = c.nseq * 2 * L;
  for (int it = c.tid; it < n_items; it += 256) {
    const int s = it / (2 * L), rem = it - s * 2 * L, h = rem / L, i = rem - h * L;
    const int row = s * L + i;
    uint32_t q[16], da[16];
    ld_head_u(Q, row, h, q);
    ld_head_u(DA, row, h, da);
    const float lse = c.LSE[h * c.NRP + row];
    const int jn = causal ? i + 1 : L;
    float o[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] = 0.f;
    for (int j = 0; j < jn; ++j) {
      const int kr = s * L + j;
      uint32_t k[16], v[16];
      ld_head_u(K, kr, h, k);
      float d = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) d = dot2(q[t], k[t], d);
      const float p = __expf(d * ATT_SCALE - lse);
      ld_head_u(V, kr, h, v);
#pragma unroll
      for (int t = 0; t < 16; ++t) { o[2 * t] += p * lo_bf(v[t]); o[2 * t + 1] += p * hi_bf(v[t]); }
    }
    float delta = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) delta += lo_bf(da[t]) * o[2 * t] + hi_bf(da[t]) * o[2 * t + 1];
    c.DEL[h * c.NRP + row] = delta;
    float dq[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) dq[d] = 0.f;
    for (int j = 0; j < jn; ++j) {
      const int kr = s * L + j;
      uint32_t k[16], v[16];
      ld_head_u(K, kr, h, k);
      ld_head_u(V, kr, h, v);
      float d = 0.f, dp = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) { d = dot2(q[t], k[t], d); dp = dot2(da[t], v[t], dp); }
      const float p = __expf(d * ATT_SCALE - lse);
      const float ds = p * (dp - delta);
#pragma unroll
      for (int t = 0; t < 16; ++t) { dq[2 * t] += ds * lo_bf(k[t]); dq[2 * t + 1] += ds * hi_bf(k[t]); }
    }
#pragma unroll
    for (int d = 0; d < 32; ++d) dq[d] *= ATT_SCALE;
    st_head_f(DQ, row, h, dq);
  }
}

// backward pass 2 (by key row): dk_j, dv_j, written in place over K / V
__device__ __forceinline__ void attn_bwd_kv(const bf16_t* Q, bf16_t* K, bf16_t* V, const bf16_t* DA, bool causal, const Ctx& c) {
#ifdef MDL_ABLATE_ATTN
  return;
#endif
  const int L = c.L, n_items = c.nseq * 2 * L;
  for (int it = c.tid; it < n_items; it += 256) {
    const int s = it / (2 * L), rem = it - s * 2 * L, h = rem / L, j = rem - h * L;
    const int row = s * L + j;
    uint32_t k[16], v[16];
    ld_head_u(K, row, h, k);
    ld_head_u(V, row, h, v);
    float dk[32], dv[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
    
    for (int i = causal ? j : 0; i < L; ++i) {
      const int qr = s * L + i;
      uint32_t q[16], da[16];
      ld_head_u(Q, qr, h, q);
      ld_head_u(DA, qr, h, da);
      float d = 0.f, dp = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) { d = dot2(q[t], k[t], d); dp = dot2(da[t], v[t], dp); }
      const float p = __expf(d * ATT_SCALE - c.LSE[h * c.NRP + qr]);
      const float ds = p * (dp - c.DEL[h * c.NRP + qr]);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        dk[2 * t] += ds * lo_bf(q[t]); dk[2 * t + 1] += ds * hi_bf(q[t]);
        dv[2 * t] += p * lo_bf(da[t]); dv[2 * t + 1] += p * hi_bf(da[t]);
      }
    }
#pragma unroll
    for (int d = 0; d < 32; ++d) dk[d] *= ATT_SCALE;
    st_head_f(K, row, h, dk);
    st_head_f(V, row, h, dv);
  }
}

