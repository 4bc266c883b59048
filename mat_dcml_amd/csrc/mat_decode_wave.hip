// mat_decode_wave — the rollout's autoregressive action decode with ONE wave per env (gfx950 / CDNA4).
//
// Reference hot loop: L decoder passes per env step (mat_src/mat/algorithms/utils/transformer_act.py:76-99), here one
// agent row per pass against K / V caches of the earlier rows (exact: row i depends only on the shifted actions 0..i).
//
// Why one wave: the 4-wave kernel (mat_decode.hip) splits every 64x64 product over the waves of a workgroup and so
// needs an LDS exchange + workgroup barrier between consecutive products — ~9 barrier-separated phases per decoder
// block; its waves spent 53 % of their cycles waiting (profiles/r3_check1/decode_pmc.txt).  Here one wave owns an
// env and runs the whole chain in registers, in the token-on-lane ("CT") layout of the training kernels
// (mat_train_ct.h): Yᵀ = W·Xᵀ with the weight as the MFMA A operand in a permuted k order, so each product's C
// registers, packed to bf16, ARE the next product's B operand — linear → bias → residual → LayerNorm → linear chains
// never leave the registers and no barrier exists anywhere in the agent loop.
//
// The live agent row is replicated over the 16 token columns of the tile, which buys two things:
//  * attention of BOTH heads in one instruction stream: columns 0..7 carry head 0's query (k-step 0 = dims 0..31),
//    columns 8..15 head 1's (k-step 1), so one online-softmax pass serves both heads; a bank-masked DPP row_ror:8
//    then hands each column the other head's half of O;
//  * elementwise work split over the row: for GELU, lane c evaluates ONE of its 16 features (feature 16(c>>2) + 4g +
//    (c&3)) and 16 DPP row_newbcast moves give every lane all 16 results (1 erf per lane instead of 16).
// Weights: the 64x64 A fragments (the training kernels' "fa" pack) live in LDS — the last NREG of the agent loop's
// matrices in registers when LDS is short (n_block 2) — biases / LayerNorm vectors / token tables in LDS, the K / V
// caches of every block in one token-major swizzled LDS array (tile.h tmo) as in the 4-wave kernel.  Block 0's
// self-attention q / K / V come from the per-token table (they depend only on the previous action), the
// cross-attention queries W_q2 rep_i are precomputed before the agent loop, the head LayerNorm is folded into the
// logit product (DecParams.hfold), sampling noise comes from in-kernel Philox (same streams as mat_decode.hip).
#define MDL_LN_ONEPASS
#include "mat_train_ct.h"
#include "decode_params.h"

namespace {

// Debug build (-DMDL_WAVE_DEBUG): the replicated CT vectors of env 0 at row g_wdbg_row after every stage -> g_wdbg
// (read back by mdl_wave_debug_read; scripts/wave_debug.py compares them with the torch decoder)
#ifdef MDL_WAVE_DEBUG
__device__ float g_wdbg[16][64];
__device__ int g_wdbg_row;
__device__ __forceinline__ void wdbg(int stage, const CT& x, int i, int lane) {
  if (blockIdx.x == 0 && i == g_wdbg_row && (lane & 15) == 0) {
    const int g = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) g_wdbg[stage][16 * mt + 4 * g + r] = x.v[mt][r];
  }
}
#define WDBG(st, x) wdbg(st, x, i, lane)
#else
#define WDBG(st, x) do { } while (0)
#endif

// ------------------------------------------------------------------------------------------ weight slots
// Matrices the agent loop multiplies by (block 0: proj1, k2, v2, proj2, mlp0, mlp2; block b > 0 adds q1, k1, v1;
// then the head's first linear), in loop order.  Slot -> decoder linear index (ops/mat_train.decoder_linears: per
// block q1 k1 v1 p1 q2 k2 v2 p2 m0 m2, then head[0]).
__host__ __device__ constexpr int wv_nm(int NB) { return 6 + 9 * (NB - 1) + 1; }
__host__ __device__ constexpr int wv_lin(int NB, int s) {
  return s < 6 ? (s == 0 ? 3 : s + 4)
               : (s == wv_nm(NB) - 1 ? 10 * NB
                                     : 10 * (1 + (s - 6) / 9) + ((s - 6) % 9 < 4 ? (s - 6) % 9 : (s - 6) % 9 + 1));
}
__host__ __device__ constexpr int wv_slot(int b, int k) {   // k = linear within block b (never 4 = q2; b = 0: k >= 3)
  return b == 0 ? (k == 3 ? 0 : k - 4) : 6 + 9 * (b - 1) + (k < 4 ? k : k - 1);
}

struct WvLds { int w, kv, q2, qt, et, bi, lp, sc, total; };   // byte offsets of the LDS carve
// wide heads (A > 4: SMAC's 38-token tables) read the embedded input rows straight from global memory (etg): the
// load is issued before block 0's attention and consumed after it, and the 9.7 KB it frees in LDS keeps two more
// weight matrices out of the register file (SMAC: 4 register matrices instead of 6, which spilled)
__host__ __device__ inline WvLds wv_lds(int NB, int L, int n_tok, int nlds, bool etg) {
  WvLds o;
  int off = 0;
  auto take = [&](int bytes) { const int r = off; off += (bytes + 15) & ~15; return r; };
  o.w = take(nlds * 8192);                   // [slot][4096] bf16 A fragments
  o.kv = take((NB * 4 * L + 32) * 128);      // K / V caches (+ 32 zero rows: 32-key chunks read past the last cache)
  o.q2 = take(NB * L * 128);                 // [block][row][64] bf16 cross-attention queries
  o.qt = take(n_tok * 3 * 128);              // [token][q, k, v][64] bf16 block-0 self-attention operands
  o.et = take(etg ? 0 : n_tok * 256);        // [token][64] f32 embedded decoder input rows (the block-0 residual)
  o.bi = take((10 * NB + 1) * 256);          // biases
  o.lp = take((3 * NB + 1) * 512);           // LayerNorm gamma / beta
  o.sc = take(64 * 4);                       // logits of the wide head
  o.total = off;
  return o;
}

// K / V cache (block b, kind: 0 self K, 1 self V, 2 cross K, 3 cross V) = rows [(4b + kind) L, (4b + kind + 1) L)
// of the KV array; rows inside a cache are swizzled relative to its first row (wv_attn)
__device__ __forceinline__ bf16_t* wv_cache(bf16_t* KV, int b, int kind, int L) { return KV + (size_t)(b * 4 + kind) * L * 64; }

template <int N>
struct RegW { AFr w[N > 0 ? N : 1]; };

template <int S, int NLDS, int NREG>
__device__ __forceinline__ void wv_getw(AFr& w, const RegW<NREG>& rw, const bf16_t* W, int lane) {
  if constexpr (S >= NLDS) {
    w = rw.w[S - NLDS];
  } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) w.f[mt][s] = *(const bf16x8*)(W + (size_t)S * 4096 + ((mt * 2 + s) * 64 + lane) * 8);
  }
}

// 8 bytes (4 bf16) of a token-major swizzled row
__device__ __forceinline__ uint2 kv_ld2(const bf16_t* KV, int row, int col) { return *(const uint2*)(KV + tmo(row, col)); }
// this lane's CT pieces of a token row -> swizzled KV row (the live row is replicated over the columns: column 0 writes)
__device__ __forceinline__ void kv_st_row(bf16_t* KV, int row, const CTr& x, int lane) {
  if ((lane & 15) == 0) {
    const int g = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) *(uint2*)(KV + tmo(row, 16 * mt + 4 * g)) = x.q[mt];
  }
}

template <int N>
__device__ __forceinline__ float row_bcast(float x) {   // lane N of each 16-lane row -> the whole row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x150 + N, 0xF, 0xF, false));
}
// lanes of the enabled banks take lane (c + 8) & 15's value, the others keep their own.  Elements go through a
// scalar: hipcc lowers __builtin_bit_cast(int, v[r]) of an ext-vector element as element 0 for every r (all four
// results became element 0's), so never bit_cast a subscripted vector element.
template <int BANKS>
__device__ __forceinline__ float ror8_bank(float x) {
  const int a = __builtin_bit_cast(int, x);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(a, a, 0x128, 0xF, BANKS, false));
}
template <int BANKS>
__device__ __forceinline__ f32x4 ror8_banks(f32x4 v) {
  return f32x4{ror8_bank<BANKS>(v.x), ror8_bank<BANKS>(v.y), ror8_bank<BANKS>(v.z), ror8_bank<BANKS>(v.w)};
}

// GELU of a replicated CT vector with one erf per lane: lane c evaluates feature 16(c>>2) + 4g + (c&3), the row
// broadcasts hand every lane its 16 results
__device__ __forceinline__ float gelu_pick(const CT& h, int lane) {
  const int c = lane & 15;
  const f32x4 a = (c & 4) ? h.v[1] : h.v[0];
  const f32x4 b = (c & 4) ? h.v[3] : h.v[2];
  const f32x4 v = (c & 8) ? b : a;
  const float lo = (c & 1) ? v[1] : v[0], hi = (c & 1) ? v[3] : v[2];
  return gelu_erf((c & 2) ? hi : lo);
}
// ... as the packed bf16 MFMA operand: even lanes pack their pair (features 4g + r, r + 1 of tile c >> 2) after one
// pair-swap DPP, and 8 row broadcasts of the packed words replace 16 fp32 broadcasts + 8 conversions
__device__ __forceinline__ CTr gelu_dist_pk(const CT& h, int lane) {
  const float ge = gelu_pick(h, lane);
  const float nb = dppf<DPP_XOR1>(ge);
  const float pk = __builtin_bit_cast(float, pk2(ge, nb));   // valid on even lanes c
  CTr o;
  o.q[0] = make_uint2(__builtin_bit_cast(uint32_t, row_bcast<0>(pk)), __builtin_bit_cast(uint32_t, row_bcast<2>(pk)));
  o.q[1] = make_uint2(__builtin_bit_cast(uint32_t, row_bcast<4>(pk)), __builtin_bit_cast(uint32_t, row_bcast<6>(pk)));
  o.q[2] = make_uint2(__builtin_bit_cast(uint32_t, row_bcast<8>(pk)), __builtin_bit_cast(uint32_t, row_bcast<10>(pk)));
  o.q[3] = make_uint2(__builtin_bit_cast(uint32_t, row_bcast<12>(pk)), __builtin_bit_cast(uint32_t, row_bcast<14>(pk)));
  return o;
}
__device__ __forceinline__ CT gelu_dist(const CT& h, int lane) {
  const float ge = gelu_pick(h, lane);
  CT o;
  o.v[0] = f32x4{row_bcast<0>(ge), row_bcast<1>(ge), row_bcast<2>(ge), row_bcast<3>(ge)};
  o.v[1] = f32x4{row_bcast<4>(ge), row_bcast<5>(ge), row_bcast<6>(ge), row_bcast<7>(ge)};
  o.v[2] = f32x4{row_bcast<8>(ge), row_bcast<9>(ge), row_bcast<10>(ge), row_bcast<11>(ge)};
  o.v[3] = f32x4{row_bcast<12>(ge), row_bcast<13>(ge), row_bcast<14>(ge), row_bcast<15>(ge)};
  return o;
}

// Causal attention of the live row i over cache rows 0..i (K rows rK + j, V rows rV + j), both heads at once:
// column c carries head c >> 3.  Scores Sᵀ = K·Qᵀ per 16-key half t (A rows = keys kb + pi_row(t, m), k = the
// head's 32 dims in the CT permuted order, so the query is its CT registers), online softmax in log2 units, P as a
// hi/lo bf16 pair, Oᵀ = Vᵀ·Pᵀ with Vᵀ from ds_read_b64_tr_b16; O returned in CT layout (replicated).
// Rows are addressed relative to each cache's first row (K = Kc, V = Vc: the swizzle only has to agree between the
// row's writer and readers), so every lane's swizzled offsets are the same for all caches and agent steps (hoisted
// out of the agent loop) and a 32-row key chunk only adds kb * 64 (a 32-row step keeps the (row >> 1) & 7 swizzle).
// One 32-key chunk of the online softmax (FIRST: the chunk at key 0, which every row has — no running state to
// rescale, so the common L <= 32 case runs no loop and carries no registers around one).
template <bool FIRST>
__device__ __forceinline__ void wv_attn_chunk(const bf16_t* Kc, const bf16_t* Vc, const bf16x8& qb0, const bf16x8& qb1,
                                              int kb, int i, int lane, float& m, float& l, f32x4 (&o)[4]) {
  const int g = lane >> 4, c = lane & 15;
  float sc[8];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const bf16_t* Kk = Kc + kb * 64;
    const int key = pi_row(t, c);
    const uint2 p0 = kv_ld2(Kk, key, 4 * g), p1 = kv_ld2(Kk, key, 16 + 4 * g);
    const uint2 p2 = kv_ld2(Kk, key, 32 + 4 * g), p3 = kv_ld2(Kk, key, 48 + 4 * g);
    f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mk8(p0.x, p0.y, p1.x, p1.y), qb0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mk8(p2.x, p2.y, p3.x, p3.y), qb1, r, 0, 0, 0);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) sc[4 * t + rr] = r[rr];
  }
  const int d0 = i - kb - 8 * g;   // key kb + 8g + j is visible iff j <= d0
  float cm = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = j <= d0 ? sc[j] : -INFINITY;
    cm = fmaxf(cm, sc[j]);
  }
  const float cmax = cross_row_max(cm) * ATT_L2;   // finite: key kb <= i is visible
  const float nm = FIRST ? cmax : fmaxf(m, cmax);
  float ps = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = fast_exp2(fmaf(sc[j], ATT_L2, -nm));
    ps += sc[j];
  }
  bf16x8 ph, pl;
  split8v(sc, ph, pl);
  if constexpr (FIRST) {
    l = ps;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const bf16x8 va = ld_frag_T(Vc, 0, 16 * mt, lane);
      o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, ph, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pl, o[mt], 0, 0, 0);
    }
  } else {
    const float alpha = fast_exp2(m - nm);
    l = l * alpha + ps;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const bf16x8 va = ld_frag_T(Vc + kb * 64, 0, 16 * mt, lane);
      o[mt] *= alpha;
      o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, ph, o[mt], 0, 0, 0);
      o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pl, o[mt], 0, 0, 0);
    }
  }
  m = nm;
}

__device__ __forceinline__ CT wv_attn(const bf16_t* Kc, const bf16_t* Vc, const CTr& qr, int i, int lane) {
  const int c = lane & 15;
  const bool h1 = c >= 8;
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16x8 qb0 = h1 ? z8 : rb(qr, 0), qb1 = h1 ? rb(qr, 1) : z8;
  float m, l;
  f32x4 o[4];
#ifdef MDL_WV_NOPEEL
  m = -INFINITY;
  l = 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb <= i; kb += 32) wv_attn_chunk<false>(Kc, Vc, qb0, qb1, kb, i, lane, m, l, o);
#else
  wv_attn_chunk<true>(Kc, Vc, qb0, qb1, 0, i, lane, m, l, o);
  for (int kb = 32; kb <= i; kb += 32) wv_attn_chunk<false>(Kc, Vc, qb0, qb1, kb, i, lane, m, l, o);
#endif
  const float il = 1.f / cross_row_sum(l);
  CT O;
  // columns c < 8 hold head 0 (dims 0..31 = mt 0, 1), c >= 8 head 1 (mt 2, 3): each takes the other half from c ^ 8
  O.v[0] = ror8_banks<0xC>(o[0] * il);
  O.v[1] = ror8_banks<0xC>(o[1] * il);
  O.v[2] = ror8_banks<0x3>(o[2] * il);
  O.v[3] = ror8_banks<0x3>(o[3] * il);
  return O;
}

struct WvCtx {
  bf16_t *W, *KV, *Q2, *QT;
  const float* ET;
  float *BI, *LP;
  int lane, L;
};

// one decoder block for the live row i (ma_transformer.py:95-98): x <- LN1(x + attn1(x)); x <- LN2(rep_i + attn2(q =
// rep_i, k = v = x)); x <- LN3(x + mlp(x)).  Block 0's q / K / V of x come from the token table (x = ET[tok]).
// STQ (the speculative kernel's PAIR main wave): block B's q / K / V rows of x were computed ahead by the speculative
// wave and staged at stq ([q, k, v][64] bf16): the row's K / V are copied into the caches, the three products skipped
template <int B, int NB, int NLDS, int NREG, bool STQ = false>
__device__ __forceinline__ void wv_block(CT& x, const WvCtx& k, const RegW<NREG>& rw, int i, int tok, const CT& repi,
                                         const CTr* q2in = nullptr, const bf16_t* stq = nullptr) {
  const int lane = k.lane, g = lane >> 4, L = k.L;
  CT xh;
  AFr w;
  CTr qr;
  if constexpr (B == 0) {
    const bf16_t* t = k.QT + tok * 192;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) qr.q[mt] = *(const uint2*)(t + 16 * mt + 4 * g);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        *(uint2*)(wv_cache(k.KV, 0, 0, L) + tmo(i, 16 * mt + 4 * g)) = *(const uint2*)(t + 64 + 16 * mt + 4 * g);
        *(uint2*)(wv_cache(k.KV, 0, 1, L) + tmo(i, 16 * mt + 4 * g)) = *(const uint2*)(t + 128 + 16 * mt + 4 * g);
      }
    }
    x = ld_vec(k.ET + tok * 64, lane);
  } else if constexpr (STQ) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) qr.q[mt] = *(const uint2*)(stq + 16 * mt + 4 * g);
    if (lane < 16) {   // lane (kind, 16-byte chunk): staged K / V row -> swizzled cache row i
      const int kind = lane >> 3, ch = lane & 7;
      *(uint4*)(wv_cache(k.KV, B, kind, L) + tmo(i, 8 * ch)) = *(const uint4*)(stq + 64 * (kind + 1) + 8 * ch);
    }
  } else {
    const CTr xp = ct_pack(x);
    CT q = ld_vec(k.BI + 64 * (10 * B + 0), lane), kk = ld_vec(k.BI + 64 * (10 * B + 1), lane);
    CT vv = ld_vec(k.BI + 64 * (10 * B + 2), lane);
    wv_getw<wv_slot(B, 0), NLDS, NREG>(w, rw, k.W, lane);
    mm(q, w, xp);
    wv_getw<wv_slot(B, 1), NLDS, NREG>(w, rw, k.W, lane);
    mm(kk, w, xp);
    wv_getw<wv_slot(B, 2), NLDS, NREG>(w, rw, k.W, lane);
    mm(vv, w, xp);
    qr = ct_pack(q);
    kv_st_row(wv_cache(k.KV, B, 0, L), i, ct_pack(kk), lane);
    kv_st_row(wv_cache(k.KV, B, 1, L), i, ct_pack(vv), lane);
  }
  asm volatile("" ::: "memory");   // the cache row above is read back by other lanes below (LDS is in order per wave)
  WDBG(6 * B + 0, x);
  {
    const CT O = wv_attn(wv_cache(k.KV, B, 0, L), wv_cache(k.KV, B, 1, L), qr, i, lane);
    WDBG(6 * B + 1, O);
    wv_getw<wv_slot(B, 3), NLDS, NREG>(w, rw, k.W, lane);
    CT t = ct_add(ld_vec(k.BI + 64 * (10 * B + 3), lane), x);
    mm(t, w, ct_pack(O));
    ln_fwd_ct(t, xh, x, ld_vec(k.LP + (3 * B + 0) * 128, lane), ld_vec(k.LP + (3 * B + 0) * 128 + 64, lane));
  }
  {   // cross-attention K / V of x1
    const CTr xp = ct_pack(x);
    CT kk = ld_vec(k.BI + 64 * (10 * B + 5), lane), vv = ld_vec(k.BI + 64 * (10 * B + 6), lane);
    wv_getw<wv_slot(B, 5), NLDS, NREG>(w, rw, k.W, lane);
    mm(kk, w, xp);
    wv_getw<wv_slot(B, 6), NLDS, NREG>(w, rw, k.W, lane);
    mm(vv, w, xp);
    kv_st_row(wv_cache(k.KV, B, 2, L), i, ct_pack(kk), lane);
    kv_st_row(wv_cache(k.KV, B, 3, L), i, ct_pack(vv), lane);
  }
  asm volatile("" ::: "memory");
  {
    CTr q2;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      q2.q[mt] = q2in ? q2in->q[mt] : *(const uint2*)(k.Q2 + (size_t)(B * L + i) * 64 + 16 * mt + 4 * g);
    WDBG(6 * B + 2, x);
    const CT O = wv_attn(wv_cache(k.KV, B, 2, L), wv_cache(k.KV, B, 3, L), q2, i, lane);
    WDBG(6 * B + 3, O);
    wv_getw<wv_slot(B, 7), NLDS, NREG>(w, rw, k.W, lane);
    CT t = ct_add(ld_vec(k.BI + 64 * (10 * B + 7), lane), repi);
    mm(t, w, ct_pack(O));
    ln_fwd_ct(t, xh, x, ld_vec(k.LP + (3 * B + 1) * 128, lane), ld_vec(k.LP + (3 * B + 1) * 128 + 64, lane));
  }
  {   // MLP
    CT h = ld_vec(k.BI + 64 * (10 * B + 8), lane);
    wv_getw<wv_slot(B, 8), NLDS, NREG>(w, rw, k.W, lane);
    mm(h, w, ct_pack(x));
    WDBG(6 * B + 4, x);
    const CTr hp = gelu_dist_pk(h, lane);
    wv_getw<wv_slot(B, 9), NLDS, NREG>(w, rw, k.W, lane);
    CT t = ct_add(ld_vec(k.BI + 64 * (10 * B + 9), lane), x);
    mm(t, w, hp);
    ln_fwd_ct(t, xh, x, ld_vec(k.LP + (3 * B + 2) * 128, lane), ld_vec(k.LP + (3 * B + 2) * 128 + 64, lane));
    WDBG(6 * B + 5, x);
  }
}

// inclusive prefix sum over the 64 lanes (DPP row shifts, then the lower rows' totals)
__device__ __forceinline__ float wv_incl_scan(float x, int lane) {
  x += dppf<0x111>(x);
  x += dppf<0x112>(x);
  x += dppf<0x114>(x);
  x += dppf<0x118>(x);
  const float t0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 15));
  const float t1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 31));
  const float t2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 47));
  const int r = lane >> 4;
  return x + ((r >= 1 ? t0 : 0.f) + (r >= 2 ? t1 : 0.f) + (r >= 3 ? t2 : 0.f));
}
__device__ __forceinline__ float rdlane(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}

// Phase profile (-DMDL_SPEC_PROF, scripts/spec_prof.py): s_memtime cycles per phase of the main wave and of the first
// speculative wave, summed over envs and agent steps (g_spprof[role][phase], read by mdl_spec_prof_read)
#ifdef MDL_SPEC_PROF
__device__ unsigned long long g_spprof[2][16];
#define SPP_DECL unsigned long long spp_t = __builtin_amdgcn_s_memtime(), spp_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define SPP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); spp_acc[k] += t_ - spp_t; spp_t = t_; } while (0)
#define SPP_END(role) do { if (lane == 0 && (role) >= 0) for (int k_ = 0; k_ < 16; ++k_) atomicAdd(&g_spprof[role][k_], spp_acc[k_]); } while (0)
// inside the head helper (main wave): marks into the caller's accumulators through hp (unsigned long long[17])
#define SPH(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); hp[k] += t_ - hp[16]; hp[16] = t_; } while (0)
#else
#define SPH(k) do { } while (0)
#define SPP_DECL do { } while (0)
#define SPP(k) do { } while (0)
#define SPP_END(role) do { } while (0)
#endif
// folded head: W' = W_h2 diag(gamma_h) as hi / lo A fragments (rows = actions 16 ma + c, k in the CT order), and
// G_a = Σ W'[a], C_a = W_h2 beta_h + b_h2 for this lane's logit slots a = 16 ma + 4 g + r
template <int MA>
struct WvHeadW { bf16x8 HH[MA][2], HL[MA][2]; f32x4 HG[MA], HC[MA]; };
template <int MA>
__device__ __forceinline__ void wv_head_load(WvHeadW<MA>& hw, const DecParams& p, int lane) {
  const int g = lane >> 4, c = lane & 15, A = p.act_dim;
#pragma unroll
  for (int ma = 0; ma < MA; ++ma) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int a = 16 * ma + c, kk = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
        const float wv = a < A ? p.hfold[(a < A ? a : 0) * 64 + kk] : 0.f;
        const bf16_t h = f2bf(wv);
        hw.HH[ma][s][j] = (short)h;
        hw.HL[ma][s][j] = (short)f2bf(wv - bf2f(h));
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 16 * ma + 4 * g + r;
      hw.HG[ma][r] = a < A ? p.hfold[A * 64 + a] : 0.f;
      hw.HC[ma][r] = a < A ? p.hfold[A * 65 + a] : 0.f;
    }
  }
}

// sampling noise of every row: lane j holds row j (+ 64, + 128); the Normal draw of the semi-discrete last row
struct WvNoise { float U[3]; float zlast; };
__device__ __forceinline__ WvNoise wv_noise_load(const DecParams& p, int env, int lane) {
  WvNoise nz{{0.f, 0.f, 0.f}, 0.f};
  const int L = p.L, A = p.act_dim, n_disc = p.n_disc;
  if (!p.deterministic) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int row = lane + 64 * q;
      if (row < n_disc) nz.U[q] = p.gen ? draw_u(p, env, row) : p.rnd_u[(size_t)env * L + row];
    }
    if (n_disc < L) nz.zlast = p.gen ? draw_n(p, env, L - 1, A - 1) : p.rnd_n[((size_t)env * L + L - 1) * A + A - 1];
  }
  // opaque: otherwise hipcc re-materialises the Philox rounds inside the agent loop (~80 VALU per agent step)
  asm volatile("" : "+v"(nz.U[0]), "+v"(nz.U[1]), "+v"(nz.U[2]), "+v"(nz.zlast));
  return nz;
}

// the head of row i (transformer_act.py:86-97): GELU(W_h1 x + b) -> folded LayerNorm -> logits (hi / lo MFMA
// products: fp32-like) -> masked categorical / the ratio agent's Normal, every lane alike; writes the row's action
// and log-prob and returns the next row's input token (unchanged after the continuous last row)
template <int NM, int NLDS, int NREG, int MA>
__device__ __forceinline__ int wv_head_sample(const CT& x, const WvHeadW<MA>& hw, const WvNoise& nz, const RegW<NREG>& rw,
                                              const bf16_t* W, const float* BI, float* SC, const DecParams& p, int env,
                                              int i, float avl, int tok, int lane,
                                              unsigned long long* hp = nullptr) {
  constexpr bool WIDE = MA > 1;
  const int g = lane >> 4, c = lane & 15, A = p.act_dim, L = p.L, n_disc = p.n_disc;
  const bool det = p.deterministic != 0;
  constexpr int NB = (NM - 7) / 9 + 1;
  CT h = ld_vec(BI + 64 * (10 * NB), lane);
  {
    AFr w;
    wv_getw<NM - 1, NLDS, NREG>(w, rw, W, lane);
    mm(h, w, ct_pack(x));
  }
  if (hp) SPH(8);
  h = gelu_dist(h, lane);
  if (hp) SPH(9);
  WDBG(12, h);
  f32x4 s4 = (h.v[0] + h.v[1]) + (h.v[2] + h.v[3]);
  f32x4 q4 = h.v[0] * h.v[0];
#pragma unroll
  for (int mt = 1; mt < 4; ++mt) q4 = h.v[mt] * h.v[mt] + q4;
  const float mean = cross_row_sum((s4[0] + s4[1]) + (s4[2] + s4[3])) * (1.f / 64.f);
  const float rstd = rsqrtf(fmaxf(cross_row_sum((q4[0] + q4[1]) + (q4[2] + q4[3])) * (1.f / 64.f) - mean * mean, 0.f) + 1e-5f);
  CTr nh, nl;
  ct_split(h, nh, nl);
  if (hp) SPH(10);
  f32x4 lg[MA];
#pragma unroll
  for (int ma = 0; ma < MA; ++ma) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hw.HH[ma][s], rb(nh, s), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hw.HH[ma][s], rb(nl, s), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hw.HL[ma][s], rb(nh, s), acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) lg[ma][r] = rstd * (acc[r] - mean * hw.HG[ma][r]) + hw.HC[ma][r];
  }
#ifdef MDL_WAVE_DEBUG
  {
    CT lgc;
#pragma unroll
    for (int ma = 0; ma < 4; ++ma) lgc.v[ma] = ma < MA ? lg[ma < MA ? ma : 0] : f32x4{0.f, 0.f, 0.f, 0.f};
    WDBG(13, lgc);
  }
#endif
  if (hp) SPH(11);
  const size_t oi = (size_t)env * L + i;
  float a_out, lp_out;
  if constexpr (!WIDE) {   // A <= 4: the logits are registers r < A of lanes g = 0
    float l[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) l[a] = rdlane(lg[0][a], 0);
    if (i < n_disc) {
      float mx = -INFINITY;
      int amax = 0;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        l[a] = a < A ? (rdlane(avl, a) == 0.f ? -1e10f : l[a]) : -INFINITY;
        if (l[a] > mx) { mx = l[a]; amax = a; }
      }
      float e[4], se = 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a) { e[a] = a < A ? __expf(l[a] - mx) : 0.f; se += e[a]; }
      const float lse = mx + __logf(se);
      int act = amax;
      if (!det) {
        const float uu = rdlane(i < 64 ? nz.U[0] : i < 128 ? nz.U[1] : nz.U[2], i & 63);
        const float inv = 1.f / se;
        float cdf = 0.f;
        int cnt = 0;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          cdf += e[a] * inv;
          cnt += (a < A) & (cdf < uu);
        }
        act = min(cnt, A - 1);
      }
      float la = l[0];
#pragma unroll
      for (int a = 1; a < 4; ++a) la = act == a ? l[a] : la;
      a_out = (float)act;
      lp_out = la - lse;
      tok = 1 + act;
    } else {
      const float mu = A == 1 ? l[0] : A == 2 ? l[1] : A == 3 ? l[2] : l[3];
      const float sd = p.stdv[A - 1];
      a_out = det ? mu : mu + sd * nz.zlast;
      const float z = (a_out - mu) / sd;
      lp_out = -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
    }
  } else {   // 4 < A <= 64: logits through LDS, lane a = action a
    if (c == 0) {
#pragma unroll
      for (int ma = 0; ma < MA; ++ma) *(f32x4*)(SC + 16 * ma + 4 * g) = lg[ma];
    }
    asm volatile("" ::: "memory");
    const bool aok = lane < A;
    const float raw = SC[lane];
    asm volatile("" ::: "memory");   // the next row's writes stay behind these reads
    if (i < n_disc) {
      const float l = aok ? (avl == 0.f ? -1e10f : raw) : -INFINITY;
      const float mx = wave_max(l);
      int act = __ffsll((unsigned long long)__ballot(l == mx)) - 1;   // first maximum (argmax)
      const float lse = mx + __logf(wave_sum(aok ? __expf(l - mx) : 0.f));
      if (!det) {   // inverse CDF: the number of actions whose running probability is below u
        const float cdf = wv_incl_scan(aok ? __expf(l - lse) : 0.f, lane);
        const float uu = rdlane(i < 64 ? nz.U[0] : i < 128 ? nz.U[1] : nz.U[2], i & 63);
        act = min((int)__popcll((unsigned long long)__ballot(aok && cdf < uu)), A - 1);
      }
      act = __builtin_amdgcn_readfirstlane(act);
      a_out = (float)act;
      lp_out = rdlane(l, act) - lse;
      tok = 1 + act;
    } else {
      const float mu = rdlane(raw, A - 1), sd = p.stdv[A - 1];
      a_out = det ? mu : mu + sd * nz.zlast;
      const float z = (a_out - mu) / sd;
      lp_out = -0.5f * z * z - __logf(sd) - 0.91893853320467274f;
    }
  }
  if (hp) SPH(12);
  if (lane == 0) {
    p.out_a[oi] = a_out;
    p.out_lp[oi] = lp_out;
  }
  if (hp) SPH(13);
  return tok;
}

// MA = logit tiles of the head: 1 (A <= 4: the logits sit in registers r < A of lanes g = 0), 3 (A <= 48: SMAC's
// 36 actions — a 4th tile was 6 dead MFMAs and 24 registers of folded weights per agent step), 4 (A <= 64)
template <int NB, int NREG, int MA>
__global__ __launch_bounds__(64, 1) void mat_decode_wave_kernel(DecParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NM = wv_nm(NB), NLDS = NM - NREG;
  constexpr bool WIDE = MA > 1;
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  const int env = blockIdx.x, L = p.L, A = p.act_dim;
  const WvLds lo = wv_lds(NB, L, p.n_tok, NLDS, WIDE);
  bf16_t* W = (bf16_t*)(smem + lo.w);
  bf16_t* KV = (bf16_t*)(smem + lo.kv);
  bf16_t* Q2 = (bf16_t*)(smem + lo.q2);
  bf16_t* QT = (bf16_t*)(smem + lo.qt);
  const float* ET = WIDE ? p.emb : (const float*)(smem + lo.et);
  float* BI = (float*)(smem + lo.bi);
  float* LP = (float*)(smem + lo.lp);
  float* SC = (float*)(smem + lo.sc);

  // ---------------------------------------------------------------- setup: weights, tables, caches
#pragma unroll 1
  for (int s = 0; s < NLDS; ++s) {
    const uint4* src = (const uint4*)(p.wfa + (size_t)wv_lin(NB, s) * 4096);
    uint4* dst = (uint4*)(W + (size_t)s * 4096);
    uint4 t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = src[lane + 64 * j];
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[lane + 64 * j] = t[j];
  }
  RegW<NREG> rw;
#pragma unroll
  for (int r = 0; r < NREG; ++r) loadA(rw.w[r], p.wfa + (size_t)wv_lin(NB, NLDS + r) * 4096, lane);
  for (int i = lane; i < p.n_tok * 192; i += 64) QT[i] = f2bf(p.qkv0[i]);
  if constexpr (!WIDE)
    for (int i = lane; i < p.n_tok * 64; i += 64) ((float*)(smem + lo.et))[i] = p.emb[i];
  for (int i = lane; i < (10 * NB + 1) * 64; i += 64) BI[i] = p.bias[i];
  for (int i = lane; i < (3 * NB + 1) * 128; i += 64) LP[i] = p.lnp[i];
  for (int i = lane * 8; i < (NB * 4 * L + 32) * 64; i += 512) *(uint4*)(KV + i) = make_uint4(0, 0, 0, 0);
  WvHeadW<MA> hw;
  wv_head_load<MA>(hw, p, lane);
  // cross-attention queries of every row and block: q2 = W_q2 rep + b (bf16, as the 4-wave kernel rounds them)
  const float* rep = p.rep + (size_t)env * L * 64;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    AFr wq;
    loadA(wq, p.wfa + (size_t)(10 * b + 4) * 4096, lane);
    const CT bq = ld_vec(p.bias + (10 * b + 4) * 64, lane);
    for (int t0 = 0; t0 < L; t0 += 16) {
      const int row = t0 + c;
      CT xr;
      if (row < L) xr = ld_vec(rep + (size_t)row * 64, lane); else ct_zero(xr);
      CT q = bq;
      mm(q, wq, ct_pack(xr));
      const CTr qp = ct_pack(q);
      if (row < L) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) *(uint2*)(Q2 + (size_t)(b * L + row) * 64 + 16 * mt + 4 * g) = qp.q[mt];
      }
    }
  }
  const WvNoise nz = wv_noise_load(p, env, lane);
  __syncthreads();

  // ---------------------------------------------------------------- agent loop
  const WvCtx k{W, KV, Q2, QT, ET, BI, LP, lane, L};
  const float* ava = p.ava ? p.ava + (size_t)env * L * A : nullptr;
  int tok = p.tok_start;
#pragma unroll 1
  for (int i = 0; i < L; ++i) {
    // per-row inputs, requested before the block chain that hides their latency: rep_i (residual of the cross
    // attention), the availability row (lane a = action a)
    const CT repi = ld_vec(rep + (size_t)i * 64, lane);
    const float avl = (ava && lane < A) ? ava[(size_t)i * A + lane] : 1.f;
    CT x;
    wv_block<0, NB, NLDS, NREG>(x, k, rw, i, tok, repi);
    if constexpr (NB > 1) wv_block<1, NB, NLDS, NREG>(x, k, rw, i, tok, repi);
    tok = wv_head_sample<NM, NLDS, NREG, MA>(x, hw, nz, rw, W, BI, SC, p, env, i, avl, tok, lane);
  }
}

// ================================================================================================ speculative block 0
// mat_decode_spec_kernel: the one-wave kernel's agent chain split over 1 + NS waves of one workgroup.  Block 0 of
// row i + 1 depends on the previous agents only through its input token (the action of agent i) and the committed
// cache rows 0..i; every candidate token is known in advance (1 + a, a < act_dim).  So while the MAIN wave (wave 0)
// runs blocks 1.. and the head of row i (the one-wave kernel's code: replicated live row, folded head, sampling),
// the SPECULATIVE waves (1..NS) run block 0 of row i + 1 for ALL candidate tokens at once — one candidate per MFMA
// token column, 16 per wave (the one-wave kernel replicates its live row over those 16 columns, so the candidates
// cost about what the replicated row did).  One workgroup barrier per agent step hands over:
//   main -> spec : the sampled token (TOK[parity]);
//   spec -> main : block 0's output row of every candidate (SLOT[parity][cand], fp32) — main reads its token's row;
//   spec -> spec : the staged cross-attention K / V rows of every candidate (STG[parity][cand]); after the barrier
//                  every spec wave commits the chosen candidate's rows (and the token's self-attention K / V table
//                  rows) to the block-0 caches itself (identical values, so the waves' writes never conflict).
// The critical path per agent step drops from blocks 0 + 1 + head to max(blocks 1 + head, block 0) + one barrier.
// Block-0 weights live in the speculative waves' registers (6 matrices, 192 VGPRs each), the main wave's matrices
// in LDS (the last NREG in its registers).  Rows of the candidate attention: keys 0..i-1 from the committed cache
// (MFMA, as the one-wave kernel), the candidate's own key i from its registers (a per-column dot product), both
// heads in separate score MFMAs (columns are no longer replicated).  Reference: transformer_act.py:76-99.
// IND (long rows, L = 101): block 0's self-attention K / V rows are the token table's rows, so instead of two caches of
// L rows the kernel keeps the row -> token array ROWTOK and reads K / V through it (25 KB less LDS at L = 101)
struct SpLds { int w, kv, q2, qt, bi, lp, sc, slot, stg, tok, rowtok, total; };
// Q2F (L = 129): no cross-attention query table either — the main wave computes block 1's query of its row from
// W_q2 (one more LDS matrix), the speculative waves block 0's from a register copy of W_q2
// PAIR (act_dim <= 2): MDL_SPEC_PAIR=0 builds keep the 16-candidate layout (A/B).  MDL_SPEC_STQ=1 (A/B, off: 256 x 33
// 147.2 -> 151.5 us, 256 x 101 534 -> 528, 256 x 129 720 -> 697 us — the speculative wave became the critical path at
// the headline shape): PAIR also stages block 1's q / k / v rows of every candidate and the main wave skips them
#ifndef MDL_SPEC_PAIR
#define MDL_SPEC_PAIR 1
#endif
#ifndef MDL_PAIR_ROR_OLD
#define MDL_PAIR_ROR_OLD 0
#endif
#ifndef MDL_SPEC_STQ
#define MDL_SPEC_STQ 0
#endif
// (when block 1's q / k / v weights are LDS-resident: at most 6 main-wave register matrices)
__host__ __device__ inline bool sp_stq(int A, int nreg) { return MDL_SPEC_STQ && MDL_SPEC_PAIR && A <= 2 && nreg <= 6; }
__host__ __device__ inline SpLds sp_lds(int NB, int L, int n_tok, int nlds_main, int A, bool ind, bool q2f = false) {
  SpLds o;
  int off = 0;
  auto take = [&](int bytes) { const int r = off; off += (bytes + 15) & ~15; return r; };
  o.w = take((nlds_main + (q2f ? 1 : 0)) * 8192);   // the main wave's LDS-resident matrices (blocks 1.., head)
  o.kv = take(((NB * 4 - (ind ? 2 : 0)) * L + 32) * 128);   // K / V caches (+ 32 zero rows)
  o.q2 = take(q2f ? 0 : NB * L * 128);       // cross-attention queries
  o.qt = take(n_tok * 3 * 128);              // block-0 q / k / v of every token
  o.bi = take((10 * NB + 1) * 256);
  o.lp = take((3 * NB + 1) * 512);
  o.sc = take(64 * 4);
  o.slot = take(2 * A * 256);                // [parity][candidate][64] f32 block-0 outputs
  o.stg = take(2 * A * (sp_stq(A, wv_nm(NB) - 6 - nlds_main) ? 640 : 256));   // [parity][candidate][rows][64] bf16: block 0's cross K / V
                                                    // (+ block 1's q, k, v: PAIR)
  o.tok = take(16);                          // [parity] token of the next row
  o.rowtok = take(ind ? ((L + 31) & ~31) * 4 : 0);   // IND: input token of every committed row (0 beyond)
  o.total = off;
  return o;
}

// Causal attention of row i for the wave's 16 candidates (column c): keys 0..i-1 from the committed caches, key i the
// candidate's own (ks, vs).  Online softmax per head in log2 units, seeded with the own key (score m, weight 1,
// value vs), so every row has a finite running max and no chunk needs a FIRST special case.
// K / V row sources of the committed keys: a swizzled cache (SpCache) or, IND, the token table through ROWTOK
struct SpCache {
  const bf16_t *K, *V;
  __device__ __forceinline__ uint2 k4(int row, int col) const { return kv_ld2(K, row, col); }
  __device__ __forceinline__ bf16x8 vT(int kb, int n0, int lane) const { return ld_frag_T(V + kb * 64, 0, n0, lane); }
};
struct SpTokRows {
  const bf16_t* QT;
  const int* rowtok;
  __device__ __forceinline__ uint2 k4(int row, int col) const {
    return *(const uint2*)(QT + rowtok[row] * 192 + 64 + col);
  }
  // ld_frag_T over rows kb + 8g + (c >> 2) (+ 4) of the V table rows: every lane addresses its own row
  __device__ __forceinline__ bf16x8 vT(int kb, int n0, int lane) const {
    const int g = lane >> 4, c = lane & 15, col = n0 + 4 * (c & 3);
    const int r0 = kb + 8 * g + (c >> 2);
    const s16x4 lo = ld_tr(QT + rowtok[r0] * 192 + 128 + col), hi = ld_tr(QT + rowtok[r0 + 4] * 192 + 128 + col);
    bf16x8 f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
};
template <class KVS>
__device__ __forceinline__ CT sp_attn(const KVS& kvs, const CTr& q, const CTr& ks, const CTr& vs, int i, int lane) {
  const int g = lane >> 4, c = lane & 15;
  float m[2], l[2];
  f32x4 o[4];
  {
    const CT qf = ct_unpack(q), kf = ct_unpack(ks), vf = ct_unpack(vs);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 d = qf.v[2 * h] * kf.v[2 * h] + qf.v[2 * h + 1] * kf.v[2 * h + 1];
      m[h] = cross_row_sum((d[0] + d[1]) + (d[2] + d[3])) * ATT_L2;
      l[h] = g == 0 ? 1.f : 0.f;   // the own key's weight, counted once per column
      o[2 * h] = vf.v[2 * h];
      o[2 * h + 1] = vf.v[2 * h + 1];
    }
  }
  const bf16x8 qb0 = rb(q, 0), qb1 = rb(q, 1);
  for (int kb = 0; kb < i; kb += 32) {
    float sc[2][8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = kb + pi_row(t, c);
      const uint2 p0 = kvs.k4(key, 4 * g), p1 = kvs.k4(key, 16 + 4 * g);
      const uint2 p2 = kvs.k4(key, 32 + 4 * g), p3 = kvs.k4(key, 48 + 4 * g);
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 r0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mk8(p0.x, p0.y, p1.x, p1.y), qb0, z, 0, 0, 0);
      const f32x4 r1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mk8(p2.x, p2.y, p3.x, p3.y), qb1, z, 0, 0, 0);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        sc[0][4 * t + rr] = r0[rr];
        sc[1][4 * t + rr] = r1[rr];
      }
    }
    const int d0 = i - 1 - kb - 8 * g;   // key kb + 8g + j is committed (< i) iff j <= d0
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float cm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[h][j] = j <= d0 ? sc[h][j] : -INFINITY;
        cm = fmaxf(cm, sc[h][j]);
      }
      const float nm = fmaxf(m[h], cross_row_max(cm) * ATT_L2);
      const float alpha = fast_exp2(m[h] - nm);
      float ps = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[h][j] = fast_exp2(fmaf(sc[h][j], ATT_L2, -nm));
        ps += sc[h][j];
      }
      l[h] = l[h] * alpha + ps;
      bf16x8 ph, pl;
      split8v(sc[h], ph, pl);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int mt = 2 * h + u;
        const bf16x8 va = kvs.vT(kb, 16 * mt, lane);
        o[mt] *= alpha;
        o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, ph, o[mt], 0, 0, 0);
        o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pl, o[mt], 0, 0, 0);
      }
      m[h] = nm;
    }
  }
  CT O;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float il = 1.f / cross_row_sum(l[h]);
    O.v[2 * h] = o[2 * h] * il;
    O.v[2 * h + 1] = o[2 * h + 1] * il;
  }
  return O;
}

// PAIR (act_dim <= 2, the DCML rollout): two candidates, so the 16 token columns hold (candidate c >> 3, head
// (c >> 2) & 1, 4 replicas) instead of 16 candidates.  Both heads then share one online-softmax pass (each column
// scores only its head's 32 dims; the other head's half of O comes from the partner column c ^ 4 by a bank-masked
// DPP rotation), and GELU costs 2 erf per lane (each lane evaluates one packed feature pair of its candidate, 8
// row broadcasts + a half select hand every lane its candidate's 8 packed words) instead of 16.
template <int CTRL, int BANKS>
__device__ __forceinline__ float dpp_banks(float x) {
  const int a = __builtin_bit_cast(int, x);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(a, a, CTRL, 0xF, BANKS, false));
}
template <int CTRL, int BANKS>
__device__ __forceinline__ f32x4 dpp_banks4(f32x4 v) {
  return f32x4{dpp_banks<CTRL, BANKS>(v.x), dpp_banks<CTRL, BANKS>(v.y), dpp_banks<CTRL, BANKS>(v.z),
               dpp_banks<CTRL, BANKS>(v.w)};
}
template <class KVS>
__device__ __forceinline__ CT sp_attn_pair(const KVS& kvs, const CTr& q, const CTr& ks, const CTr& vs, int i, int lane) {
  const int g = lane >> 4, c = lane & 15, hd = (c >> 2) & 1;
  float m, l;
  f32x4 o[4];
  {
    const CT qf = ct_unpack(q), kf = ct_unpack(ks), vf = ct_unpack(vs);
    const f32x4 d = hd ? qf.v[2] * kf.v[2] + qf.v[3] * kf.v[3] : qf.v[0] * kf.v[0] + qf.v[1] * kf.v[1];
    m = cross_row_sum((d[0] + d[1]) + (d[2] + d[3])) * ATT_L2;
    l = g == 0 ? 1.f : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) o[mt] = vf.v[mt];
  }
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16x8 qb0 = hd ? z8 : rb(q, 0), qb1 = hd ? rb(q, 1) : z8;
  for (int kb = 0; kb < i; kb += 32) {
    float sc[8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = kb + pi_row(t, c);
      const uint2 p0 = kvs.k4(key, 4 * g), p1 = kvs.k4(key, 16 + 4 * g);
      const uint2 p2 = kvs.k4(key, 32 + 4 * g), p3 = kvs.k4(key, 48 + 4 * g);
      f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mk8(p0.x, p0.y, p1.x, p1.y), qb0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mk8(p2.x, p2.y, p3.x, p3.y), qb1, r, 0, 0, 0);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) sc[4 * t + rr] = r[rr];
    }
    const int d0 = i - 1 - kb - 8 * g;   // key kb + 8g + j is committed (< i) iff j <= d0
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = j <= d0 ? sc[j] : -INFINITY;
      cm = fmaxf(cm, sc[j]);
    }
    const float nm = fmaxf(m, cross_row_max(cm) * ATT_L2);
    const float alpha = fast_exp2(m - nm);
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = fast_exp2(fmaf(sc[j], ATT_L2, -nm));
      ps += sc[j];
    }
    l = l * alpha + ps;
    bf16x8 ph, pl;
    split8v(sc, ph, pl);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const bf16x8 va = kvs.vT(kb, 16 * mt, lane);
      o[mt] *= alpha;
      o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, ph, o[mt], 0, 0, 0);
      o[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pl, o[mt], 0, 0, 0);
    }
    m = nm;
  }
  const float il = 1.f / cross_row_sum(l);
  CT O;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) O.v[mt] = o[mt] * il;
  // head-0 columns (banks 0, 2) take head 1's dims from column c + 4, head-1 columns (banks 1, 3) head 0's from c - 4.
  // row_ror:N moves a value N lanes UP the row (lane c reads lane c - N mod 16, tests/native/dpp_ror_probe.hip), so
  // "from c + 4" is row_ror:12 and "from c - 4" row_ror:4.  (Rounds 5: the two were swapped — each candidate took the
  // OTHER candidate's second head, invisible with near-identical candidates (random-init weights) but 0.1 nats of
  // log-prob error per row with a trained policy; MDL_PAIR_ROR_OLD=1 rebuilds that variant for the A/B check.)
#if MDL_PAIR_ROR_OLD
  constexpr int ROR_UP = 0x124, ROR_DN = 0x12C;
#else
  constexpr int ROR_UP = 0x12C, ROR_DN = 0x124;
#endif
  O.v[2] = dpp_banks4<ROR_UP, 0x5>(O.v[2]);
  O.v[3] = dpp_banks4<ROR_UP, 0x5>(O.v[3]);
  O.v[0] = dpp_banks4<ROR_DN, 0xA>(O.v[0]);
  O.v[1] = dpp_banks4<ROR_DN, 0xA>(O.v[1]);
  return O;
}
// packed word K of this lane's candidate half: lane K (lower half) or 8 + K (upper half) of the row
template <int K>
__device__ __forceinline__ uint32_t pair_word(float pk, bool up) {
  return __builtin_bit_cast(uint32_t, up ? row_bcast<8 + K>(pk) : row_bcast<K>(pk));
}
// GELU of the PAIR layout as the packed bf16 MFMA operand: lane (c & 7) = j evaluates features 2j, 2j + 1 of its row
// (packed word j = CTr q[j >> 1] half j & 1); 8 row broadcasts per candidate half
__device__ __forceinline__ CTr gelu_pair_pk(const CT& h, int lane) {
  const int c = lane & 15, j = c & 7;
  const f32x4 a01 = (j & 2) ? h.v[1] : h.v[0], a23 = (j & 2) ? h.v[3] : h.v[2];   // feature tile j >> 1
  const f32x4 a = (j & 4) ? a23 : a01;
  const float lo = (j & 1) ? a[2] : a[0], hi = (j & 1) ? a[3] : a[1];
  const float pk = __builtin_bit_cast(float, pk2(gelu_erf(lo), gelu_erf(hi)));
  const bool up = c & 8;
  CTr o;
  o.q[0] = make_uint2(pair_word<0>(pk, up), pair_word<1>(pk, up));
  o.q[1] = make_uint2(pair_word<2>(pk, up), pair_word<3>(pk, up));
  o.q[2] = make_uint2(pair_word<4>(pk, up), pair_word<5>(pk, up));
  o.q[3] = make_uint2(pair_word<6>(pk, up), pair_word<7>(pk, up));
  return o;
}

// block 0 (ma_transformer.py:95-98) of row i for the wave's 16 candidates: x = the candidates' embedded input rows in,
// block 0's output out; kp / vp = their cross-attention K / V rows (staged for the commit)
template <bool PAIR, class KVS>
__device__ __forceinline__ void sp_block0(CT& x, const CTr& cq, const CTr& ck, const CTr& cv, const RegW<6>& w0,
                                          const WvCtx& k, const KVS& selfkv, int i, const CT& repi, const CTr& q2,
                                          CTr& kp, CTr& vp) {
  const int lane = k.lane, g = lane >> 4, L = k.L;
  CT xh;
  {
    CT O;
    if constexpr (PAIR) O = sp_attn_pair(selfkv, cq, ck, cv, i, lane);
    else O = sp_attn(selfkv, cq, ck, cv, i, lane);
    CT t = ct_add(ld_vec(k.BI + 64 * 3, lane), x);
    mm(t, w0.w[0], ct_pack(O));
    ln_fwd_ct(t, xh, x, ld_vec(k.LP, lane), ld_vec(k.LP + 64, lane));
  }
  {
    const CTr xp = ct_pack(x);
    CT kk = ld_vec(k.BI + 64 * 5, lane), vv = ld_vec(k.BI + 64 * 6, lane);
    mm(kk, w0.w[1], xp);
    mm(vv, w0.w[2], xp);
    kp = ct_pack(kk);
    vp = ct_pack(vv);
  }
  {
    const SpCache cross{wv_cache(k.KV, 0, 2, L), wv_cache(k.KV, 0, 3, L)};
    CT O;
    if constexpr (PAIR) O = sp_attn_pair(cross, q2, kp, vp, i, lane);
    else O = sp_attn(cross, q2, kp, vp, i, lane);
    CT t = ct_add(ld_vec(k.BI + 64 * 7, lane), repi);
    mm(t, w0.w[3], ct_pack(O));
    ln_fwd_ct(t, xh, x, ld_vec(k.LP + 128, lane), ld_vec(k.LP + 128 + 64, lane));
  }
  {
    CT h = ld_vec(k.BI + 64 * 8, lane);
    mm(h, w0.w[4], ct_pack(x));
    CTr hp;
    if constexpr (PAIR) {
      hp = gelu_pair_pk(h, lane);
    } else {
      gelu_ct(h);
      hp = ct_pack(h);
    }
    CT t = ct_add(ld_vec(k.BI + 64 * 9, lane), x);
    mm(t, w0.w[5], hp);
    ln_fwd_ct(t, xh, x, ld_vec(k.LP + 256, lane), ld_vec(k.LP + 256 + 64, lane));
  }
}

// candidate token constants of one lane: block-0 q / k / v table rows (bf16) and the embedded input row (f32)
struct SpCand { CTr q, k, v; CT e; };
__device__ __forceinline__ SpCand sp_cand(const bf16_t* QT, const float* emb, int tok, int lane) {
  const int g = lane >> 4;
  SpCand cd;
  const bf16_t* t = QT + tok * 192;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    cd.q.q[mt] = *(const uint2*)(t + 16 * mt + 4 * g);
    cd.k.q[mt] = *(const uint2*)(t + 64 + 16 * mt + 4 * g);
    cd.v.q[mt] = *(const uint2*)(t + 128 + 16 * mt + 4 * g);
  }
  cd.e = ld_vec(emb + tok * 64, lane);
  return cd;
}

// q2 = W_q2 rep + b (bf16) of one row: the query table's values, computed in place (Q2F)
__device__ __forceinline__ CTr sp_q2(const AFr& wq, const float* bias, const CT& repr, int lane) {
  CT q = ld_vec(bias, lane);
  mm(q, wq, ct_pack(repr));
  return ct_pack(q);
}

template <int NB, int NS, int NREG, int MA, bool IND, bool Q2F, bool PAIR>
__global__ __launch_bounds__(64 * (1 + NS), 1) void mat_decode_spec_kernel(DecParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef MDL_SPEC_PROF
  const unsigned long long spp_t0 = __builtin_amdgcn_s_memtime();
#endif
  constexpr int NM = wv_nm(NB), NMM = NM - 6, NLDS = NM - NREG;   // main: slots 6 .. NM - 1, LDS: 6 .. NLDS - 1
  constexpr int NT = 64 * (1 + NS);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int env = blockIdx.x, L = p.L, A = p.act_dim;
  static_assert(!Q2F || NB == 2, "Q2F: n_block 2");
  const SpLds lo = sp_lds(NB, L, p.n_tok, NMM - NREG, A, IND, Q2F);
  bf16_t* Wl = (bf16_t*)(smem + lo.w);
  bf16_t* KV = (bf16_t*)(smem + lo.kv) - (IND ? 2 * L * 64 : 0);   // IND: no block-0 self K / V caches (kinds 0, 1)
  int* ROWTOK = (int*)(smem + lo.rowtok);
  bf16_t* Q2 = (bf16_t*)(smem + lo.q2);
  bf16_t* QT = (bf16_t*)(smem + lo.qt);
  float* BI = (float*)(smem + lo.bi);
  float* LP = (float*)(smem + lo.lp);
  float* SC = (float*)(smem + lo.sc);
  float* SLOT = (float*)(smem + lo.slot);
  bf16_t* STG = (bf16_t*)(smem + lo.stg);
  int* TOK = (int*)(smem + lo.tok);
  constexpr bool STQ = MDL_SPEC_STQ && PAIR && NREG <= 6;   // = sp_stq
  constexpr int SR = STQ ? 320 : 128;     // staged bf16 elements per candidate
  const float* rep = p.rep + (size_t)env * L * 64;

  // ---------------------------------------------------------------- setup (all waves)
  for (int e = tid; e < (NLDS - 6 + (Q2F ? 1 : 0)) * 512; e += NT) {
    const int sl = 6 + e / 512, j = e % 512;
    const int lin = sl < NLDS ? wv_lin(NB, sl) : 10 * 1 + 4;   // Q2F: block 1's W_q2 after the main wave's slots
    ((uint4*)(Wl + (size_t)(sl - 6) * 4096))[j] = ((const uint4*)(p.wfa + (size_t)lin * 4096))[j];
  }
  for (int e = tid; e < p.n_tok * 192; e += NT) QT[e] = f2bf(p.qkv0[e]);
  for (int e = tid; e < (10 * NB + 1) * 64; e += NT) BI[e] = p.bias[e];
  for (int e = tid; e < (3 * NB + 1) * 128; e += NT) LP[e] = p.lnp[e];
  {
    bf16_t* kv0 = (bf16_t*)(smem + lo.kv);
    for (int e = tid * 8; e < ((NB * 4 - (IND ? 2 : 0)) * L + 32) * 64; e += NT * 8) *(uint4*)(kv0 + e) = make_uint4(0, 0, 0, 0);
    if constexpr (IND)
      for (int e = tid; e < ((L + 31) & ~31); e += NT) ROWTOK[e] = 0;
  }
  // cross-attention queries q2 = W_q2 rep + b of every row and block, 16-row tiles spread over the waves
  if constexpr (!Q2F) {
    const int ntile = (L + 15) >> 4;
    for (int jt = wave; jt < NB * ntile; jt += 1 + NS) {
      const int b = jt / ntile, t0 = 16 * (jt % ntile);
      AFr wq;
      loadA(wq, p.wfa + (size_t)(10 * b + 4) * 4096, lane);
      const int row = t0 + c;
      CT xr;
      if (row < L) xr = ld_vec(rep + (size_t)row * 64, lane); else ct_zero(xr);
      CT q = ld_vec(p.bias + (10 * b + 4) * 64, lane);
      mm(q, wq, ct_pack(xr));
      const CTr qp = ct_pack(q);
      if (row < L) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) *(uint2*)(Q2 + (size_t)(b * L + row) * 64 + 16 * mt + 4 * g) = qp.q[mt];
      }
    }
  }
  __syncthreads();

  const WvCtx k{Wl - 6 * 4096, KV, Q2, QT, p.emb, BI, LP, lane, L};
  if (wave == 0) {
    // ---------------------------------------------------------------- main wave: blocks 1.., head, sampling
    RegW<NREG> rw;
#pragma unroll
    for (int r = 0; r < NREG; ++r) loadA(rw.w[r], p.wfa + (size_t)wv_lin(NB, NLDS + r) * 4096, lane);
    WvHeadW<MA> hw;
    wv_head_load<MA>(hw, p, lane);
    const WvNoise nz = wv_noise_load(p, env, lane);
    const float* ava = p.ava ? p.ava + (size_t)env * L * A : nullptr;
    int tok = p.tok_start;
    if (lane == 0) TOK[0] = tok;
    __syncthreads();   // (1) row 0's block 0 is staged
    SPP_DECL;
#ifdef MDL_SPEC_PROF
    spp_acc[3] = spp_t - spp_t0;   // 3: setup + row 0's block 0 (kernel start -> first agent step)
#endif
#pragma unroll 1
    for (int i = 0; i < L; ++i) {
      SPP(0);   // 0: barrier wait
      const CT repi = ld_vec(rep + (size_t)i * 64, lane);
      const float avl = (ava && lane < A) ? ava[(size_t)i * A + lane] : 1.f;
      const int cidx = (i & 1) * A + (i == 0 ? 0 : tok - 1);
      CT x = ld_vec(SLOT + (size_t)cidx * 64, lane);
      const bf16_t* stq = STG + (size_t)cidx * SR + 128;   // PAIR: the staged q / k / v of block 1
      if constexpr (Q2F) {
        AFr wq;
        wv_getw<0, 1, 0>(wq, RegW<0>{}, Wl + (size_t)(NLDS - 6) * 4096, lane);
        const CTr q2 = sp_q2(wq, BI + 64 * (10 * 1 + 4), repi, lane);
        wv_block<1, NB, NLDS, NREG, STQ>(x, k, rw, i, tok, repi, &q2, stq);
      } else if constexpr (NB > 1) {
        wv_block<1, NB, NLDS, NREG, STQ>(x, k, rw, i, tok, repi, nullptr, stq);
      }
      SPP(1);   // 1: slot read + block 1
#ifdef MDL_SPEC_PROF
      unsigned long long hp[17] = {0};
      hp[16] = spp_t;
      tok = wv_head_sample<NM, NLDS, NREG, MA>(x, hw, nz, rw, k.W, BI, SC, p, env, i, avl, tok, lane, hp);
      for (int k_ = 8; k_ < 14; ++k_) spp_acc[k_] += hp[k_];
      spp_t = hp[16];
#else
      tok = wv_head_sample<NM, NLDS, NREG, MA>(x, hw, nz, rw, k.W, BI, SC, p, env, i, avl, tok, lane);
#endif
      if (lane == 0) TOK[(i + 1) & 1] = tok;
      SPP(2);   // 2: head + sampling (rest)
      __syncthreads();   // (2) token of row i + 1 published; block 0 of row i + 1 staged for every candidate
    }
    SPP_END(0);
  } else {
    // ---------------------------------------------------------------- speculative waves: block 0 of the next row
    RegW<6> w0;
#pragma unroll
    for (int r = 0; r < 6; ++r) loadA(w0.w[r], p.wfa + (size_t)wv_lin(NB, r) * 4096, lane);
    RegW<Q2F ? 1 : 0> wq0;   // Q2F: block 0's W_q2
    if constexpr (Q2F) loadA(wq0.w[0], p.wfa + (size_t)4 * 4096, lane);
    auto q2row = [&](int row, const CT& repr) {
      CTr q2;
      if constexpr (Q2F) {
        q2 = sp_q2(wq0.w[0], BI + 64 * 4, repr, lane);
      } else {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) q2.q[mt] = *(const uint2*)(Q2 + (size_t)row * 64 + 16 * mt + 4 * g);
      }
      return q2;
    };
    const auto selfkv = [&] {
      if constexpr (IND) return SpTokRows{QT, ROWTOK};
      else return SpCache{wv_cache(KV, 0, 0, L), wv_cache(KV, 0, 1, L)};
    }();
    // this lane's candidate: input token 1 + cand (rows >= 1); PAIR: columns c >> 3, one writer column each
    const int cand = PAIR ? c >> 3 : 16 * (wave - 1) + c;
    const bool own = cand < A && (!PAIR || (c & 7) == 0);
    auto stage = [&](int par, const CT& x, const CTr& kp, const CTr& vp) {
      CTr pr[3];   // PAIR: block 1's q / k / v of the candidate's block-0 output (weights: the main wave's LDS slots)
      if constexpr (STQ && NB > 1) {
        const CTr xp = ct_pack(x);
        AFr w;
        wv_getw<wv_slot(1, 0), NLDS, 0>(w, RegW<0>{}, k.W, lane);
        CT t0 = ld_vec(BI + 64 * 10, lane);
        mm(t0, w, xp);
        wv_getw<wv_slot(1, 1), NLDS, 0>(w, RegW<0>{}, k.W, lane);
        CT t1 = ld_vec(BI + 64 * 11, lane);
        mm(t1, w, xp);
        wv_getw<wv_slot(1, 2), NLDS, 0>(w, RegW<0>{}, k.W, lane);
        CT t2 = ld_vec(BI + 64 * 12, lane);
        mm(t2, w, xp);
        pr[0] = ct_pack(t0);
        pr[1] = ct_pack(t1);
        pr[2] = ct_pack(t2);
      }
      if (own) {
        float* sl = SLOT + (size_t)(par * A + cand) * 64;
        bf16_t* st = STG + (size_t)(par * A + cand) * SR;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          *(f32x4*)(sl + 16 * mt + 4 * g) = x.v[mt];
          *(uint2*)(st + 16 * mt + 4 * g) = kp.q[mt];
          *(uint2*)(st + 64 + 16 * mt + 4 * g) = vp.q[mt];
          if constexpr (STQ && NB > 1) {
#pragma unroll
            for (int j = 0; j < 3; ++j) *(uint2*)(st + 128 + 64 * j + 16 * mt + 4 * g) = pr[j].q[mt];
          }
        }
      }
    };
    {   // row 0: every column runs the start token
      const SpCand c0 = sp_cand(QT, p.emb, p.tok_start, lane);
      CT x = c0.e;
      CTr kp, vp;
      const CT rep0 = ld_vec(rep, lane);
      sp_block0<PAIR>(x, c0.q, c0.k, c0.v, w0, k, selfkv, 0, rep0, q2row(0, rep0), kp, vp);
      stage(0, x, kp, vp);
    }
    const SpCand cd = sp_cand(QT, p.emb, min(1 + cand, p.n_tok - 1), lane);
    __syncthreads();   // (1)
    SPP_DECL;
#ifdef MDL_SPEC_PROF
    spp_acc[3] = spp_t - spp_t0;
#endif
#pragma unroll 1
    for (int i = 0; i < L; ++i) {
      SPP(4);   // 4: barrier wait
      const CT repn = ld_vec(rep + (size_t)min(i + 1, L - 1) * 64, lane);
      // commit row i of the block-0 caches: the token's self-attention K / V table rows and the staged cross K / V
      // rows of its candidate; lane (kind, 16-byte chunk), kinds 0..3 = self K, self V, cross K, cross V
      const int tk = TOK[i & 1];
      if (IND && lane == 0) ROWTOK[i] = tk;
      if (lane < 32 && (!IND || lane >= 16)) {
        const int kind = lane >> 3, ch = lane & 7;
        const bf16_t* src = kind < 2 ? QT + tk * 192 + 64 * (kind + 1) + 8 * ch
                                     : STG + (size_t)((i & 1) * A + (i == 0 ? 0 : tk - 1)) * SR + 64 * (kind - 2) + 8 * ch;
        *(uint4*)(wv_cache(KV, 0, kind, L) + tmo(i, 8 * ch)) = *(const uint4*)src;
      }
      asm volatile("" ::: "memory");   // the committed row is read back by other lanes below (LDS is in order per wave)
      SPP(5);   // 5: commit
      if (i + 1 < L) {
        CT x = cd.e;
        CTr kp, vp;
        sp_block0<PAIR>(x, cd.q, cd.k, cd.v, w0, k, selfkv, i + 1, repn, q2row(i + 1, repn), kp, vp);
        SPP(6);   // 6: block 0
        stage((i + 1) & 1, x, kp, vp);
        SPP(7);   // 7: staging stores
      }
      __syncthreads();   // (2)
    }
    SPP_END(wave == 1 ? 1 : -1);
  }
}

template <int NB, int NS, int NREG, int MA, bool IND, bool Q2F>
int sp_launch_wide(const DecParams* p, size_t lds, hipStream_t st) {   // 3..4 narrow-head actions: 16-candidate layout
  hipError_t e = hipFuncSetAttribute((const void*)mat_decode_spec_kernel<NB, NS, NREG, MA, IND, Q2F, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((mat_decode_spec_kernel<NB, NS, NREG, MA, IND, Q2F, false>), dim3(p->B), dim3(64 * (1 + NS)), lds, st, *p);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}
template <int NB, int NS, int NREG, int MA, bool IND = false, bool Q2F = false>
int sp_launch(const DecParams* p, size_t lds, hipStream_t st) {
  constexpr bool PAIR = MDL_SPEC_PAIR && NS == 1 && MA == 1;
  if (PAIR && p->act_dim > 2) return sp_launch_wide<NB, NS, NREG, MA, IND, Q2F>(p, lds, st);
  hipError_t e = hipFuncSetAttribute((const void*)mat_decode_spec_kernel<NB, NS, NREG, MA, IND, Q2F, PAIR>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((mat_decode_spec_kernel<NB, NS, NREG, MA, IND, Q2F, PAIR>), dim3(p->B), dim3(64 * (1 + NS)), lds, st, *p);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}
template <int NS, int MA>
int sp_launch_nreg(const DecParams* p, int nreg, size_t lds, hipStream_t st) {
  switch (nreg) {
    case 2: return sp_launch<2, NS, 2, MA>(p, lds, st);
    case 4: return sp_launch<2, NS, 4, MA>(p, lds, st);
    case 6: return sp_launch<2, NS, 6, MA>(p, lds, st);
    case 8:   // the narrow head only (465 VGPRs; the wide head's folded logit fragments spill with 8)
      if constexpr (MA == 1) return sp_launch<2, NS, 8, MA>(p, lds, st);
      return -1;
    default: return sp_launch<2, NS, 0, MA>(p, lds, st);
  }
}

template <int NB, int NREG, int MA>
int wv_launch_ma(const DecParams* p, size_t lds, hipStream_t st) {
  hipError_t e = hipFuncSetAttribute((const void*)mat_decode_wave_kernel<NB, NREG, MA>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((mat_decode_wave_kernel<NB, NREG, MA>), dim3(p->B), dim3(64), lds, st, *p);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}
template <int NB, int NREG>
int wv_launch(const DecParams* p, bool wide, size_t lds, hipStream_t st) {
  if (!wide) return wv_launch_ma<NB, NREG, 1>(p, lds, st);
  return p->act_dim <= 48 ? wv_launch_ma<NB, NREG, 3>(p, lds, st) : wv_launch_ma<NB, NREG, 4>(p, lds, st);
}

}  // namespace

#ifdef MDL_WAVE_DEBUG
MDL_API int mdl_wave_debug_read(float* out, int row) {
  if (row >= 0) return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_wdbg_row), &row, sizeof(int));
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wdbg), sizeof(float) * 16 * 64, 0, hipMemcpyDeviceToHost);
}
#endif

// The one-wave path: one-row token passes (stride 1: every stochastic rollout step; deterministic decisions with
// stride 1) of the Discrete / Semi_Discrete(-1) action types with the block-0 token table and the folded head,
// n_block 1 or 2, L up to what the LDS carve holds (weights beyond it in registers, at most 6 matrices).
// Returns the number of register-resident weight matrices of the launch it would make, or -1 (not on this path).
static bool wv_eligible(const DecParams* p, int NB) {
  if (!p->wfa || p->cont || p->avail_cont || !p->qkv0 || !p->hfold || !p->rep || p->epw != 1) return false;
  if (NB < 1 || NB > 2 || p->act_dim < 1 || p->act_dim > 64 || p->stride != 1 || p->L < 1 || p->L > 192) return false;
  if (p->n_disc != p->L && p->n_disc != p->L - 1) return false;
  if (!p->deterministic && !p->gen && (!p->rnd_u || (p->n_disc < p->L && !p->rnd_n))) return false;
  return true;
}
#ifdef MDL_SPEC_PROF
MDL_API int mdl_spec_prof_read(unsigned long long* out, int reset) {
  if (reset) {
    static const unsigned long long z[32] = {0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_spprof), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spprof), sizeof(unsigned long long) * 32, 0, hipMemcpyDeviceToHost);
}
#endif
MDL_API int mdl_decode_wave_plan(const DecParams* p, int NB) {
  if (!wv_eligible(p, NB)) return -1;
  for (int nreg = 0; nreg <= (NB == 1 ? 4 : 6); nreg += 2)
    if (wv_lds(NB, p->L, p->n_tok, wv_nm(NB) - nreg, p->act_dim > 4).total <= 160 * 1024) return nreg;
  return -1;
}

// The speculative-block-0 path (mat_decode_spec_kernel): n_block 2 one-wave-path calls with act_dim <= 48 (one to
// three speculative waves).  MAT_DCML_DECODE_SPEC=0 or mdl_decode_spec_enable(0) keeps the one-wave kernel.
// Returns the number of register-resident main-wave matrices, or -1 (not on this path).
static int g_spec_enable = -1;
MDL_API void mdl_decode_spec_enable(int on) { g_spec_enable = on; }
// tests: 1 = the token-table layout, 2 = token table + in-place queries even where the plain carve fits; 0 = auto
static int g_spec_layout = 0;
MDL_API void mdl_decode_spec_layout(int v) { g_spec_layout = v; }
static bool spec_enabled() {
  if (g_spec_enable < 0) {
    const char* e = getenv("MAT_DCML_DECODE_SPEC");
    g_spec_enable = !(e && e[0] == '0');
  }
  return g_spec_enable != 0;
}
MDL_API int mdl_decode_spec_plan(const DecParams* p, int NB) {
  if (!spec_enabled() || NB != 2 || !wv_eligible(p, NB) || p->act_dim > 48) return -1;
  if (p->n_tok < p->act_dim + 1) return -1;
  const int nmm = wv_nm(NB) - 6;
  // register-resident main-wave matrices, in the order measured fastest (scripts/r5_nreg.sh, profiles/r5_spec):
  // narrow head (DCML) 0 < 8 < 2 < 6 < 4 (148.8 / 150.1 / 153.5 / 155.6 / 157.9 us at 256 x 33; 8 also beats the
  // token-table layout at 256 x 101, 530.6 vs 541 us); wide head (SMAC) 6 < 4 (134.1 / 139.8 us).
  // MAT_DCML_SPEC_NREG=k forces k when it fits.
  static const int force = [] { const char* e = getenv("MAT_DCML_SPEC_NREG"); return e ? atoi(e) : -1; }();
  static const int narrow[] = {0, 8, 2, 6, 4}, wide[] = {6, 4, 2, 0};
  const bool nar = p->act_dim <= 4;
  const int* order = nar ? narrow : wide;
  const int norder = nar ? 5 : 4;
  for (int j = -1; j < norder && g_spec_layout == 0; ++j) {
    const int nreg = j < 0 ? force : order[j];
    if (nreg < 0 || nreg > (nar ? 8 : 6) || (nreg & 1)) continue;
    if (sp_lds(NB, p->L, p->n_tok, nmm - nreg, p->act_dim, false).total <= 160 * 1024) return nreg;
  }
  // long rows (A <= 4): block 0's self K / V through the token table (+ 16 marks the IND layout), then without the
  // query table as well (+ 32: Q2F)
  if (p->act_dim <= 4) {
    for (int nreg = 4; nreg <= 6 && g_spec_layout <= 1; nreg += 2)
      if (sp_lds(NB, p->L, p->n_tok, nmm - nreg, p->act_dim, true).total <= 160 * 1024) return 16 + nreg;
    if (sp_lds(NB, p->L, p->n_tok, nmm - 6, p->act_dim, true, true).total <= 160 * 1024) return 32 + 16 + 6;
  }
  return -1;
}
static int mdl_decode_spec(const DecParams* p, int NB, hipStream_t st) {
  int nreg = mdl_decode_spec_plan(p, NB);
  if (nreg < 0) return 1;
  const bool ind = nreg & 16, q2f = nreg & 32;
  nreg &= 15;
  const int A = p->act_dim, NS = (A + 15) / 16;
  const size_t lds = (size_t)sp_lds(NB, p->L, p->n_tok, wv_nm(NB) - 6 - nreg, A, ind, q2f).total;
  if (q2f) return sp_launch<2, 1, 6, 1, true, true>(p, lds, st);
  if (ind) return nreg == 4 ? sp_launch<2, 1, 4, 1, true>(p, lds, st) : sp_launch<2, 1, 6, 1, true>(p, lds, st);
  if (A <= 4) return sp_launch_nreg<1, 1>(p, nreg, lds, st);
  if (NS == 1) return sp_launch_nreg<1, 3>(p, nreg, lds, st);
  if (NS == 2) return sp_launch_nreg<2, 3>(p, nreg, lds, st);
  return sp_launch_nreg<3, 3>(p, nreg, lds, st);
}

int mdl_decode_wave(const DecParams* p, int NB, hipStream_t st) {
  if (p->B > 0) {
    const int r = mdl_decode_spec(p, NB, st);
    if (r <= 0) return r;
  }
  const int nreg = mdl_decode_wave_plan(p, NB);
  if (nreg < 0) return 1;
  if (p->B <= 0) return 0;
  const bool wide = p->act_dim > 4;
  const size_t lds = (size_t)wv_lds(NB, p->L, p->n_tok, wv_nm(NB) - nreg, wide).total;
  if (NB == 1) {
    if (nreg == 0) return wv_launch<1, 0>(p, wide, lds, st);
    if (nreg == 2) return wv_launch<1, 2>(p, wide, lds, st);
    return wv_launch<1, 4>(p, wide, lds, st);
  }
  if (nreg == 0) return wv_launch<2, 0>(p, wide, lds, st);
  if (nreg == 2) return wv_launch<2, 2>(p, wide, lds, st);
  if (nreg == 4) return wv_launch<2, 4>(p, wide, lds, st);
  return wv_launch<2, 6>(p, wide, lds, st);
}
