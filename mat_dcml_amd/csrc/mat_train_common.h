// Shared pieces of the fused MAT training kernels (mat_train_ct.h, mat_enc_ct.hip, mat_dec_ct.hip): the kernel
// argument structs, the per-tile context, the sequence-block-diagonal MFMA score chunk, and the persistent tiling.
//
// Replaces the eager forward/backward of the reference's Encoder / Decoder (mat_src/mat/algorithms/mat/algorithm/
// ma_transformer.py:72-230) used by TransformerPolicy.evaluate_actions / get_values (transformer_policy.py:158-217)
// inside MATTrainer.ppo_update (mat_trainer.py:96-156).
//
// One workgroup owns SQ whole sequences at a time (NR = SQ*L token rows, NT 16-row MFMA tiles; wave w owns tiles
// w, w + NW, ...).  Weight gradients dW = dYᵀ·X reduce over the token axis from token-major LDS tiles
// (ds_read_b64_tr_b16 transposed reads).
#pragma once
#include "tile.h"
#include <cstdlib>

using namespace mdl;

__host__ __device__ inline size_t mat_train_lds_main_bytes(int NRP) {
  const size_t aux = (size_t)NRP * 2 * 4 * 2;   // LSE / delta [2][NRP] f32 (also the decoder's embedding-grad scratch)
  return (size_t)NRP * 64 * 2 * 6 + (aux < 9 * 64 * 4 ? 9 * 64 * 4 : aux);
}
// Behind the token buffers (NRP <= 192: 150.5 KB + 12.2 KB + 16 B < 160 KB):
//  * the per-workgroup parameter-vector accumulators (VSLOTS x 64, int64 fixed point) and their global destinations
//    (VSLOTS pointers): LayerNorm / bias / log-std gradient partials are summed here with LDS atomics across ALL of
//    the workgroup's chunks and leave once, at the end of the launch.  A global atomic sits in the issuing wave's
//    in-order vmcnt queue for ~3,000 cycles under load, so one flushed per LayerNorm made the next phase's
//    saved-activation loads wait for it (~16 such stalls per chunk).
//    Round 6: the partials are added as 2^-32 fixed-point int64 (ds_add_u64): integer addition is associative, so the
//    sum no longer depends on the order in which the 8 waves reach their LDS atomics — the workgroup's vector
//    gradients are bit-reproducible (fp32 LDS atomics were not).  A partial of magnitude >= 2^24 (or non-finite)
//    raises the workgroup's overflow flag, and the flush then writes NaN: the optimizer skips such a step, exactly
//    as it skips any non-finite gradient.
constexpr int VSLOTS = 24;
constexpr float VFX_SCALE = 4294967296.f;        // 2^32
constexpr float VFX_INV = 1.f / 4294967296.f;
constexpr float VFX_MAX = 16777216.f;            // 2^24: larger partials -> overflow flag (<= 2^7 adds per slot
                                                 // element stay below 2^63)
__host__ __device__ inline size_t mat_train_lds_bytes(int NRP, int SQ, int L) {
  return mat_train_lds_main_bytes(NRP) + (size_t)VSLOTS * (64 * 8 + 8 + 4) + 16;
}

namespace {

#ifndef MDL_MAXRT
#define MDL_MAXRT 3
#endif
#ifndef MDL_NW
#define MDL_NW 4     // waves per workgroup (the round-2 backward translation units build with 8)
#endif
constexpr int NW = MDL_NW;
constexpr int NTHR = 64 * NW;
constexpr int MAXRT = MDL_MAXRT;  // row tiles per wave (NT <= NW * MAXRT; wave w owns tiles w, w + NW, ...)
constexpr int WGPC = 1;           // resident backward workgroups per CU (the forward kernels: FWD_WGPC)
constexpr int LDS_BUDGET = 160 * 1024 / WGPC;

// fw: B fragments of W (the rollout decode's row layout); bw: unused (null); fa / ba: A fragments of W / Wᵀ with the permuted k order of
// the token-on-lane tiles (mat_train_ct.h)
struct Mat { const bf16_t* fw; const bf16_t* bw; const float* b; float* dW; float* db; const bf16_t* fa; const bf16_t* ba; };
struct LNp { const float* g; const float* b; float* dg; float* db; };
struct Blk { Mat m[10]; LNp ln[3]; };
// saved activations of one block; a1lo / a2lo = the bf16 residual O - bf16(O) of the attention outputs, so the
// backward's delta = rowsum(dO O) sees O to ~16 significant bits (bf16 O alone put 10-40 % errors on dK / dQ);
// g / gp = the MLP's GELU(h) (the exact bf16 operand the forward fed to W2) and GELU'(h): the backward evaluates
// no erf for the MLP (round 3 recomputed GELU and GELU' from h: two erf per element)
// xh[k] / rs = x-hat (bf16) and rstd (f32, [3][tok], slot k) of the block's k-th LayerNorm as the forward computed
// them: the backward's LayerNorm passes read them instead of recomputing the producing linear + LayerNorm forward
// (round 4: no weight fragments, bias / residual loads or LN statistics in those passes)
struct Sv { bf16_t* xin; bf16_t* a1; float* lse1; bf16_t* x1; bf16_t* a2; float* lse2; bf16_t* x2; bf16_t* g;
            bf16_t* a1lo; bf16_t* a2lo; bf16_t* gp; bf16_t* xh[3]; float* rs; };
// the same for a GELU -> LayerNorm stage outside the blocks (value / action head, observation embedding): x-hat,
// GELU'(pre-activation) (bf16) and rstd ([tok] f32); null = not saved (rollout passes)
struct HSv { bf16_t* xh; bf16_t* gp; float* rs; };

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
  HSv hs, es;                    // value head, observation embedding (round 4)
  int g_mode;                    // 1: one PRIVATE workspace copy per workgroup, plain stores (GradMode below)
  const long long* sidx;         // minibatch sequence -> rollout-buffer sequence of `obs` (null: obs is dense)
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
  HSv hs;                // action head (round 4)
  int g_mode;            // 1: one PRIVATE workspace copy per workgroup, plain stores (GradMode below)
  const long long* sidx; // minibatch sequence -> rollout-buffer sequence of `act` / `ava` (null: dense)
};

// Round 6: the training kernels read the minibatch's INPUTS (observations, stored actions, availability) straight
// from the rollout buffer through the epoch permutation (sidx), so no gather copy precedes them; token tok of the
// dense minibatch order (outputs, saved activations, loss gradients) reads input row src_tok(tok).
#ifndef MDL_NO_SIDX
#define MDL_NO_SIDX 0   // A/B: compile the sequence index out (dense inputs only)
#endif
__device__ __forceinline__ size_t src_tok(const long long* sidx, size_t tok, int L) {
  if (MDL_NO_SIDX || !sidx) return tok;
  const int t = (int)tok, s = t / L;   // a minibatch has < 2^31 tokens: 32-bit division (64-bit is emulated)
  return (size_t)sidx[s] * (size_t)L + (size_t)(t - s * L);
}

// Weight-gradient flush modes (round 6).  ATOMIC (rounds 2-5): fp32 atomics into a workspace copy shared by
// g_copies / G workgroups — the memory-side atomic unit (~1.35 TB/s chip-wide) made them cost ~121 us per
// minibatch, and their order made every run's gradient differ in the last bits.  PRIVATE: the gradient workspace
// has ONE copy per workgroup of the launch; a workgroup's first chunk STORES its partial gradients, its later chunks
// load + add + store their own earlier values (the loads issued before the weight-gradient MFMA loop, so their
// latency hides under it).  No atomics, no cross-workgroup races, a fixed summation order: the gradient is
// bit-reproducible, and csrc/ppo.hip:grad_reduce_priv folds the copies in copy order.  The 64 x 64 weight
// gradients sit in the copies in the MFMA fragment order (each lane stores its two f32x4 accumulators as 16-byte
// pieces: 1 KB per wave-instruction pair) and the reduction maps them back to row-major.
// Micro-benchmark (tests/native/wgrad_flush_bench.hip, 256 workgroups x 8 waves x 22 matrices x 3 chunks):
// atomics 207 us + 6 us reduction, private copies 73 us + 17 us.
struct GradMode { bool priv, first; };
#ifndef MDL_NO_PRIV
#define MDL_NO_PRIV 0   // A/B: compile the private-copy flush paths out (shared-copy atomics only)
#endif
#ifndef MDL_VACC_F32
#define MDL_VACC_F32 0  // A/B: fp32 LDS atomics for the vector accumulators (order-dependent; rounds 2-5)
#endif

struct Ctx {
  int tid, lane, wave, L, nseq, NR, NT, NRP, KP, tok0;   // KP: rows [0, KP) = NR rounded up to 32 (<= NRP)
  ptrdiff_t gofs;   // gradient-copy offset (floats): this block's copy of the dW workspace, 0 = direct
  GradMode gm;      // flush mode of this chunk (private copies: first chunk of the workgroup stores)
  __device__ __forceinline__ float* g(float* p) const { return p ? p + gofs : p; }
  bf16_t *QB, *KB, *VB, *DA, *DQ, *XB;
  float *LSE, *DEL;
  unsigned long long* VACC;  // [VSLOTS][64] parameter-vector gradient accumulators (LDS, 2^-32 fixed point)
  float** VPT;               // [VSLOTS] their global destinations (null = unused slot)
  int* VLEN;                 // [VSLOTS] 1 + the largest element index added (the flush writes no further)
  int* VOVF;                 // overflow / non-finite flag of the accumulators
};

constexpr float ATT_SCALE = 0.17677669529663687f;  // 1/sqrt(32)

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

// saved per-row log-sum-exp ([tok][2] global) -> LDS [head][NRP]
__device__ __forceinline__ void load_lse(const float* sv_lse, const Ctx& c) {
  for (int i = c.tid; i < 2 * c.NRP; i += NTHR) {
    const int h = i / c.NRP, row = i - h * c.NRP;
    c.LSE[i] = row < c.NR ? sv_lse[(size_t)(c.tok0 + row) * 2 + h] : 0.f;
  }
}

// the same in two halves: issue the global loads early (lse_fetch, registers), store them to LDS later (lse_store),
// so the load latency hides under the work in between instead of stalling right before a barrier
struct LseR { float v[2]; };
__device__ __forceinline__ LseR lse_fetch(const float* sv_lse, const Ctx& c) {
  LseR r;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = c.tid + j * NTHR;
    const int h = i / c.NRP, row = i - h * c.NRP;
    r.v[j] = (i < 2 * c.NRP && row < c.NR) ? sv_lse[(size_t)(c.tok0 + row) * 2 + h] : 0.f;
  }
  return r;
}
__device__ __forceinline__ void lse_store(const LseR& r, const Ctx& c) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = c.tid + j * NTHR;
    if (i < 2 * c.NRP) c.LSE[i] = r.v[j];
  }
}

// Backward tile start: zero only what no phase rewrites before reading — the rows [NR, KP) past the chunk's
// tokens in the six token-major buffers and in delta (a shorter chunk after a longer one would otherwise see the
// previous chunk's rows there: the tail of its last 16-row tile and the 32-row key chunks read past it).  Rows
// below NR are always written before they are read; LSE is fully rewritten per attention; nothing reads a row at
// or past KP (32-row key chunks and the weight-gradient K loop stop there).  (Round 2 zeroed all ~150 KB per tile.)
__device__ __forceinline__ void zero_pad_rows(const Ctx& c) {
  const int r0 = c.NR, nr = c.KP - r0;
  if (nr <= 0) return;
  bf16_t* bufs[6] = {c.QB, c.KB, c.VB, c.DA, c.DQ, c.XB};
  const int per = nr * 8;   // 16-byte pieces per buffer
  for (int i = c.tid; i < 6 * per; i += NTHR) {
    const int b = i / per, o = i - b * per;
    *(uint4*)(bufs[b] + (size_t)r0 * 64 + (size_t)o * 8) = make_uint4(0, 0, 0, 0);
  }
  for (int i = c.tid; i < 2 * nr; i += NTHR) c.DEL[(i / nr) * c.NRP + r0 + (i % nr)] = 0.f;
}

// Forward tile start: the forward kernels keep only Q / K / V in LDS; rows below NR are rewritten by every
// projection pass (padded rows of the last 16-row tile as zeros) and nothing reads a row at or past KP, so only the
// rows [NT*16, KP) that no pass writes need zeros (round 3 zeroed all ~74 KB per tile: 4-7 % of the forwards)
__device__ __forceinline__ void zero_pad_rows_fwd(const Ctx& c) {
  const int r0 = c.NT * 16 < c.KP ? c.NT * 16 : c.KP, nr = c.KP - r0;
  if (nr <= 0) return;
  bf16_t* bufs[3] = {c.QB, c.KB, c.VB};
  const int per = nr * 8;   // 16-byte pieces per buffer
  for (int i = c.tid; i < 3 * per; i += NTHR) {
    const int b = i / per, o = i - b * per;
    *(uint4*)(bufs[b] + (size_t)r0 * 64 + (size_t)o * 8) = make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void zero_lds(char* smem, size_t bytes, int tid) {
  for (size_t i = (size_t)tid * 16; i < bytes; i += NTHR * 16) *(uint4*)(smem + i) = make_uint4(0, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------ context
template <typename PT>
__device__ __forceinline__ Ctx make_ctx(const PT& p, char* smem, int seq0, int nseq, bool first_chunk = true) {
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
  c.KP = min(p.NRP, (c.NR + 31) & ~31);
  c.tok0 = seq0 * p.L;
  // spread the fp32 weight-gradient atomics over g_copies copies (blockIdx % 8 ~ the XCD the block runs on):
  // 8x fewer adders per address than every workgroup hitting the same 16 KB matrix
  c.gofs = p.g_copies > 0 ? (ptrdiff_t)p.g_delta + (ptrdiff_t)(blockIdx.x % p.g_copies) * (ptrdiff_t)p.g_stride : 0;
  c.gm.priv = !MDL_NO_PRIV && p.g_copies > 0 && p.g_mode == 1;   // private mode: the host sized g_copies >= grid
  c.gm.first = first_chunk;
  const size_t bs = (size_t)p.NRP * 64;
  bf16_t* base = (bf16_t*)smem;
  c.QB = base; c.KB = base + bs; c.VB = base + 2 * bs; c.DA = base + 3 * bs; c.DQ = base + 4 * bs; c.XB = base + 5 * bs;
  c.LSE = (float*)(base + 6 * bs);
  c.DEL = c.LSE + 2 * p.NRP;
  c.VACC = (unsigned long long*)(smem + mat_train_lds_main_bytes(p.NRP));
  c.VPT = (float**)(c.VACC + VSLOTS * 64);
  c.VLEN = (int*)(c.VPT + VSLOTS);
  c.VOVF = c.VLEN + VSLOTS;
  return c;
}

// parameter-vector accumulators: zeroed before a workgroup's first chunk, flushed after its last (backward kernels)
template <typename PT>
__device__ __forceinline__ void vacc_begin(const PT& p, char* smem) {
  unsigned long long* V = (unsigned long long*)(smem + mat_train_lds_main_bytes(p.NRP));
  float** P = (float**)(V + VSLOTS * 64);
  int* N = (int*)(P + VSLOTS);   // VLEN [VSLOTS], then the overflow flag
  for (int i = threadIdx.x; i < VSLOTS * 64; i += NTHR) V[i] = 0ull;
  for (int i = threadIdx.x; i < VSLOTS; i += NTHR) {
    P[i] = nullptr;
    N[i] = 0;
  }
  if (threadIdx.x == 0) N[VSLOTS] = 0;
  __syncthreads();
}
// private mode: every element [0, VLEN) of a used slot is STORED (its workgroup's copy holds nothing else there:
// zeros included, so a stale value of an earlier launch never survives) and nothing past it — a slot shorter than 64
// (log_std, value-head bias, LN_obs) must not touch the neighbouring parameters' entries; shared copies: fp32 atomics
template <typename PT>
__device__ __forceinline__ void vacc_end(const PT& p, char* smem) {
  __syncthreads();
  const unsigned long long* V = (const unsigned long long*)(smem + mat_train_lds_main_bytes(p.NRP));
  float* const* P = (float* const*)(V + VSLOTS * 64);
  const int* N = (const int*)(P + VSLOTS);
  const bool bad = N[VSLOTS] != 0;
  const bool priv = p.g_copies > 0 && p.g_mode == 1;
  for (int i = threadIdx.x; i < VSLOTS * 64; i += NTHR) {
    float* d = P[i >> 6];
    if (!d || (i & 63) >= N[i >> 6]) continue;
    const float v = MDL_VACC_F32 ? *reinterpret_cast<const float*>(V + i)
                                 : bad ? __builtin_nanf("") : (float)(long long)V[i] * VFX_INV;
    if (priv) d[i & 63] = v;
    else if (v != 0.f) atomicAdd(d + (i & 63), v);
  }
}
// add v to element idx (< len <= 64) of the parameter-vector gradient dst (already offset to this block's gradient
// copy); len = the parameter's length (the flush writes [0, len) of the slot).  Every writer of a slot stores the same
// pointer and length (plain LDS stores: an LDS atomic-max from 64 lanes onto one address serialised 64-fold).
#ifndef MDL_VACC_NOCHECK
#define MDL_VACC_NOCHECK 0   // A/B: no overflow / non-finite check on the fixed-point partials
#endif
__device__ __forceinline__ void vacc_add(float* dst, int slot, int idx, float v, const Ctx& c, int len = 64) {
  if (!dst) return;
  if constexpr (MDL_VACC_F32) {
    atomicAdd(reinterpret_cast<float*>(c.VACC + slot * 64 + idx), v);
  } else {
    const float s = v * VFX_SCALE;
    const bool in = fabsf(s) < VFX_MAX * VFX_SCALE;   // false for NaN / inf too
    if (!MDL_VACC_NOCHECK && !in) *c.VOVF = 1;
    const long long q = (MDL_VACC_NOCHECK || in) ? (long long)__builtin_rintf(s) : 0ll;
    atomicAdd(c.VACC + slot * 64 + idx, (unsigned long long)q);   // LDS integer atomic (ds_add_u64): order-free
  }
  c.VLEN[slot] = len;
  c.VPT[slot] = dst;
}

}  // namespace



// Persistent tiling: workgroup w owns the contiguous sequence range [Bs*w/G, Bs*(w+1)/G) and walks it in chunks of
// <= SQ sequences.  With G = #CUs the makespan is ceil(Bs/G) sequences per CU instead of ceil(Bs/SQ/G) full tiles
// (640 tiles of 5 on 256 CUs = 3 rounds of 5 -> 13 sequences per CU).
//
// Chunk plan: the token-parallel phases run in rounds of NW 16-row tiles (wave w owns tiles w, w + NW, ...), so a
// chunk costs ceil(NT / NW) rounds plus a fixed per-chunk part (weight-fragment loads, barriers, the per-chunk
// gradient flushes), MDL_CHUNK_A4 / 4 rounds.  Of: near-equal chunks (fewest chunks), full SQ chunks + a remainder,
// and near-equal chunks with one more chunk, the cheapest is taken.  L = 33 in the 8-wave backward: 13 sequences
// were (4, 4, 5) = 9 + 9 + 11 tiles = 6 rounds; (5, 5, 3) = 11 + 11 + 7 tiles = 5 rounds.
#ifndef MDL_CHUNK_A4
#define MDL_CHUNK_A4 8
#endif
__device__ __forceinline__ int chunk_rounds(int s, int L) {
  const int nt = (s * L + 15) >> 4;
  return (nt + NW - 1) / NW;
}
// > 0: that many near-equal chunks; < 0: -(number of chunks) of SQ sequences each but the last
__device__ __forceinline__ int chunk_plan(int n, int SQ, int L) {
  if (n <= 0) return 0;
  const int n0 = (n + SQ - 1) / SQ;
  auto bal = [&](int k) {
    const int q = n / k, r = n - q * k;
    return 4 * (r * chunk_rounds(q + 1, L) + (k - r) * chunk_rounds(q, L)) + MDL_CHUNK_A4 * k;
  };
  int best = n0, cost = bal(n0);
  const int cg = 4 * ((n0 - 1) * chunk_rounds(SQ, L) + chunk_rounds(n - (n0 - 1) * SQ, L)) + MDL_CHUNK_A4 * n0;
  if (cg < cost) { best = -n0; cost = cg; }
  if (n0 + 1 <= n && bal(n0 + 1) < cost) best = n0 + 1;
  return best;
}
// Every other group of 8 workgroups (one per XCD) walks its chunks in reverse order (MDL_STAGGER=1): with unequal chunks (L = 33: 5, 5, 3
// sequences) half the workgroups of every XCD are then out of phase with the other half, so their weight-gradient atomic bursts
// (the memory-side atomic unit's 1.3 TB/s is chip-wide) interleave instead of coinciding.
// Measured in the bench (profiles/r5_ab): dec_bwd 457.6 -> 428.5 us, enc_bwd 305.1 -> 274.3 us per minibatch; the
// forwards (no atomics) measured +2 us with it, so only the backward translation units default to it.
// MDL_STAGGER=2 (A/B): three groups — the third walks (0, 2, 1) — measured the same as 1.
#ifndef MDL_STAGGER
#ifdef MDL_CT_BWD_TU
#define MDL_STAGGER 1
#else
#define MDL_STAGGER 0
#endif
#endif
__device__ __forceinline__ int stagger_chunk(int it, int nch, int grp) {
  if (MDL_STAGGER == 0 || nch < 2) return it;
  if (MDL_STAGGER == 1) return (grp & 1) ? nch - 1 - it : it;
  const int k = grp % 3;
  if (k == 0) return it;
  if (k == 1) return nch - 1 - it;
  return it == 0 ? 0 : nch - it;   // (0, nch - 1, ..., 1)
}
#define FOR_TILES(p, CALL)                                                                         \
  {                                                                                                \
    const long long G_ = gridDim.x, w_ = blockIdx.x;                                               \
    const int lo_ = (int)((long long)(p).Bs * w_ / G_), hi_ = (int)((long long)(p).Bs * (w_ + 1) / G_); \
    const int n_ = hi_ - lo_, plan_ = chunk_plan(n_, (p).SQ, (p).L);                               \
    const int nch_ = plan_ < 0 ? -plan_ : plan_;                                                   \
    for (int it_ = 0; it_ < nch_; ++it_) {                                                         \
      const int ch_ = stagger_chunk(it_, nch_, (int)(w_ >> 3));                                       \
      int s0, ns;                                                                                  \
      if (plan_ < 0) {                                                                             \
        s0 = lo_ + ch_ * (p).SQ;                                                                   \
        ns = min((p).SQ, n_ - ch_ * (p).SQ);                                                       \
      } else {                                                                                     \
        s0 = lo_ + (int)((long long)n_ * ch_ / nch_);                                              \
        ns = lo_ + (int)((long long)n_ * (ch_ + 1) / nch_) - s0;                                   \
      }                                                                                            \
      if (it_) __syncthreads();                                                                    \
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
