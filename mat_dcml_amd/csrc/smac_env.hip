// SMAC-shaped synthetic battle env (BASELINE config #5, envs/smac/synthetic.py) as ONE launch per env step.
//
// One 1024-thread workgroup per env.  Wave 0 runs the step dynamics over the env's units (lane = ally i for the
// ally phases, lane = enemy j for the enemy phases; state staged in LDS): moves, ally attacks, nearest-ally enemy
// behaviour, battle end, reward, per-agent dones, battle counters, the auto-reset of a finished battle (Philox
// draws keyed by (episode counter, global env id, unit, purpose): draw-for-draw identical to the torch path) and
// the per-episode agent permutation (Random_StarCraft2_Env.py:386-389).  Then all 16 waves write the observation
// (A x obs_dim), per-agent state (A x state_dim) and availability (A x n_actions) rows, one coalesced element per
// thread per iteration.  The torch env issued ~150 elementwise launches per step for the same work.
//
// Semantics (the reference env's contract, StarCraft2_Env.py:474-653, get_obs_agent :1559-1660,
// get_state_agent :1662-1740, get_avail_agent_actions): dead units take no-op only; enemies walk to / shoot the
// nearest living ally; reward = (damage dealt + 10 / kill + 200 on a win) / (max_reward / 20), positive only.
// Rounding: every product / sum the torch path rounds separately is rounded separately here (__fmul_rn etc.,
// no FMA contraction); distances are sqrt(dx*dx + dy*dy) in that order on both paths.
#include "common.h"

using namespace mdl;

namespace {

constexpr int SM_MAXU = 64;          // allies and enemies per env (largest registered map: 2c_vs_64zg, 64 enemies)
constexpr int SM_THREADS = 1024;
constexpr uint32_t P_SMAC = 32;      // Philox purpose of the battle reset draws (utils/philox.py P_SMAC)
constexpr float INV_SIGHT = (float)(1.0 / 9.0);   // x / SIGHT as torch computes it: x * fl(1/9)
constexpr float MAP = 32.f, SIGHT = 9.f, SHOOT = 6.f, MOVE = 1.f, EMOVE = 0.6f, ADMG = 0.15f, EDMG = 0.06f;

struct SmacCfg {
  int E, A, N, nA, u, limit, obs_dim, state_dim, rao, mode;   // mode 0: step, 1: reset every env
  uint32_t k0, k1;
  float inv_reward_scale;   // fl(1 / reward_scale): reward = rw * it, as the torch path
};

struct SmacState {
  const int64_t* gid;     // (E) global env id
  int64_t* ep_ctr;        // (E) battles started (reset draw counter)
  float* apos;            // (E, A, 2)
  float* ahp;             // (E, A)
  float* epos;            // (E, N, 2)
  float* ehp;             // (E, N)
  int64_t* t;             // (E)
  int64_t* last;          // (E, A) last action per agent (agent order)
  float* battles_won;     // (E)
  float* battles_game;    // (E)
  int64_t* perm;          // (E, A) output row j = agent perm[j]
};

struct SmacOut {
  const float* actions;   // (E, A) policy rows (row j acts for agent perm[j])
  float* obs;             // (E, A, obs_dim)
  float* state;           // (E, A, state_dim)
  float* ava;             // (E, A, nA)
  float* reward;          // (E)
  bool* dones;            // (E, A) in the PRE-reset row order
  bool* won; bool* lost; bool* timeout;   // (E)
  float* dead_allies; float* dead_enemies;   // (E)
  float* battles_won_out; float* battles_game_out;   // (E) copies of the counters after this step
};

__device__ __forceinline__ float dist2(float ax, float ay, float bx, float by, float& dx, float& dy) {
  dx = __fsub_rn(bx, ax);
  dy = __fsub_rn(by, ay);
  return (float)__dsqrt_rn((double)__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));   // as the torch path
}

__device__ __forceinline__ float sq2(float ax, float ay, float bx, float by) {   // squared distance, torch order
  const float dx = __fsub_rn(bx, ax), dy = __fsub_rn(by, ay);
  return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
}
constexpr float SHOOT2 = 36.f, SIGHT2 = 81.f;

__device__ __forceinline__ float u01f(uint32_t u) { return (float)u01_open(u); }

__device__ __forceinline__ float dir_x(int k) { return k == 2 ? 1.f : (k == 3 ? -1.f : 0.f); }   // N, S, E, W
__device__ __forceinline__ float dir_y(int k) { return k == 0 ? 1.f : (k == 1 ? -1.f : 0.f); }

// grid (E, P): the P workgroups of env e each run the (cheap, deterministic) step on their own LDS copy of the env
// and build 1/P of its observation / state / availability rows (SMAC 27m_vs_30m: 27 x (1288 + 1458 + 36) values per
// env — one workgroup per env left 224 of 256 CUs idle at 32 envs: 81 us per step).  The state is read from `s` and
// written, by workgroup 0 of each env only, to the other copy `so` (ping-pong, swapped by the host), so no
// workgroup can see a half-updated env.
__global__ __launch_bounds__(SM_THREADS) void smac_env_kernel(SmacCfg c, SmacState s, SmacState so, SmacOut o) {
  __shared__ float ax[SM_MAXU], ay[SM_MAXU], ah[SM_MAXU], ex[SM_MAXU], ey[SM_MAXU], eh[SM_MAXU];
  __shared__ int nhit[SM_MAXU], ahit[SM_MAXU];   // hit counts: damage = count x per-hit damage, one rounding
  __shared__ float dealt[SM_MAXU];
  __shared__ int act[SM_MAXU], lst[SM_MAXU], prm[SM_MAXU];
  __shared__ uint32_t keys[SM_MAXU];
  __shared__ int s_reset;
  const int e = blockIdx.x, tid = threadIdx.x, A = c.A, N = c.N;
  const int part = blockIdx.y, P = gridDim.y;
  const bool lead = part == 0;   // writes the state and the per-env outputs
  __shared__ long long s_t, s_ctr;
  const uint32_t g = (uint32_t)s.gid[e];
  if (tid < A) {
    ax[tid] = s.apos[((size_t)e * A + tid) * 2];
    ay[tid] = s.apos[((size_t)e * A + tid) * 2 + 1];
    ah[tid] = s.ahp[(size_t)e * A + tid];
    lst[tid] = (int)s.last[(size_t)e * A + tid];
    prm[tid] = (int)s.perm[(size_t)e * A + tid];
  }
  if (tid < N) {
    ex[tid] = s.epos[((size_t)e * N + tid) * 2];
    ey[tid] = s.epos[((size_t)e * N + tid) * 2 + 1];
    eh[tid] = s.ehp[(size_t)e * N + tid];
  }
  if (tid < SM_MAXU) { nhit[tid] = 0; ahit[tid] = 0; dealt[tid] = 0.f; }
  if (tid == 0) {
    s_reset = c.mode == 1;
    s_t = s.t[e];
    s_ctr = s.ep_ctr[e];
  }
  __syncthreads();
  if (c.mode == 0) {
    // ---- actions of the policy rows -> agents; dead agents no-op
    if (tid < A) {
      const int agent = c.rao ? prm[tid] : tid;
      int a = (int)o.actions[(size_t)e * A + tid];
      act[agent] = a;
    }
    __syncthreads();
    if (tid < A) {
      const bool alive = ah[tid] > 0.f;
      const int a = alive ? act[tid] : 0;
      act[tid] = a;
      if (a >= 2 && a < 6) {   // move, clamped to the map
        ax[tid] = fminf(fmaxf(__fadd_rn(ax[tid], dir_x(a - 2) * MOVE), 0.f), MAP);
        ay[tid] = fminf(fmaxf(__fadd_rn(ay[tid], dir_y(a - 2) * MOVE), 0.f), MAP);
      }
    }
    __syncthreads();
    // ---- ally attacks (new ally positions, enemy hp before this step's damage)
    if (tid < A) {
      const int a = act[tid];
      if (a >= 6 && ah[tid] > 0.f) {
        const int tg = min(max(a - 6, 0), N - 1);
        if (sq2(ax[tid], ay[tid], ex[tg], ey[tg]) <= SHOOT2 && eh[tg] > 0.f) atomicAdd(&nhit[tg], 1);
      }
    }
    __syncthreads();
    // ---- enemies: damage, then the nearest living ally (allies alive before the enemy fire)
    if (tid < N) {
      const float old = eh[tid];
      const float nh = fmaxf(__fsub_rn(old, __fmul_rn((float)nhit[tid], ADMG)), 0.f);
      eh[tid] = nh;
      dealt[tid] = __fsub_rn(old, nh);
      if (nh > 0.f) {
        float best = INFINITY;
        int near = 0;
        for (int i = 0; i < A; ++i) {
          if (!(ah[i] > 0.f)) continue;
          const float d = sq2(ax[i], ay[i], ex[tid], ey[tid]);   // squared: no square root in the dynamics
          if (d < best) { best = d; near = i; }
        }
        if (best <= SHOOT2) {
          atomicAdd(&ahit[near], 1);
        } else if (best < INFINITY) {
          float vx, vy;
          float nrm = dist2(ex[tid], ey[tid], ax[near], ay[near], vx, vy);
          nrm = fmaxf(nrm, 1e-6f);
          ex[tid] = __fadd_rn(ex[tid], __fmul_rn(__fdiv_rn(vx, nrm), EMOVE));
          ey[tid] = __fadd_rn(ey[tid], __fmul_rn(__fdiv_rn(vy, nrm), EMOVE));
        }
      }
    }
    __syncthreads();
    if (tid < A) {
      ah[tid] = fmaxf(__fsub_rn(ah[tid], __fmul_rn((float)ahit[tid], EDMG)), 0.f);
      lst[tid] = act[tid];
    }
    __syncthreads();
    // ---- battle end, reward, dones, counters (thread 0, fixed order)
    if (tid == 0) {
      int e_alive = 0, a_alive = 0, kills = 0;
      float sum_dealt = 0.f;
      for (int j = 0; j < N; ++j) {
        e_alive += eh[j] > 0.f;
        kills += (dealt[j] > 0.f) && !(eh[j] > 0.f);
        sum_dealt = __fadd_rn(sum_dealt, dealt[j]);
      }
      for (int i = 0; i < A; ++i) a_alive += ah[i] > 0.f;
      const long long t = s_t + 1;
      const bool won = e_alive == 0;
      const bool lost = a_alive == 0 && !won;
      const bool tout = t >= c.limit && !won && !lost;
      const bool done = won || lost || tout;
      const float rw = __fadd_rn(__fadd_rn(sum_dealt, __fmul_rn(10.f, (float)kills)), won ? 200.f : 0.f);
      const float bg = s.battles_game[e] + (done ? 1.f : 0.f), bw = s.battles_won[e] + (won ? 1.f : 0.f);
      if (lead) {
        o.reward[e] = __fmul_rn(rw, c.inv_reward_scale);
        o.won[e] = won;
        o.lost[e] = lost;
        o.timeout[e] = tout;
        o.dead_allies[e] = (float)(A - a_alive);
        o.dead_enemies[e] = (float)(N - e_alive);
        so.battles_game[e] = bg;
        so.battles_won[e] = bw;
        o.battles_game_out[e] = bg;
        o.battles_won_out[e] = bw;
      }
      s_t = t;
      s_reset = done;
    }
    __syncthreads();
    if (lead && tid < A) o.dones[(size_t)e * A + tid] = s_reset || !(ah[c.rao ? prm[tid] : tid] > 0.f);
  } else if (lead && tid == 0) {   // reset of every env: the counters carry over
    so.battles_game[e] = s.battles_game[e];
    so.battles_won[e] = s.battles_won[e];
  }
  // ---- battle reset (new unit positions, full hp, fresh agent order)
  if (s_reset) {
    const uint32_t ctr = (uint32_t)s_ctr;
    if (tid < A) {
      const u4 r = philox4x32_10(ctr, g, (uint32_t)tid, P_SMAC, c.k0, c.k1);
      ax[tid] = __fadd_rn(8.f, __fmul_rn(3.f, u01f(r.x)));
      ay[tid] = __fadd_rn(16.f, __fmul_rn(6.f, __fsub_rn(u01f(r.y), 0.5f)));
      ah[tid] = 1.f;
      lst[tid] = 0;
      keys[tid] = r.z;
    }
    if (tid < N) {
      const u4 r = philox4x32_10(ctr, g, 64u + (uint32_t)tid, P_SMAC, c.k0, c.k1);
      ex[tid] = __fadd_rn(22.f, __fmul_rn(3.f, u01f(r.x)));
      ey[tid] = __fadd_rn(16.f, __fmul_rn(6.f, __fsub_rn(u01f(r.y), 0.5f)));
      eh[tid] = 1.f;
    }
    __syncthreads();
    if (c.rao && tid < A) {   // stable argsort of the keys: row (rank of agent i) = i
      int rank = 0;
      for (int k = 0; k < A; ++k) rank += (keys[k] < keys[tid]) || (keys[k] == keys[tid] && k < tid);
      prm[rank] = tid;
    }
    if (tid == 0) {
      s_t = 0;
      s_ctr = (long long)ctr + 1;
    }
  }
  __syncthreads();
  // ---- write back the state (the other copy; workgroup 0 of the env)
  if (lead) {
    if (tid < A) {
      so.apos[((size_t)e * A + tid) * 2] = ax[tid];
      so.apos[((size_t)e * A + tid) * 2 + 1] = ay[tid];
      so.ahp[(size_t)e * A + tid] = ah[tid];
      so.last[(size_t)e * A + tid] = lst[tid];
      so.perm[(size_t)e * A + tid] = prm[tid];
    }
    if (tid < N) {
      so.epos[((size_t)e * N + tid) * 2] = ex[tid];
      so.epos[((size_t)e * N + tid) * 2 + 1] = ey[tid];
      so.ehp[(size_t)e * N + tid] = eh[tid];
    }
    if (tid == 0) {
      so.t[e] = s_t;
      so.ep_ctr[e] = s_ctr;
    }
  }
  // ---- observations (StarCraft2_Env.get_obs_agent layout with the map's unit-type bits)
  const int u = c.u, nA = c.nA;
  const int EF = 5 + u, AF = 5 + u + nA, OF = 5 + u + nA;
  const int o_e = 4, o_a = o_e + N * EF, o_o = o_a + (A - 1) * AF, o_i = o_o + OF;
  for (int x = part * SM_THREADS + tid; x < A * c.obs_dim; x += P * SM_THREADS) {
    const int j = x / c.obs_dim, f = x - j * c.obs_dim;
    const int i = c.rao ? prm[j] : j;
    const float al = ah[i] > 0.f ? 1.f : 0.f;
    float v = 0.f;
    if (f < o_e) {
      const int k = f;
      const float nx = __fadd_rn(ax[i], dir_x(k) * MOVE), ny = __fadd_rn(ay[i], dir_y(k) * MOVE);
      v = (nx >= 0.f && nx <= MAP && ny >= 0.f && ny <= MAP) ? al : 0.f;
    } else if (f < o_a) {
      const int k = (f - o_e) / EF, q = f - o_e - k * EF;
      float dx, dy;
      const float d = dist2(ax[i], ay[i], ex[k], ey[k], dx, dy);
      const float d2 = sq2(ax[i], ay[i], ex[k], ey[k]);
      const float vis = (d2 <= SIGHT2 ? 1.f : 0.f) * (eh[k] > 0.f ? 1.f : 0.f) * al;
      const float fv = q == 0 ? (d2 <= SHOOT2 ? 1.f : 0.f) * vis : q == 1 ? __fmul_rn(d, INV_SIGHT)
                     : q == 2 ? __fmul_rn(dx, INV_SIGHT) : q == 3 ? __fmul_rn(dy, INV_SIGHT) : q == 4 ? eh[k] : 0.f;
      v = fv * vis;
    } else if (f < o_o) {
      const int qa = (f - o_a) / AF, q = f - o_a - qa * AF;
      const int oa = qa < i ? qa : qa + 1;
      float dx, dy;
      const float d = dist2(ax[i], ay[i], ax[oa], ay[oa], dx, dy);
      const float vis = (sq2(ax[i], ay[i], ax[oa], ay[oa]) <= SIGHT2 ? 1.f : 0.f) * (ah[oa] > 0.f ? 1.f : 0.f) * al;
      float fv;
      if (q == 0) fv = vis;
      else if (q == 1) fv = __fmul_rn(d, INV_SIGHT);
      else if (q == 2) fv = __fmul_rn(dx, INV_SIGHT);
      else if (q == 3) fv = __fmul_rn(dy, INV_SIGHT);
      else if (q == 4) fv = ah[oa];
      else if (q < 5 + u) fv = q == 5 ? 1.f : 0.f;
      else fv = (q - 5 - u) == lst[oa] ? 1.f : 0.f;
      v = fv * vis;
    } else if (f < o_i) {
      const int q = f - o_o;
      float fv;
      if (q == 0) fv = ah[i];
      else if (q == 1) fv = __fdiv_rn(ax[i], MAP);
      else if (q == 2) fv = __fdiv_rn(ay[i], MAP);
      else if (q == 3) fv = 0.f;
      else if (q == 4) fv = al;
      else if (q < 5 + u) fv = q == 5 ? 1.f : 0.f;
      else fv = (q - 5 - u) == lst[i] ? 1.f : 0.f;
      v = fv * al;
    } else {
      v = (f - o_i) == i ? 1.f : 0.f;
    }
    o.obs[(size_t)e * A * c.obs_dim + x] = v;
  }
  // ---- per-agent state (get_state_agent layout: absolute positions per entity, centre offsets for the agent)
  const int SE = 8 + u, SA = 8 + u + nA, SO = 7 + u + nA;
  const int s_e = 4, s_a = s_e + N * SE, s_o = s_a + (A - 1) * SA, s_i = s_o + SO;
  for (int x = part * SM_THREADS + tid; x < A * c.state_dim; x += P * SM_THREADS) {
    const int j = x / c.state_dim, f = x - j * c.state_dim;
    const int i = c.rao ? prm[j] : j;
    const float al = ah[i] > 0.f ? 1.f : 0.f;
    float v = 0.f;
    if (f < s_e) {
      const int k = f;
      const float nx = __fadd_rn(ax[i], dir_x(k) * MOVE), ny = __fadd_rn(ay[i], dir_y(k) * MOVE);
      v = (nx >= 0.f && nx <= MAP && ny >= 0.f && ny <= MAP) ? al : 0.f;
    } else if (f < s_a) {
      const int k = (f - s_e) / SE, q = f - s_e - k * SE;
      float dx, dy;
      const float d = dist2(ax[i], ay[i], ex[k], ey[k], dx, dy);
      const float ea = eh[k] > 0.f ? 1.f : 0.f;
      const float d2 = sq2(ax[i], ay[i], ex[k], ey[k]);
      const float vis = (d2 <= SIGHT2 ? 1.f : 0.f) * ea * al;
      v = q == 0 ? (d2 <= SHOOT2 ? 1.f : 0.f) * vis : q == 1 ? __fmul_rn(d, INV_SIGHT) : q == 2 ? __fmul_rn(dx, INV_SIGHT)
        : q == 3 ? __fmul_rn(dy, INV_SIGHT) : q == 4 ? eh[k] : q == 5 ? __fdiv_rn(ex[k], MAP)
        : q == 6 ? __fdiv_rn(ey[k], MAP) : q == 7 ? ea : 0.f;
    } else if (f < s_o) {
      const int qa = (f - s_a) / SA, q = f - s_a - qa * SA;
      const int oa = qa < i ? qa : qa + 1;
      float dx, dy;
      const float d = dist2(ax[i], ay[i], ax[oa], ay[oa], dx, dy);
      const float aa = ah[oa] > 0.f ? 1.f : 0.f;
      if (q == 0) v = (sq2(ax[i], ay[i], ax[oa], ay[oa]) <= SIGHT2 ? 1.f : 0.f) * aa * al;
      else if (q == 1) v = __fmul_rn(d, INV_SIGHT);
      else if (q == 2) v = __fmul_rn(dx, INV_SIGHT);
      else if (q == 3) v = __fmul_rn(dy, INV_SIGHT);
      else if (q == 4) v = ah[oa];
      else if (q == 5) v = __fdiv_rn(ax[oa], MAP);
      else if (q == 6) v = __fdiv_rn(ay[oa], MAP);
      else if (q == 7) v = aa;
      else if (q < 8 + u) v = q == 8 ? 1.f : 0.f;
      else v = (q - 8 - u) == lst[oa] ? 1.f : 0.f;
    } else if (f < s_i) {
      const int q = f - s_o;
      if (q == 0) v = ah[i];
      else if (q == 1) v = __fdiv_rn(ax[i], MAP);
      else if (q == 2) v = __fdiv_rn(ay[i], MAP);
      else if (q == 3) v = al;
      else if (q == 4) v = __fdiv_rn(__fsub_rn(ax[i], 0.5f * MAP), MAP);
      else if (q == 5) v = __fdiv_rn(__fsub_rn(ay[i], 0.5f * MAP), MAP);
      else if (q == 6) v = 0.f;
      else if (q < 7 + u) v = q == 7 ? 1.f : 0.f;
      else v = (q - 7 - u) == lst[i] ? 1.f : 0.f;
    } else {
      v = (f - s_i) == i ? 1.f : 0.f;
    }
    o.state[(size_t)e * A * c.state_dim + x] = v;
  }
  // ---- availability (get_avail_agent_actions): dead -> no-op only
  for (int x = part * SM_THREADS + tid; x < A * nA; x += P * SM_THREADS) {
    const int j = x / nA, q = x - j * nA;
    const int i = c.rao ? prm[j] : j;
    const float al = ah[i] > 0.f ? 1.f : 0.f;
    float v;
    if (q == 0) v = 1.f - al;
    else if (q == 1) v = al;
    else if (q < 6) {
      const float nx = __fadd_rn(ax[i], dir_x(q - 2) * MOVE), ny = __fadd_rn(ay[i], dir_y(q - 2) * MOVE);
      v = (nx >= 0.f && nx <= MAP && ny >= 0.f && ny <= MAP) ? al : 0.f;
    } else {
      const int k = q - 6;
      float dx, dy;
      const float d2 = k < N ? sq2(ax[i], ay[i], ex[k], ey[k]) : INFINITY;
      v = (k < N && d2 <= SHOOT2 && d2 <= SIGHT2 && eh[k] > 0.f) ? al : 0.f;
    }
    o.ava[(size_t)e * A * nA + x] = v;
  }
}

}  // namespace

MDL_API int mdl_smac_env(const SmacCfg* c, const SmacState* s, const SmacState* so, const SmacOut* o, hipStream_t st) {
  if (c->A < 1 || c->A > SM_MAXU || c->N < 1 || c->N > SM_MAXU || c->nA != 6 + c->N || c->E < 1) return -1;
  if (c->obs_dim != 4 + c->N * (5 + c->u) + (c->A - 1) * (5 + c->u + c->nA) + (5 + c->u + c->nA) + c->A) return -2;
  if (c->state_dim != 4 + c->N * (8 + c->u) + (c->A - 1) * (8 + c->u + c->nA) + (7 + c->u + c->nA) + c->A) return -2;
  if (c->mode == 0 && !o->actions) return -1;
  // workgroups per env: enough for ~2 per CU of a 256-CU device, each with at least one thread per 4 of its values
  const int work = c->A * (c->obs_dim + c->state_dim + c->nA);
  int P = (512 + c->E - 1) / c->E;
  P = P < 1 ? 1 : P;
  const int pmax = (work + 4 * SM_THREADS - 1) / (4 * SM_THREADS);
  P = P > pmax ? pmax : P;
  P = P < 1 ? 1 : (P > 16 ? 16 : P);
  hipLaunchKernelGGL(smac_env_kernel, dim3(c->E, P), dim3(SM_THREADS), 0, st, *c, *s, *so, *o);
  MDL_CHECK_LAUNCH();
  return 0;
}
