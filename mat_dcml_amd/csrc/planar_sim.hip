// Fused planar-surrogate physics step for the multi-agent MuJoCo family (envs/mujoco/physics.py PlanarSim).
//
// The torch path issues ~50 small elementwise kernels per sub-step (nsub sub-steps per env step); even captured
// in a hipGraph that is ~3 M launches of a few microseconds each per profiled training run
// (profiles/r1_final/mujoco_kernel_stats.csv).  Here one thread owns one env copy and integrates all nsub
// sub-steps in a single launch: the link chain (J <= 64) lives in private arrays, the model constants
// (ancestor matrix, link geometry, actuator map) are staged once per block in LDS.  Math is the torch path's
// operation for operation (PlanarSim._fk / _point_vel / _forces / substep), fp32.
//
// Kinds: 0 = ground contact, 1 = viscous fluid (swimmer), 2 = fixed-base arm (reacher).  The tendon-coupled
// twin model (coupled_half_cheetah) stays on the torch path.
#include "common.h"

#define PS_MAXJ 64
#define PS_MAXR 8
#define PS_MAXU 64

struct PlanarConsts {
  int B, J, R, nu, nsub, kind;
  float h, mass, root_I, k_contact, c_contact, mu, grav_y, cn, ct;
};

// consts layout (floats): anc[J*J] | attach[J*2] | length[J] | rest[J] | damp[J] | stiff[J] | lo[J] | hi[J] |
//                         inertia[J] | root_attached[J] | root_ends[R*2] | gear[nu] | act_map[nu*(J+1)]
__global__ __launch_bounds__(64) void planar_step_kernel(PlanarConsts c, const float* __restrict__ consts,
                                                         int n_consts, const float* __restrict__ act,
                                                         float* p2, float* th_, float* v2, float* w_, float* q_,
                                                         float* qd_, float* tau_, float* f_end, float* f_root) {
  extern __shared__ float sc[];
  for (int i = threadIdx.x; i < n_consts; i += blockDim.x) sc[i] = consts[i];
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= c.B) return;
  const int J = c.J, R = c.R, nu = c.nu;
  const float* anc = sc;
  const float* attach = anc + J * J;
  const float* length = attach + 2 * J;
  const float* rest = length + J;
  const float* damp = rest + J;
  const float* stiff = damp + J;
  const float* lo = stiff + J;
  const float* hi = lo + J;
  const float* inertia = hi + J;
  const float* root_att = inertia + J;
  const float* root_ends = root_att + J;
  const float* gear = root_ends + 2 * R;
  const float* act_map = gear + nu;

  // motor torques: clamp(a) * gear @ act_map -> (J + 1), the last entry drives the root angle
  float tau_m[PS_MAXJ];
  float tau_root_m = 0.f;
  for (int j = 0; j < J; ++j) tau_m[j] = 0.f;
  for (int u = 0; u < nu; ++u) {
    float a = fminf(fmaxf(act[(size_t)b * nu + u], -1.f), 1.f) * gear[u];
    const float* row = act_map + u * (J + 1);
    for (int j = 0; j < J; ++j) tau_m[j] += a * row[j];
    tau_root_m += a * row[J];
  }

  float px = p2[2 * b], py = p2[2 * b + 1], th = th_[b], vx = v2[2 * b], vy = v2[2 * b + 1], w = w_[b];
  float q[PS_MAXJ], qd[PS_MAXJ];
  for (int j = 0; j < J; ++j) { q[j] = q_[(size_t)b * J + j]; qd[j] = qd_[(size_t)b * J + j]; }
  float flx[PS_MAXJ], fly[PS_MAXJ];
  float frx = 0.f, fry = 0.f;

  for (int s = 0; s < c.nsub; ++s) {
    float dx[PS_MAXJ], dy[PS_MAXJ], ex[PS_MAXJ], ey[PS_MAXJ], aw[PS_MAXJ], tau[PS_MAXJ];
    const float cth = cosf(th), sth = sinf(th);
    // forward kinematics: link angles, link vectors, absolute angular velocities
    for (int l = 0; l < J; ++l) {
      float ang = th, om = w;
      for (int a = 0; a < J; ++a) {
        const float m = anc[l * J + a];
        ang += m * (rest[a] + q[a]);
        om += m * qd[a];
      }
      dx[l] = length[l] * cosf(ang);
      dy[l] = length[l] * sinf(ang);
      aw[l] = om;
    }
    float vex[PS_MAXJ], vey[PS_MAXJ];
    for (int l = 0; l < J; ++l) {
      float x = px + cth * attach[2 * l] - sth * attach[2 * l + 1];
      float y = py + sth * attach[2 * l] + cth * attach[2 * l + 1];
      float ux = 0.f, uy = 0.f;
      for (int a = 0; a < J; ++a) {
        const float m = anc[l * J + a];
        x += m * dx[a];
        y += m * dy[a];
        ux += m * (-dy[a] * aw[a]);
        uy += m * (dx[a] * aw[a]);
      }
      ex[l] = x;
      ey[l] = y;
      const float rx = x - px, ry = y - py;
      vex[l] = vx + w * (-ry) + ux;
      vey[l] = vy + w * rx + uy;
    }
    for (int j = 0; j < J; ++j) {
      float t = tau_m[j] - damp[j] * qd[j] - stiff[j] * q[j];
      const float over = fmaxf(q[j] - hi[j], 0.f) + fminf(q[j] - lo[j], 0.f);
      tau[j] = t - 200.f * over * (1.f + 0.1f * fabsf(qd[j]));
    }
    if (c.kind == 2) {   // fixed-base arm
      for (int j = 0; j < J; ++j) {
        flx[j] = 0.f; fly[j] = 0.f;
        qd[j] = fminf(fmaxf(qd[j] + c.h * (tau[j] / inertia[j]), -50.f), 50.f);
        q[j] = q[j] + c.h * qd[j];
      }
      continue;
    }
    // external forces at the link points (ends for ground contact, midpoints in the fluid) and at the root
    float plx[PS_MAXJ], ply[PS_MAXJ];
    float Fx = 0.f, Fy = 0.f, troot = 0.f;
    frx = 0.f; fry = 0.f;
    if (c.kind == 0) {
      for (int i = 0; i < R; ++i) {
        const float rx = cth * root_ends[2 * i] - sth * root_ends[2 * i + 1];
        const float ry = sth * root_ends[2 * i] + cth * root_ends[2 * i + 1];
        const float y = py + ry;
        const float vxi = vx + w * (-ry), vyi = vy + w * rx;
        const float pen = fmaxf(-y, 0.f);
        const float fn = pen > 0.f ? fmaxf(c.k_contact * pen - c.c_contact * vyi, 0.f) : 0.f;
        const float ft = -c.mu * fn * tanhf(vxi / 0.05f);
        frx += ft; fry += fn;
        troot += rx * fn - ry * ft;
      }
      for (int l = 0; l < J; ++l) {
        const float pen = fmaxf(-ey[l], 0.f);
        const float fn = pen > 0.f ? fmaxf(c.k_contact * pen - c.c_contact * vey[l], 0.f) : 0.f;
        flx[l] = -c.mu * fn * tanhf(vex[l] / 0.05f);
        fly[l] = fn;
        plx[l] = ex[l];
        ply[l] = ey[l];
      }
    } else {
      // torso segment between root_ends[0] and root_ends[1], force at its midpoint
      const float r0x = cth * root_ends[0] - sth * root_ends[1], r0y = sth * root_ends[0] + cth * root_ends[1];
      const float r1x = cth * root_ends[2] - sth * root_ends[3], r1y = sth * root_ends[2] + cth * root_ends[3];
      float sx = r1x - r0x, sy = r1y - r0y;
      const float relx = 0.5f * (r0x + r1x), rely = 0.5f * (r0y + r1y);
      float tvx = vx + w * (-rely), tvy = vy + w * relx;
      {
        const float ln = fmaxf(sqrtf(sx * sx + sy * sy), 1e-6f);
        const float tx = sx / ln, ty = sy / ln, nx = -ty, ny = tx;
        const float vt = tvx * tx + tvy * ty, vn = tvx * nx + tvy * ny;
        const float fx = -(c.ct * vt * tx + c.cn * vn * nx) * ln, fy = -(c.ct * vt * ty + c.cn * vn * ny) * ln;
        frx = fx; fry = fy;
        troot += relx * fy - rely * fx;
      }
      for (int l = 0; l < J; ++l) {
        const float mx = ex[l] - 0.5f * dx[l], my = ey[l] - 0.5f * dy[l];
        const float mvx = vex[l] - 0.5f * (-dy[l]) * aw[l], mvy = vey[l] - 0.5f * dx[l] * aw[l];
        const float ln = fmaxf(sqrtf(dx[l] * dx[l] + dy[l] * dy[l]), 1e-6f);
        const float tx = dx[l] / ln, ty = dy[l] / ln, nx = -ty, ny = tx;
        const float vt = mvx * tx + mvy * ty, vn = mvx * nx + mvy * ny;
        flx[l] = -(c.ct * vt * tx + c.cn * vn * nx) * ln;
        fly[l] = -(c.ct * vt * ty + c.cn * vn * ny) * ln;
        plx[l] = mx;
        ply[l] = my;
      }
    }
    Fx = frx; Fy = fry;
    for (int l = 0; l < J; ++l) {
      Fx += flx[l];
      Fy += fly[l];
      troot += (plx[l] - px) * fly[l] - (ply[l] - py) * flx[l];
      troot -= tau_m[l] * root_att[l];
    }
    troot += tau_root_m;
    // joint torques: moments about each joint (start of its link) of every force downstream of it
    for (int j = 0; j < J; ++j) {
      float cp = 0.f, fdx = 0.f, fdy = 0.f;
      for (int l = 0; l < J; ++l) {
        const float m = anc[l * J + j];   // down[j, l]
        cp += m * (plx[l] * fly[l] - ply[l] * flx[l]);
        fdx += m * flx[l];
        fdy += m * fly[l];
      }
      const float sxj = ex[j] - dx[j], syj = ey[j] - dy[j];
      tau[j] += cp - (sxj * fdy - syj * fdx);
    }
    if (c.kind == 0) Fy += c.grav_y;
    vx = fminf(fmaxf(vx + c.h * (Fx / c.mass), -30.f), 30.f);
    vy = fminf(fmaxf(vy + c.h * (Fy / c.mass), -30.f), 30.f);
    w = fminf(fmaxf(w + c.h * (troot / c.root_I), -40.f), 40.f);
    for (int j = 0; j < J; ++j) qd[j] = fminf(fmaxf(qd[j] + c.h * (tau[j] / inertia[j]), -60.f), 60.f);
    px += c.h * vx;
    py += c.h * vy;
    th += c.h * w;
    for (int j = 0; j < J; ++j) q[j] += c.h * qd[j];
  }

  for (int j = 0; j < J; ++j) {
    q_[(size_t)b * J + j] = q[j];
    qd_[(size_t)b * J + j] = qd[j];
    f_end[((size_t)b * J + j) * 2] = flx[j];
    f_end[((size_t)b * J + j) * 2 + 1] = fly[j];
  }
  if (c.kind != 2) {
    p2[2 * b] = px; p2[2 * b + 1] = py; th_[b] = th; v2[2 * b] = vx; v2[2 * b + 1] = vy; w_[b] = w;
    for (int j = 0; j < J; ++j) tau_[(size_t)b * J + j] = tau_m[j];
    f_root[2 * b] = frx; f_root[2 * b + 1] = fry;
  }
}

MDL_API int mdl_planar_step(const PlanarConsts* c, const float* consts, int n_consts, const float* act,
                               float* p, float* th, float* v, float* w, float* q, float* qd, float* tau,
                               float* f_end, float* f_root, hipStream_t stream) {
  if (c->J < 1 || c->J > PS_MAXJ || c->R > PS_MAXR || c->nu > PS_MAXU || c->kind < 0 || c->kind > 2) return -1;
  if (c->kind == 1 && c->R < 2) return -1;
  if ((size_t)n_consts * sizeof(float) > 64 * 1024) return -1;
  const int threads = 64;
  const int blocks = (c->B + threads - 1) / threads;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(planar_step_kernel, dim3(blocks), dim3(threads), n_consts * sizeof(float), stream, *c, consts,
                     n_consts, act, p, th, v, w, q, qd, tau, f_end, f_root);
  return (int)hipGetLastError();
}
