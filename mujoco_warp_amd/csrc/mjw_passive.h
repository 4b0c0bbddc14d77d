// mjw_passive.h -- body forces of the passive stage beyond springs and dampers: gravity compensation
// (passive.py:246-272) and the fluid model (passive.py:276-533), shared by the world-per-wave forward
// kernel (mjw_step.hip) and the workgroup-per-world sparse path (mjw_sparse.hip).
//
// Both are forces on bodies applied at the body's inertial frame origin xipos and mapped to the dofs
// with the body Jacobian (support.py:174-216 apply_ft): dof i receives, over the bodies b of its body's
// subtree, cdof_i . W_b with W_b = (torque + off_b x force, force), off_b = xipos_b - subtree_com[root(b)].
#pragma once

#include "mjw_common.h"
#include "mjw_narrow.h"  // mat_t_vec3 (R^T v); matvec3 (R v) is in mjw_math.h

namespace mjw {

// world-frame wrench W = (t + off x f, f) of a body force (f, t) at xipos (see above)
__device__ __forceinline__ void body_wrench(float* W, const float* f, const float* t, const float* xipos, const float* sc_root) {
  const float off[3] = {xipos[0] - sc_root[0], xipos[1] - sc_root[1], xipos[2] - sc_root[2]};
  float c[3];
  cross3(c, off, f);
  for (int k = 0; k < 3; k++) { W[k] = t[k] + c[k]; W[3 + k] = f[k]; }
}

// passive.py:246-272: f = -gravity * mass * gravcomp, no torque
__device__ __forceinline__ void gravcomp_force(const mjw_model_t& m, int wid, int b, float* f) {
  const float gc = MR(body_gravcomp)[b];
  const float* g = MR(opt_gravity);
  const float s = b > 0 ? -MR(body_mass)[b] * gc : 0.0f;
  for (int k = 0; k < 3; k++) f[k] = gc != 0.0f ? g[k] * s : 0.0f;
}

// passive.py:42-59
__device__ __forceinline__ void fluid_semiaxes(const float* size, int type, float* s) {
  if (type == GEOM_SPHERE) { s[0] = s[1] = s[2] = size[0]; return; }
  if (type == GEOM_CAPSULE) { s[0] = s[1] = size[0]; s[2] = size[1] + size[0]; return; }
  if (type == GEOM_CYLINDER) { s[0] = s[1] = size[0]; s[2] = size[1]; return; }
  s[0] = size[0]; s[1] = size[1]; s[2] = size[2];
}

__device__ __forceinline__ float pow4f(float x) { const float q = x * x; return q * q; }

// passive.py:276-500 _fluid_force: the world-frame fluid force f and torque t on body b (zero for the
// world body and massless bodies).  cvel: the body's (angular, linear) com-based velocity; xipos / ximat:
// its inertial frame; sc_root: subtree_com of its root; gxpos / gxmat: the world's geom frames.
__device__ __forceinline__ void fluid_force(const mjw_model_t& m, int wid, int b, const float* xipos, const float* ximat, const float* cvel,
                                            const float* sc_root, const float* gxpos, const float* gxmat, float* f, float* t) {
  for (int k = 0; k < 3; k++) f[k] = t[k] = 0.0f;
  const float mass = MR(body_mass)[b];
  if (b == 0 || mass < MJW_MINVAL) return;
  const float* wind = MR(opt_wind);
  const float density = MR(opt_density)[0], viscosity = MR(opt_viscosity)[0];
  const float* ang = cvel;
  float lin_com[3];
  {
    const float off[3] = {xipos[0] - sc_root[0], xipos[1] - sc_root[1], xipos[2] - sc_root[2]};
    float c[3];
    cross3(c, off, ang);
    for (int k = 0; k < 3; k++) lin_com[k] = cvel[3 + k] - c[k];
  }
  if (m.body_fluid_ellipsoid[b]) {
    const float* gsize = MR(geom_size);
    const float* gfluid = MR(geom_fluid);
    const int g0 = m.body_geomadr[b], ng = m.body_geomnum[b];
    for (int g = g0; g < g0 + ng; g++) {
      const float* fl = gfluid + 12 * g;
      const float coef = fl[0];
      if (coef <= 0.0f) continue;
      float sa[3];
      fluid_semiaxes(gsize + 3 * g, m.geom_type[g], sa);
      const float* gr = gxmat + 9 * g;
      const float* gp = gxpos + 3 * g;
      float lin_point[3], d[3], c[3];
      for (int k = 0; k < 3; k++) d[k] = gp[k] - xipos[k];
      cross3(c, ang, d);
      for (int k = 0; k < 3; k++) lin_point[k] = lin_com[k] + c[k];
      float l_ang[3], l_lin[3], l_wind[3];
      mat_t_vec3(l_ang, gr, ang);
      mat_t_vec3(l_lin, gr, lin_point);
      mat_t_vec3(l_wind, gr, wind);
      for (int k = 0; k < 3; k++) l_lin[k] -= l_wind[k];
      float tq[3] = {0.0f, 0.0f, 0.0f}, fo[3] = {0.0f, 0.0f, 0.0f};
      if (density > 0.0f) {
        // added-mass forces and torques
        float vlm[3], vam[3], a1[3], a2[3];
        for (int k = 0; k < 3; k++) { vlm[k] = density * fl[6 + k] * l_lin[k]; vam[k] = density * fl[9 + k] * l_ang[k]; }
        cross3(a1, vlm, l_ang);
        for (int k = 0; k < 3; k++) fo[k] += a1[k];
        cross3(a1, vlm, l_lin);
        cross3(a2, vam, l_ang);
        for (int k = 0; k < 3; k++) tq[k] += a1[k] + a2[k];
      }
      const float magnus_coef = fl[5], kutta_coef = fl[4], blunt_drag_coef = fl[1], slender_drag_coef = fl[2], ang_drag_coef = fl[3];
      const float volume = (4.0f / 3.0f * 3.14159265358979f) * sa[0] * sa[1] * sa[2];
      const float d_max = fmaxf(fmaxf(sa[0], sa[1]), sa[2]), d_min = fminf(fminf(sa[0], sa[1]), sa[2]);
      const float d_mid = sa[0] + sa[1] + sa[2] - d_max - d_min;
      const float A_max = 3.14159265358979f * d_max * d_mid;
      const float lin_speed = sqrtf(l_lin[0] * l_lin[0] + l_lin[1] * l_lin[1] + l_lin[2] * l_lin[2]);
      float magnus[3];
      cross3(magnus, l_ang, l_lin);
      for (int k = 0; k < 3; k++) magnus[k] *= magnus_coef * density * volume;
      const float s12 = sa[1] * sa[2], s20 = sa[2] * sa[0], s01 = sa[0] * sa[1];
      const float proj_denom = pow4f(s12) * l_lin[0] * l_lin[0] + pow4f(s20) * l_lin[1] * l_lin[1] + pow4f(s01) * l_lin[2] * l_lin[2];
      const float proj_num = (s12 * l_lin[0]) * (s12 * l_lin[0]) + (s20 * l_lin[1]) * (s20 * l_lin[1]) + (s01 * l_lin[2]) * (s01 * l_lin[2]);
      float A_proj = 0.0f, cos_alpha = 0.0f;
      if (proj_num > MJW_MINVAL && proj_denom > MJW_MINVAL) {
        A_proj = 3.14159265358979f * sqrtf(proj_denom / fmaxf(MJW_MINVAL, proj_num));
        if (lin_speed > MJW_MINVAL) cos_alpha = proj_num / fmaxf(MJW_MINVAL, lin_speed * proj_denom);
      }
      const float nrm[3] = {s12 * s12 * l_lin[0], s20 * s20 * l_lin[1], s01 * s01 * l_lin[2]};
      float kutta[3] = {0.0f, 0.0f, 0.0f};
      if (density > 0.0f && kutta_coef != 0.0f && lin_speed > MJW_MINVAL) {
        float circ[3];
        cross3(circ, nrm, l_lin);
        for (int k = 0; k < 3; k++) circ[k] *= kutta_coef * density * cos_alpha * A_proj;
        cross3(kutta, circ, l_lin);
      }
      const float eq_D = (2.0f / 3.0f) * (sa[0] + sa[1] + sa[2]);
      const float lin_visc_force_coef = (3.0f * 3.14159265358979f) * eq_D;
      const float lin_visc_torq_coef = 3.14159265358979f * eq_D * eq_D * eq_D;
      const float I_max = (8.0f / 15.0f * 3.14159265358979f) * d_mid * pow4f(d_max);
      float mom_visc[3];
      for (int k = 0; k < 3; k++) {
        const float II = (8.0f / 15.0f * 3.14159265358979f) * sa[k] * pow4f(fmaxf(sa[(k + 1) % 3], sa[(k + 2) % 3]));
        mom_visc[k] = l_ang[k] * (ang_drag_coef * II + slender_drag_coef * (I_max - II));
      }
      const float drag_lin = viscosity * lin_visc_force_coef + density * lin_speed * (A_proj * blunt_drag_coef + slender_drag_coef * (A_max - A_proj));
      const float drag_ang =
          viscosity * lin_visc_torq_coef + density * sqrtf(mom_visc[0] * mom_visc[0] + mom_visc[1] * mom_visc[1] + mom_visc[2] * mom_visc[2]);
      for (int k = 0; k < 3; k++) {
        tq[k] = (tq[k] - drag_ang * l_ang[k]) * coef;
        fo[k] = (fo[k] + magnus[k] + kutta[k] - drag_lin * l_lin[k]) * coef;
      }
      float wt[3], wf[3];
      matvec3(wt, gr, tq);
      matvec3(wf, gr, fo);
      for (int k = 0; k < 3; k++) { t[k] += wt[k]; f[k] += wf[k]; }
    }
    return;
  }
  // inertia-box model (passive.py:455-500)
  float l_ang[3], l_lin[3], l_wind[3];
  mat_t_vec3(l_ang, ximat, ang);
  mat_t_vec3(l_lin, ximat, lin_com);
  mat_t_vec3(l_wind, ximat, wind);
  for (int k = 0; k < 3; k++) l_lin[k] -= l_wind[k];
  const bool has_visc = viscosity > 0.0f, has_dens = density > 0.0f;
  if (!has_visc && !has_dens) return;
  const float* inertia = MR(body_inertia) + 3 * b;
  const float scl = 6.0f / mass;
  const float box0 = sqrtf(fmaxf(MJW_MINVAL, inertia[1] + inertia[2] - inertia[0]) * scl);
  const float box1 = sqrtf(fmaxf(MJW_MINVAL, inertia[0] + inertia[2] - inertia[1]) * scl);
  const float box2 = sqrtf(fmaxf(MJW_MINVAL, inertia[0] + inertia[1] - inertia[2]) * scl);
  float tq[3] = {0.0f, 0.0f, 0.0f}, fo[3] = {0.0f, 0.0f, 0.0f};
  if (has_visc) {
    const float diam = (box0 + box1 + box2) / 3.0f;
    const float kt = diam * diam * diam * 3.14159265358979f * viscosity, kf = -3.0f * diam * 3.14159265358979f * viscosity;
    for (int k = 0; k < 3; k++) { tq[k] = -l_ang[k] * kt; fo[k] = kf * l_lin[k]; }
  }
  if (has_dens) {
    fo[0] -= 0.5f * density * box1 * box2 * fabsf(l_lin[0]) * l_lin[0];
    fo[1] -= 0.5f * density * box0 * box2 * fabsf(l_lin[1]) * l_lin[1];
    fo[2] -= 0.5f * density * box0 * box1 * fabsf(l_lin[2]) * l_lin[2];
    const float s = density / 64.0f;
    const float b0 = pow4f(box0), b1 = pow4f(box1), b2 = pow4f(box2);
    tq[0] -= box0 * (b1 + b2) * fabsf(l_ang[0]) * l_ang[0] * s;
    tq[1] -= box1 * (b0 + b2) * fabsf(l_ang[1]) * l_ang[1] * s;
    tq[2] -= box2 * (b0 + b1) * fabsf(l_ang[2]) * l_ang[2] * s;
  }
  matvec3(t, ximat, tq);
  matvec3(f, ximat, fo);
}

}  // namespace mjw
