// mjw_tendon.h -- tendons on the world-per-wavefront path: fixed (joint) tendons (smooth.py:3085-3121)
// and spatial tendons -- site paths wrapping around spheres / cylinders, split by pulleys
// (smooth.py:3172-3465, util_misc.py:30-450) -- with their armature in qM (smooth.py:916-1000) and armature
// bias (smooth.py:1590-1932), velocity (forward.py:604-609), spring / damper (passive.py:183-252),
// friction and limit rows (constraint.py:1204-1313, 1547-1665), tendon transmissions
// (smooth.py:2244-2260) and the tendon actuator force range (forward.py:739-779).
//
// A fixed tendon's Jacobian is its wrap coefficients at the joints' dofs, the same in every world, so
// the helpers recompute lengths and coefficients from the model and the world's qpos / qvel in LDS
// instead of keeping per-stage copies.  A spatial tendon's length and Jacobian depend on the pose: the
// position stage computes them once per world (one lane per tendon) into the Data's ten_length / ten_J,
// and every later user reads them there.  Every routine is a no-op for models without tendons
// (ntendon = 0 is a wave-uniform branch), which keeps the hot kernels' registers untouched.
#pragma once
#include "mjw_common.h"

namespace mjw {

#define WRAP_JOINT 1
#define WRAP_PULLEY 2
#define WRAP_SITE 3
#define WRAP_SPHERE 4
#define WRAP_CYLINDER 5
#define TEN_MAXVAL 1.0e10f

__device__ __forceinline__ bool ten_spatial(const mjw_model_t& m, int t) { return m.wrap_type[m.tendon_adr[t]] != WRAP_JOINT; }

// coefficient of tendon t at dof `dof`: for a fixed tendon the last wrap on that dof's joint (as
// _joint_tendon writes it), for a spatial one the Data's ten_J entry
__device__ __forceinline__ float ten_coef(const mjw_model_t& m, const mjw_data_t& d, int wid, int t, int dof) {
  float c = 0.0f;
  if (ten_spatial(m, t)) {
    const int ra = m.ten_J_rowadr[t];
    for (int k = 0; k < m.ten_J_rownnz[t]; k++)
      if (m.ten_J_colind[ra + k] == dof) c = d.ten_J[(long)wid * m.nJten + ra + k];
    return c;
  }
  const float* prm = MR(wrap_prm);
  for (int w = m.tendon_adr[t]; w < m.tendon_adr[t] + m.tendon_num[t]; w++)
    if (m.jnt_dofadr[m.wrap_objid[w]] == dof) c = prm[w];
  return c;
}

// tendon length: sum coef * qpos (qpos: the world's qpos in LDS) or the spatial tendon's Data length
__device__ __forceinline__ float ten_len(const mjw_model_t& m, const mjw_data_t& d, int wid, const float* qpos, int t) {
  if (ten_spatial(m, t)) return d.ten_length[(long)wid * m.ntendon + t];
  float L = 0.0f;
  const float* prm = MR(wrap_prm);
  for (int w = m.tendon_adr[t]; w < m.tendon_adr[t] + m.tendon_num[t]; w++) L += prm[w] * qpos[m.jnt_qposadr[m.wrap_objid[w]]];
  return L;
}

// tendon velocity J qvel over the sparse row
__device__ __forceinline__ float ten_vel(const mjw_model_t& m, const mjw_data_t& d, int wid, const float* qvel, int t) {
  float v = 0.0f;
  for (int k = 0; k < m.ten_J_rownnz[t]; k++) {
    const int dof = m.ten_J_colind[m.ten_J_rowadr[t] + k];
    v += ten_coef(m, d, wid, t, dof) * qvel[dof];
  }
  return v;
}

// ---- wrap geometry (util_misc.py), fp32 -------------------------------------------------------------
__device__ __forceinline__ float ten_len2(float x, float y) { return sqrtf(x * x + y * y); }

// util_misc.py:30-56
__device__ __forceinline__ bool wrap_is_intersect(const float* p1, const float* p2, const float* p3, const float* p4) {
  const float det = (p4[1] - p3[1]) * (p2[0] - p1[0]) - (p4[0] - p3[0]) * (p2[1] - p1[1]);
  if (fabsf(det) < MJW_MINVAL) return false;
  const float a = ((p4[0] - p3[0]) * (p1[1] - p3[1]) - (p4[1] - p3[1]) * (p1[0] - p3[0])) / det;
  const float b = ((p2[0] - p1[0]) * (p1[1] - p3[1]) - (p2[1] - p1[1]) * (p1[0] - p3[0])) / det;
  return a >= 0.0f && a <= 1.0f && b >= 0.0f && b <= 1.0f;
}

// util_misc.py:76-100
__device__ __forceinline__ float wrap_length_circle(const float* p0, const float* p1, int ind, float radius) {
  const float n0 = ten_len2(p0[0], p0[1]), n1 = ten_len2(p1[0], p1[1]);
  const float c = n0 > 0.0f && n1 > 0.0f ? (p0[0] * p1[0] + p0[1] * p1[1]) / (n0 * n1) : 0.0f;
  float angle = acosf(fminf(fmaxf(c, -1.0f), 1.0f));
  const float cross = p0[1] * p1[0] - p0[0] * p1[1];
  if ((cross > 0.0f && ind != 0) || (cross < 0.0f && ind == 0)) angle = 2.0f * (float)M_PI - angle;
  return radius * angle;
}

__device__ __forceinline__ float ten_safe_div(float x, float y) { return x / (y != 0.0f ? y : MJW_MINVAL); }

// util_misc.py:103-198: 2D wrap of end[0:2] - end[2:4] around a circle at the origin; -1 when it does not wrap
__device__ float wrap_circle(const float* end, const float* side, float radius, float* q0, float* q1) {
  const bool valid_side = ten_len2(side[0], side[1]) < TEN_MAXVAL;
  const float sq0 = end[0] * end[0] + end[1] * end[1], sq1 = end[2] * end[2] + end[3] * end[3], sqr = radius * radius;
  q0[0] = q0[1] = q1[0] = q1[1] = TEN_MAXVAL;
  if (sq0 < sqr || sq1 < sqr || radius < MJW_MINVAL) return -1.0f;
  const float dx = end[2] - end[0], dy = end[3] - end[1], dd = dx * dx + dy * dy;
  if (dd < MJW_MINVAL) return -1.0f;
  const float a = fminf(fmaxf(-(dx * end[0] + dy * end[1]) / dd, 0.0f), 1.0f);
  const float tx = a * dx + end[0], ty = a * dy + end[1];
  if (tx * tx + ty * ty > sqr && (!valid_side || side[0] * tx + side[1] * ty >= 0.0f)) return -1.0f;
  const float s0 = sqrtf(sq0 - sqr), s1 = sqrtf(sq1 - sqr);
  const float sol00[2] = {ten_safe_div(end[0] * sqr + radius * end[1] * s0, sq0), ten_safe_div(end[1] * sqr - radius * end[0] * s0, sq0)};
  const float sol01[2] = {ten_safe_div(end[2] * sqr - radius * end[3] * s1, sq1), ten_safe_div(end[3] * sqr + radius * end[2] * s1, sq1)};
  const float sol10[2] = {ten_safe_div(end[0] * sqr - radius * end[1] * s0, sq0), ten_safe_div(end[1] * sqr + radius * end[0] * s0, sq0)};
  const float sol11[2] = {ten_safe_div(end[2] * sqr + radius * end[3] * s1, sq1), ten_safe_div(end[3] * sqr - radius * end[2] * s1, sq1)};
  float good0, good1;
  if (valid_side) {
    const float m0x = sol00[0] + sol01[0], m0y = sol00[1] + sol01[1], m1x = sol10[0] + sol11[0], m1y = sol10[1] + sol11[1];
    const float n0 = ten_len2(m0x, m0y), n1 = ten_len2(m1x, m1y);
    good0 = n0 > 0.0f ? (m0x * side[0] + m0y * side[1]) / n0 : 0.0f;
    good1 = n1 > 0.0f ? (m1x * side[0] + m1y * side[1]) / n1 : 0.0f;
  } else {
    const float d0x = sol00[0] - sol01[0], d0y = sol00[1] - sol01[1], d1x = sol10[0] - sol11[0], d1y = sol10[1] - sol11[1];
    good0 = -(d0x * d0x + d0y * d0y);
    good1 = -(d1x * d1x + d1y * d1y);
  }
  const float e0[2] = {end[0], end[1]}, e1[2] = {end[2], end[3]};
  if (wrap_is_intersect(e0, sol00, e1, sol01)) good0 = -10000.0f;
  if (wrap_is_intersect(e0, sol10, e1, sol11)) good1 = -10000.0f;
  const bool first = good0 > good1;
  const float* p0 = first ? sol00 : sol10;
  const float* p1 = first ? sol01 : sol11;
  if (wrap_is_intersect(e0, p0, e1, p1)) return -1.0f;
  q0[0] = p0[0]; q0[1] = p0[1]; q1[0] = p1[0]; q1[1] = p1[1];
  return wrap_length_circle(p0, p1, first ? 0 : 1, radius);
}

// util_misc.py:201-323: the single tangent point of an inside wrap (sidesite within the geom)
__device__ float wrap_inside(const float* end, float radius, float* q0, float* q1) {
  q0[0] = q0[1] = q1[0] = q1[1] = TEN_MAXVAL;
  const float len0 = ten_len2(end[0], end[1]), len1 = ten_len2(end[2], end[3]);
  const float dx = end[2] - end[0], dy = end[3] - end[1], dd = dx * dx + dy * dy;
  if (len0 <= radius || len1 <= radius || radius < MJW_MINVAL || len0 < MJW_MINVAL || len1 < MJW_MINVAL) return -1.0f;
  if (dd > MJW_MINVAL) {
    const float a = -(dx * end[0] + dy * end[1]) / dd;
    if (a > 0.0f && a < 1.0f && ten_len2(end[0] + a * dx, end[1] + a * dy) <= radius) return -1.0f;
  }
  const float mx = 0.5f * (end[0] + end[2]), my = 0.5f * (end[1] + end[3]), mn = ten_len2(mx, my);
  q0[0] = q1[0] = mn > 0.0f ? mx / mn * radius : 0.0f;
  q0[1] = q1[1] = mn > 0.0f ? my / mn * radius : 0.0f;
  const float A = ten_safe_div(radius, len0), B = ten_safe_div(radius, len1);
  const float cosG = ten_safe_div(len0 * len0 + len1 * len1 - dd, 2.0f * len0 * len1);
  if (cosG < -1.0f + MJW_MINVAL) return -1.0f;
  if (cosG > 1.0f - MJW_MINVAL) return 0.0f;
  const float G = acosf(cosG);
  float z = 1.0f - 1.0e-7f;
  float f = asinf(A * z) + asinf(B * z) - 2.0f * asinf(z) + G;
  if (f > 0.0f) return 0.0f;
  int it = 0;
  while (it < 20 && fabsf(f) > 1.0e-6f) {
    const float sz = z * z;
    const float df = A / fmaxf(MJW_MINVAL, sqrtf(1.0f - sz * A * A)) + B / fmaxf(MJW_MINVAL, sqrtf(1.0f - sz * B * B)) -
                     2.0f / fmaxf(MJW_MINVAL, sqrtf(1.0f - sz));
    if (df > -MJW_MINVAL) return 0.0f;
    const float z1 = z - ten_safe_div(f, df);
    if (z1 > z) return 0.0f;
    z = z1;
    f = asinf(A * z) + asinf(B * z) - 2.0f * asinf(z) + G;
    if (f > 1.0e-6f) return 0.0f;
    it++;
  }
  if (it >= 20) return 0.0f;
  const bool left = end[0] * end[3] - end[1] * end[2] > 0.0f;
  const float vx = left ? end[0] : end[2], vy = left ? end[1] : end[3], vn = ten_len2(vx, vy);
  const float ang = asinf(z) - asinf((left ? A : B) * z);
  const float ux = vn > 0.0f ? vx / vn : 0.0f, uy = vn > 0.0f ? vy / vn : 0.0f;
  q0[0] = q1[0] = radius * (cosf(ang) * ux - sinf(ang) * uy);
  q0[1] = q1[1] = radius * (sinf(ang) * ux + cosf(ang) * uy);
  return 0.0f;
}

// util_misc.py:326-450: wrap x0 - x1 around a sphere / infinite cylinder at pos / mat (row-major); side =
// sidesite position or TEN_MAXVAL.  Returns the wrapped length or -1, world tangent points in w0 / w1.
__device__ float wrap_geom(const float* x0, const float* x1, const float* pos, const float* mat, float radius, int type, const float* side,
                           float* w0, float* w1) {
  float d0[3], d1[3], p0[3], p1[3];
  for (int i = 0; i < 3; i++) { d0[i] = x0[i] - pos[i]; d1[i] = x1[i] - pos[i]; }
  for (int i = 0; i < 3; i++) {
    p0[i] = mat[i] * d0[0] + mat[3 + i] * d0[1] + mat[6 + i] * d0[2];
    p1[i] = mat[i] * d1[0] + mat[3 + i] * d1[1] + mat[6 + i] * d1[2];
  }
  if (sqrtf(dot3(p0, p0)) < MJW_MINVAL || sqrtf(dot3(p1, p1)) < MJW_MINVAL) return -1.0f;
  float axis0[3], axis1[3];
  if (type == WRAP_SPHERE) {
    const float n0 = sqrtf(dot3(p0, p0));
    for (int i = 0; i < 3; i++) axis0[i] = p0[i] / n0;
    float nrm[3];
    cross3(nrm, p0, p1);
    float nn = sqrtf(dot3(nrm, nrm));
    if (nn < MJW_MINVAL) {
      const float ab0 = fabsf(axis0[0]), ab1 = fabsf(axis0[1]), ab2 = fabsf(axis0[2]);
      int i = 0;
      if (ab1 > ab0 && ab1 > ab2) i = 1;
      if (ab2 > ab0 && ab2 > ab1) i = 2;
      float a1[3] = {1.0f, 1.0f, 1.0f};
      a1[i] = 0.0f;
      cross3(nrm, axis0, a1);
      nn = sqrtf(dot3(nrm, nrm));
    }
    for (int i = 0; i < 3; i++) nrm[i] = nn > 0.0f ? nrm[i] / nn : 0.0f;
    cross3(axis1, nrm, axis0);
    const float n1 = sqrtf(dot3(axis1, axis1));
    for (int i = 0; i < 3; i++) axis1[i] = n1 > 0.0f ? axis1[i] / n1 : 0.0f;
  } else {
    axis0[0] = 1.0f; axis0[1] = 0.0f; axis0[2] = 0.0f;
    axis1[0] = 0.0f; axis1[1] = 1.0f; axis1[2] = 0.0f;
  }
  const float end[4] = {dot3(p0, axis0), dot3(p0, axis1), dot3(p1, axis0), dot3(p1, axis1)};
  const bool valid_side = sqrtf(dot3(side, side)) < TEN_MAXVAL;
  float sidepnt[3] = {0.0f, 0.0f, 0.0f}, sproj[2] = {TEN_MAXVAL, TEN_MAXVAL};
  if (valid_side) {
    const float ds[3] = {side[0] - pos[0], side[1] - pos[1], side[2] - pos[2]};
    for (int i = 0; i < 3; i++) sidepnt[i] = mat[i] * ds[0] + mat[3 + i] * ds[1] + mat[6 + i] * ds[2];
    const float sx = dot3(sidepnt, axis0), sy = dot3(sidepnt, axis1), sn = ten_len2(sx, sy);
    sproj[0] = sn > 0.0f ? sx / sn * radius : 0.0f;
    sproj[1] = sn > 0.0f ? sy / sn * radius : 0.0f;
  }
  float q0[2], q1[2];
  float wlen = (valid_side && sqrtf(dot3(sidepnt, sidepnt)) < radius) ? wrap_inside(end, radius, q0, q1) : wrap_circle(end, sproj, radius, q0, q1);
  if (wlen < 0.0f) return -1.0f;
  float r0[3], r1[3];
  for (int i = 0; i < 3; i++) {
    r0[i] = axis0[i] * q0[0] + axis1[i] * q0[1];
    r1[i] = axis0[i] * q1[0] + axis1[i] * q1[1];
  }
  if (type == WRAP_CYLINDER) {
    const float L0 = ten_len2(p0[0] - r0[0], p0[1] - r0[1]), L1 = ten_len2(p1[0] - r1[0], p1[1] - r1[1]);
    r0[2] = p0[2] + (p1[2] - p0[2]) * ten_safe_div(L0, L0 + wlen + L1);
    r1[2] = p0[2] + (p1[2] - p0[2]) * ten_safe_div(L0 + wlen, L0 + wlen + L1);
    wlen = sqrtf(wlen * wlen + (r1[2] - r0[2]) * (r1[2] - r0[2]));
  }
  for (int i = 0; i < 3; i++) {
    w0[i] = mat[3 * i] * r0[0] + mat[3 * i + 1] * r0[1] + mat[3 * i + 2] * r0[2] + pos[i];
    w1[i] = mat[3 * i] * r1[0] + mat[3 * i + 1] * r1[1] + mat[3 * i + 2] * r1[2] + pos[i];
  }
  return wlen;
}

// ---- spatial tendon length / Jacobian (smooth.py:3126-3465) -----------------------------------------
struct TenFrames {
  const float* site_xpos;    // world's site positions (the Data's, written by kinematics)
  const float* gxpos;        // geom positions / frames
  const float* gxmat;
  const float* subtree_com;  // LDS
  const float* cdof;         // LDS
};

// smooth.py:3126-3170: J[k] += scale vec . (cdof_lin + cdof_ang x (pnt - subtree_com[root])) along the chain
__device__ __forceinline__ void ten_jac_chain(const mjw_model_t& m, float* J, int t, int body, const float* pnt, const float* vec, float scale,
                                              const TenFrames& f) {
  const int ra = m.ten_J_rowadr[t], rn = m.ten_J_rownnz[t];
  const float* sc = f.subtree_com + 3 * m.body_rootid[body];
  const float off[3] = {pnt[0] - sc[0], pnt[1] - sc[1], pnt[2] - sc[2]};
  int k = rn - 1;  // colind ascending, the chain's dofs descending
  for (int b = body; b > 0; b = m.body_parentid[b]) {
    for (int dof = m.body_dofadr[b] + m.body_dofnum[b] - 1; dof >= m.body_dofadr[b]; dof--) {
      while (k >= 0 && m.ten_J_colind[ra + k] > dof) k--;
      if (k < 0 || m.ten_J_colind[ra + k] != dof) continue;
      const float* cd = f.cdof + 6 * dof;
      float c[3];
      cross3(c, cd, off);
      J[k] += scale * ((cd[3] + c[0]) * vec[0] + (cd[4] + c[1]) * vec[1] + (cd[5] + c[2]) * vec[2]);
    }
  }
}

__device__ __forceinline__ float ten_segment(const mjw_model_t& m, float* J, int t, const float* p0, int b0, const float* p1, int b1, float scale,
                                             const TenFrames& f) {
  float v[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
  const float len = sqrtf(dot3(v, v));
  if (len < MJW_MINVAL) { v[0] = 1.0f; v[1] = 0.0f; v[2] = 0.0f; }
  else { v[0] /= len; v[1] /= len; v[2] /= len; }
  if (b0 != b1) {
    ten_jac_chain(m, J, t, b0, p0, v, -scale, f);
    ten_jac_chain(m, J, t, b1, p1, v, scale, f);
  }
  return len;
}

// length of spatial tendon t; its ten_J row J (rownnz entries, zeroed by the caller) accumulated
__device__ float spatial_tendon(const mjw_model_t& m, int wid, float* J, int t, const TenFrames& f) {
  const int a = m.tendon_adr[t], n = m.tendon_num[t];
  const float* psc = MR(wrap_pulley_scale);
  const float* prm = MR(wrap_prm);
  const float* gsize = MR(geom_size);
  float L = 0.0f;
  int j = 0;
  while (j < n - 1) {
    const int t0 = m.wrap_type[a + j], t1 = m.wrap_type[a + j + 1];
    if (t0 == WRAP_PULLEY || t1 == WRAP_PULLEY) { j++; continue; }
    const int s0 = m.wrap_objid[a + j];
    const float* p0 = f.site_xpos + 3 * s0;
    const int b0 = m.site_bodyid[s0];
    if (t1 == WRAP_SPHERE || t1 == WRAP_CYLINDER) {
      const int g = m.wrap_objid[a + j + 1], s1 = m.wrap_objid[a + j + 2], gb = m.geom_bodyid[g];
      const float* p1 = f.site_xpos + 3 * s1;
      const int b1 = m.site_bodyid[s1];
      const float sc = psc[a + j + 1];
      const int sid = (int)rintf(prm[a + j + 1]);
      float side[3] = {TEN_MAXVAL, TEN_MAXVAL, TEN_MAXVAL}, g0[3], g1[3];
      if (sid >= 0)
        for (int i = 0; i < 3; i++) side[i] = f.site_xpos[3 * sid + i];
      const float wl = wrap_geom(p0, p1, f.gxpos + 3 * g, f.gxmat + 9 * g, gsize[3 * g], t1, side, g0, g1);
      if (wl >= 0.0f) {
        const float l0 = ten_segment(m, J, t, p0, b0, g0, gb, sc, f);
        const float l1 = ten_segment(m, J, t, g1, gb, p1, b1, sc, f);
        L += (l0 + wl + l1) * sc;
      } else {
        L += ten_segment(m, J, t, p0, b0, p1, b1, sc, f) * sc;
      }
      j += 2;
    } else {
      const int s1 = m.wrap_objid[a + j + 1];
      const float sc = psc[a + j];
      L += ten_segment(m, J, t, p0, b0, f.site_xpos + 3 * s1, m.site_bodyid[s1], sc, f) * sc;
      j++;
    }
  }
  return L;
}

// position stage: ten_length, ten_J (Data contract).  Spatial tendons: one lane per tendon accumulates
// its row in registers-then-global (the row's owner is the only writer); the caller syncs the wave
// before any reader.
__device__ __forceinline__ void tendon_pos(const mjw_model_t& m, const mjw_data_t& d, const float* qpos, const TenFrames& f, int wid, int lane,
                                           int stride = 64) {
  for (int t = lane; t < m.ntendon; t += stride) {
    float* J = d.ten_J + (long)wid * m.nJten + m.ten_J_rowadr[t];
    if (ten_spatial(m, t)) {
      for (int k = 0; k < m.ten_J_rownnz[t]; k++) J[k] = 0.0f;
      d.ten_length[(long)wid * m.ntendon + t] = spatial_tendon(m, wid, J, t, f);
      continue;
    }
    d.ten_length[(long)wid * m.ntendon + t] = ten_len(m, d, wid, qpos, t);
    for (int k = 0; k < m.ten_J_rownnz[t]; k++) J[k] = ten_coef(m, d, wid, t, m.ten_J_colind[m.ten_J_rowadr[t] + k]);
  }
}

// smooth.py:1590-1653 (_accumulate_jac_dot_chain), summed against qvel: sum_k Jdot_k qvel_k over the chain
__device__ __forceinline__ float ten_jacdot_chain(const mjw_model_t& m, int body, const float* off, const float* pvel, const float* dpnt,
                                                  const float* dvel, const float* cdof, const float* cdof_dot, const float* cvel,
                                                  const float* qvel) {
  float acc = 0.0f;
  for (int b = body; b > 0; b = m.body_parentid[b])
    for (int dof = m.body_dofadr[b]; dof < m.body_dofadr[b] + m.body_dofnum[b]; dof++) {
      const float* cd = cdof + 6 * dof;
      float cdd[6];
      const int jid = m.dof_jntid[dof], jt = m.jnt_type[jid];
      if (jt == JNT_BALL || (jt == JNT_FREE && dof >= m.jnt_dofadr[jid] + 3)) motion_cross(cdd, cvel + 6 * b, cd);
      else
        for (int i = 0; i < 6; i++) cdd[i] = cdof_dot[6 * dof + i];
      float c1[3], c2[3], c3[3];
      cross3(c1, cdd, off);
      cross3(c2, cd, pvel);
      cross3(c3, cd, off);
      float jd = 0.0f;
      for (int i = 0; i < 3; i++) jd += (cdd[3 + i] + c1[i] + c2[i]) * dpnt[i] + (cd[3 + i] + c3[i]) * dvel[i];
      acc += jd * qvel[dof];
    }
  return acc;
}

// smooth.py:1656-1840 (_tendon_dot, _tendon_bias_coef): armature_t (dJ_t/dt qvel) of spatial tendon t (0 for fixed
// tendons and tendons without armature); as the reference, a site-geom-site wrap ends the tendon's Jdot
// (segments before it count)
__device__ float tendon_bias_coef(const mjw_model_t& m, int wid, int t, const float* qvel, const TenFrames& f, const float* cvel,
                                  const float* cdof_dot) {
  const float* arm = MR(tendon_armature);
  if (arm[t] == 0.0f || !ten_spatial(m, t)) return 0.0f;
  const int a = m.tendon_adr[t], n = m.tendon_num[t];
  float divisor = 1.0f, c = 0.0f;
  for (int j = 0; j < n - 1; j++) {
    const int t0 = m.wrap_type[a + j], t1 = m.wrap_type[a + j + 1];
    if (t0 == WRAP_PULLEY || t1 == WRAP_PULLEY) {
      if (t0 == WRAP_PULLEY) divisor = MR(wrap_prm)[a + j];
      continue;
    }
    if (t1 == WRAP_SPHERE || t1 == WRAP_CYLINDER) break;
    const int s0 = m.wrap_objid[a + j], s1 = m.wrap_objid[a + j + 1];
    const int b0 = m.site_bodyid[s0], b1 = m.site_bodyid[s1];
    if (b0 == b1) continue;
    const float *p0 = f.site_xpos + 3 * s0, *p1 = f.site_xpos + 3 * s1;
    const float *sc0 = f.subtree_com + 3 * m.body_rootid[b0], *sc1 = f.subtree_com + 3 * m.body_rootid[b1];
    float off0[3], off1[3], v0[3], v1[3], dif[3], c0[3], c1[3];
    for (int i = 0; i < 3; i++) { off0[i] = p0[i] - sc0[i]; off1[i] = p1[i] - sc1[i]; dif[i] = p1[i] - p0[i]; }
    cross3(c0, off0, cvel + 6 * b0);
    cross3(c1, off1, cvel + 6 * b1);
    for (int i = 0; i < 3; i++) { v0[i] = cvel[6 * b0 + 3 + i] - c0[i]; v1[i] = cvel[6 * b1 + 3 + i] - c1[i]; }
    const float nrm = sqrtf(dot3(dif, dif));
    float dpnt[3], dvel[3];
    for (int i = 0; i < 3; i++) dpnt[i] = nrm > 0.0f ? dif[i] / nrm : 0.0f;
    for (int i = 0; i < 3; i++) dvel[i] = v1[i] - v0[i];
    const float dt = dot3(dpnt, dvel);
    for (int i = 0; i < 3; i++) dvel[i] = nrm > MJW_MINVAL ? (dvel[i] - dpnt[i] * dt) / nrm : 0.0f;
    const float inv = ten_safe_div(1.0f, divisor);
    c += inv * (ten_jacdot_chain(m, b1, off1, v1, dpnt, dvel, f.cdof, cdof_dot, cvel, qvel) -
                ten_jacdot_chain(m, b0, off0, v0, dpnt, dvel, f.cdof, cdof_dot, cvel, qvel));
  }
  return c * arm[t];
}

// smooth.py:1843-1932 (_tendon_bias_qfrc): out[i] = sum_t coef_t J_ti for the wave's world (lane stride 64;
// coef: 64 floats of LDS scratch)
__device__ __forceinline__ void tendon_bias(const mjw_model_t& m, const mjw_data_t& d, int wid, int lane, const float* qvel, const TenFrames& f,
                                            const float* cvel, const float* cdof_dot, float* coef, float* out) {
  for (int i = lane; i < m.nv; i += 64) out[i] = 0.0f;
  for (int base = 0; base < m.ntendon; base += 64) {
    const int t = base + lane;
    coef[lane] = t < m.ntendon ? tendon_bias_coef(m, wid, t, qvel, f, cvel, cdof_dot) : 0.0f;
    __syncthreads();
    for (int i = lane; i < m.nv; i += 64) {
      float acc = 0.0f;
      for (int q = 0; q < 64 && base + q < m.ntendon; q++)
        if (coef[q] != 0.0f) acc += coef[q] * ten_coef(m, d, wid, base + q, i);
      out[i] += acc;
    }
    __syncthreads();
  }
}

// qM[i][j] += armature J_i J_j for j = i or an ancestor of i (the pattern of qM), M row stride nvs;
// one tendon at a time, lanes over its (k1, k2) entry pairs (distinct (i, j) within a tendon)
__device__ __forceinline__ void tendon_armature(const mjw_model_t& m, const mjw_data_t& d, float* M, int nvs, int wid, int lane) {
  const float* arm = MR(tendon_armature);
  for (int t = 0; t < m.ntendon; t++) {
    if (arm[t] == 0.0f) continue;
    const int rn = m.ten_J_rownnz[t], ra = m.ten_J_rowadr[t];
    for (int p = lane; p < rn * rn; p += 64) {
      const int k1 = p / rn, k2 = p - k1 * rn;
      if (k2 > k1) continue;
      const int i = m.ten_J_colind[ra + k1], j = m.ten_J_colind[ra + k2];  // colind ascending: j <= i
      int a = i;
      while (a > j) a = m.dof_parentid[a];
      if (a != j) continue;
      const float v = arm[t] * ten_coef(m, d, wid, t, i) * ten_coef(m, d, wid, t, j);
      M[i * nvs + j] += v;
      if (i != j) M[j * nvs + i] += v;
    }
    __syncthreads();
  }
}

// velocity stage: ten_velocity and the spring / damper forces added into spring[] / damper[] (LDS, nv)
__device__ __forceinline__ void tendon_passive(const mjw_model_t& m, const mjw_data_t& d, const float* qpos, const float* qvel,
                                               float* spring, float* damper, int wid, int lane) {
  for (int t = lane; t < m.ntendon; t += 64) d.ten_velocity[(long)wid * m.ntendon + t] = ten_vel(m, d, wid, qvel, t);
  const int dsbl_spring = m.opt_disableflags & DSBL_SPRING, dsbl_damper = m.opt_disableflags & DSBL_DAMPER;
  const float* stiff = MR(tendon_stiffness);
  const float* damp = MR(tendon_damping);
  const float* ls = MR(tendon_lengthspring);
  for (int t = 0; t < m.ntendon; t++) {
    const bool hs = stiff[t] != 0.0f && !dsbl_spring, hd = damp[t] != 0.0f && !dsbl_damper;
    if (!hs && !hd) continue;
    const float L = ten_len(m, d, wid, qpos, t), v = ten_vel(m, d, wid, qvel, t);
    const float lo = ls[2 * t], hi = ls[2 * t + 1];
    const float fs = L > hi ? stiff[t] * (hi - L) : (L < lo ? stiff[t] * (lo - L) : 0.0f);
    const float fd = -damp[t] * v;
    for (int k = lane; k < m.ten_J_rownnz[t]; k += 64) {
      const int dof = m.ten_J_colind[m.ten_J_rowadr[t] + k];
      const float J = ten_coef(m, d, wid, t, dof);
      if (hs) spring[dof] += J * fs;
      if (hd) damper[dof] += J * fd;
    }
    __syncthreads();
  }
}

// forward.py:739-779: scale the forces of the actuators on a force-limited tendon so that their sum
// stays in tendon_actfrcrange (force[]: this world's actuator forces in LDS)
__device__ __forceinline__ void tendon_actuator_clamp(const mjw_model_t& m, float* force, int wid, int lane) {
  const float* rng = MR(tendon_actfrcrange);
  for (int t = 0; t < m.ntendon; t++) {
    if (!m.tendon_actfrclimited[t]) continue;
    float tot = 0.0f;
    for (int a = 0; a < m.nu; a++)
      if (m.actuator_trntype[a] == 3 && m.actuator_trnid[2 * a] == t) tot += force[a];
    __syncthreads();
    for (int a = lane; a < m.nu; a += 64) {
      if (m.actuator_trntype[a] != 3 || m.actuator_trnid[2 * a] != t) continue;
      if (tot < rng[2 * t]) force[a] *= rng[2 * t] / tot;
      else if (tot > rng[2 * t + 1]) force[a] *= rng[2 * t + 1] / tot;
    }
    __syncthreads();
  }
}

}  // namespace mjw
