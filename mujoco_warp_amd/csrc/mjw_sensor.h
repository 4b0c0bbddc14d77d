// mjw_sensor.h -- sensor evaluation shared by the forward kernel (position / velocity sensors,
// mjw_step.hip) and the post-solve kernel (rne_postconstraint + acceleration sensors,
// mjw_sensor.hip).  Restates mujoco_warp/_src/sensor.py for the supported sensor types; the
// caller passes where each frame quantity lives (LDS in the forward kernel, HBM afterwards).
#pragma once

#include "mjw_common.h"
#include "mjw_narrow.h"
#include "mjw_ccd.h"

namespace mjw {

// per-world frame sources (each a per-world base pointer)
struct Frames {
  const float *xpos, *xquat, *xmat, *xipos, *ximat, *gxpos, *gxmat, *cxpos, *cxmat, *subtree_com, *cvel;
  const float* scc;  // convex / heightfield collision-sensor records' results (SCC_WORDS each, LDS), or null
};

// a lockstep-evaluated sensor record: count, then per point (dist, pos[3], normal[3]) x 4
constexpr int SCC_WORDS = 32;

// type-sorted pairs of collision_driver.py:43-77's CONVEX entries without heightfields (GJK / EPA)
__device__ __forceinline__ bool sensor_convex(int t1, int t2) {
  if (t1 == GEOM_PLANE || t1 == GEOM_HFIELD) return false;
  if (t2 == GEOM_MESH || t2 == GEOM_ELLIPSOID || t1 == GEOM_ELLIPSOID) return true;
  if (t2 == GEOM_CYLINDER) return t1 == GEOM_CAPSULE || t1 == GEOM_CYLINDER;
  return t2 == GEOM_BOX && (t1 == GEOM_CYLINDER || t1 == GEOM_BOX);
}

// site pose from the body pose (smooth.py:205-224, same operations as kinematics)
__device__ __forceinline__ void site_pose(const mjw_model_t& m, int wid, const Frames& F, int id, float* pos, float* mat) {
  const float* site_pos = MR(site_pos);
  const float* site_quat = MR(site_quat);
  int b = m.site_bodyid[id];
  float q[4] = {F.xquat[4 * b], F.xquat[4 * b + 1], F.xquat[4 * b + 2], F.xquat[4 * b + 3]};
  float t[3], sq[4];
  rot_vec_quat(t, site_pos + 3 * id, q);
  mul_quat(sq, q, site_quat + 4 * id);
  quat_to_mat(mat, sq);
  for (int i = 0; i < 3; i++) pos[i] = F.xpos[3 * b + i] + t[i];
}

// object frame position / rotation / body (sensor.py:282-340, 1011-1050)
__device__ __forceinline__ int obj_frame(const mjw_model_t& m, int wid, const Frames& F, int type, int id, float* pos, float* mat) {
  int body = 0;
  const float *p = nullptr, *R = nullptr;
  if (type == OBJ_BODY) { p = F.xipos + 3 * id; R = F.ximat + 9 * id; body = id; }
  else if (type == OBJ_XBODY) { p = F.xpos + 3 * id; R = F.xmat + 9 * id; body = id; }
  else if (type == OBJ_GEOM) { p = F.gxpos + 3 * id; R = F.gxmat + 9 * id; body = m.geom_bodyid[id]; }
  else if (type == OBJ_CAMERA) { p = F.cxpos + 3 * id; R = F.cxmat + 9 * id; body = m.cam_bodyid[id]; }
  if (type == OBJ_SITE) {
    site_pose(m, wid, F, id, pos, mat);
    return m.site_bodyid[id];
  }
  if (p) {
    for (int i = 0; i < 3; i++) pos[i] = p[i];
    for (int i = 0; i < 9; i++) mat[i] = R[i];
  } else {
    for (int i = 0; i < 3; i++) pos[i] = 0.0f;
    for (int i = 0; i < 9; i++) mat[i] = (i % 4 == 0) ? 1.0f : 0.0f;
  }
  return body;
}

__device__ __forceinline__ void mat_t_vec(float* r, const float* M, const float* v) {
  for (int i = 0; i < 3; i++) r[i] = M[i] * v[0] + M[3 + i] * v[1] + M[6 + i] * v[2];
}

// sensor.py:54-110 _write_scalar / _write_vector
__device__ __forceinline__ void sensor_write(const mjw_model_t& m, const mjw_data_t& d, int wid, int s, const float* v, int dim) {
  const float cutoff = MR(sensor_cutoff)[s];
  const int dt = m.sensor_datatype[s];
  float* out = d.sensordata + (long)wid * m.nsensordata + m.sensor_adr[s];
  for (int i = 0; i < dim; i++) {
    float x = v[i];
    const bool clip = cutoff > 0.0f && m.sensor_type[s] != SENS_GEOMFROMTO;  // sensor.py:69, 98
    if (clip && dt == DATATYPE_REAL) x = clampf(x, -cutoff, cutoff);
    else if (clip && dt == DATATYPE_POSITIVE) x = fminf(x, cutoff);
    out[i] = x;
  }
}

// sensor.py:394-446 _frame_quat
__device__ __forceinline__ void frame_quat(const mjw_model_t& m, int wid, const Frames& F, int type, int id, float* q) {
  q[0] = 1.0f; q[1] = q[2] = q[3] = 0.0f;
  const float* xq = F.xquat;
  if (type == OBJ_BODY) mul_quat(q, xq + 4 * id, MR(body_iquat) + 4 * id);
  else if (type == OBJ_XBODY) for (int i = 0; i < 4; i++) q[i] = xq[4 * id + i];
  else if (type == OBJ_GEOM) mul_quat(q, xq + 4 * m.geom_bodyid[id], MR(geom_quat) + 4 * id);
  else if (type == OBJ_SITE) mul_quat(q, xq + 4 * m.site_bodyid[id], MR(site_quat) + 4 * id);
  else if (type == OBJ_CAMERA) mul_quat(q, xq + 4 * m.cam_bodyid[id], MR(cam_quat) + 4 * id);
}

// sensor.py:1011-1050 _cvel_offset
__device__ __forceinline__ const float* cvel_offset(const mjw_model_t& m, int wid, const Frames& F, int type, int id, float* off) {
  float p[3], R[9];
  int b = obj_frame(m, wid, F, type, id, p, R);
  const float* com = F.subtree_com + 3 * m.body_rootid[b];
  for (int i = 0; i < 3; i++) off[i] = p[i] - com[i];
  return F.cvel + 6 * b;
}

// ---- ray-zone intersection of the touch sensor (ray.py:105-450, distances only) ---------------------------
__device__ __forceinline__ float ray_quad(float a, float b, float c, float* x) {
  float det = b * b - a * c;
  x[0] = x[1] = -1.0f;
  if (det < MJW_MINVAL) return -1.0f;
  det = sqrtf(det);
  const float den = 1.0f / (a != 0.0f ? a : MJW_MINVAL);
  x[0] = (-b - det) * den;
  x[1] = (-b + det) * den;
  return x[0] >= 0.0f ? x[0] : (x[1] >= 0.0f ? x[1] : -1.0f);
}

__device__ __forceinline__ float ray_sphere0(float r2, const float* p, const float* v) {
  float x[2];
  return ray_quad(dot3(v, v), dot3(v, p), dot3(p, p) - r2, x);
}

// the ray lp + t lv in the geom's frame against a sphere / capsule / ellipsoid / cylinder / box of `size`
__device__ float ray_geom_local(int type, const float* size, const float* lp, const float* lv) {
  float x[2];
  if (type == GEOM_SPHERE) return ray_sphere0(size[0] * size[0], lp, lv);
  if (type == GEOM_CAPSULE) {
    const float ssz = size[0] + size[1];
    if (ray_sphere0(ssz * ssz, lp, lv) < 0.0f) return -1.0f;
    const float sq = size[0] * size[0];
    float a = lv[0] * lv[0] + lv[1] * lv[1];
    float best = -1.0f;
    const float sol = ray_quad(a, lv[0] * lp[0] + lv[1] * lp[1], lp[0] * lp[0] + lp[1] * lp[1] - sq, x);
    if (sol >= 0.0f && fabsf(lp[2] + sol * lv[2]) <= size[1]) best = sol;
    a += lv[2] * lv[2];
    for (int side = 1; side >= -1; side -= 2) {
      const float ld[3] = {lp[0], lp[1], lp[2] - side * size[1]};
      ray_quad(a, dot3(lv, ld), dot3(ld, ld) - sq, x);
      for (int i = 0; i < 2; i++)
        if (x[i] >= 0.0f && (side > 0 ? lp[2] + x[i] * lv[2] >= size[1] : lp[2] + x[i] * lv[2] <= -size[1]) && (best < 0.0f || x[i] < best))
          best = x[i];
    }
    return best;
  }
  if (type == GEOM_ELLIPSOID) {
    float s[3], sv[3], sp[3];
    for (int i = 0; i < 3; i++) {
      const float q = size[i] * size[i];
      s[i] = 1.0f / (q != 0.0f ? q : MJW_MINVAL);
      sv[i] = s[i] * lv[i];
      sp[i] = s[i] * lp[i];
    }
    return ray_quad(dot3(sv, lv), dot3(sv, lp), dot3(sp, lp) - 1.0f, x);
  }
  if (type == GEOM_CYLINDER) {
    if (ray_sphere0(size[0] * size[0] + size[1] * size[1], lp, lv) < 0.0f) return -1.0f;
    float best = -1.0f;
    if (fabsf(lv[2]) > MJW_MINVAL)
      for (int side = -1; side <= 1; side += 2) {
        const float sol = (side * size[1] - lp[2]) / lv[2];
        const float p0 = lp[0] + sol * lv[0], p1 = lp[1] + sol * lv[1];
        if (sol >= 0.0f && p0 * p0 + p1 * p1 <= size[0] * size[0] && (best < 0.0f || sol < best)) best = sol;
      }
    const float sol = ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1], lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0], x);
    if (sol >= 0.0f && fabsf(lp[2] + sol * lv[2]) <= size[1] && (best < 0.0f || sol < best)) best = sol;
    return best;
  }
  if (type == GEOM_BOX) {
    if (ray_sphere0(dot3(size, size), lp, lv) < 0.0f) return -1.0f;
    float best = -1.0f;
    for (int i = 0; i < 3; i++) {
      if (fabsf(lv[i]) <= MJW_MINVAL) continue;
      const int i0 = i == 0 ? 1 : 0, i1 = i == 2 ? 1 : 2;
      for (int side = -1; side <= 1; side += 2) {
        const float sol = (side * size[i] - lp[i]) / lv[i];
        if (sol >= 0.0f && fabsf(lp[i0] + sol * lv[i0]) <= size[i0] && fabsf(lp[i1] + sol * lv[i1]) <= size[i1] && (best < 0.0f || sol < best))
          best = sol;
      }
    }
    return best;
  }
  return -1.0f;
}

// sensor.py:2001-2076 touch: normal forces of the site body's contacts whose ray along the contact normal
// (away from the body) meets the site's zone.  Contacts are visited at their first constraint row.
__device__ float touch_sensor(const mjw_model_t& m, const mjw_data_t& d, int wid, int site, const float* sxpos, const float* sxmat) {
  const int body = m.site_bodyid[site];
  const float* ssize = MR(site_size) + 3 * site;
  const int nefc = min(d.nefc[wid], d.njmax);
  const long wr = (long)wid * d.njmax;
  float total = 0.0f;
  for (int r = 0; r < nefc; r++) {
    const int type = d.efc_type[wr + r];
    if (type != CNSTR_CONTACT_FRICTIONLESS && type != CNSTR_CONTACT_PYRAMIDAL && type != CNSTR_CONTACT_ELLIPTIC) continue;
    const int cid = d.efc_id[wr + r];
    if (cid < 0 || cid >= d.naconmax || d.contact_efc_address[(long)cid * m.nmaxpyramid] != r) continue;
    const int g1 = d.contact_geom[2L * cid], g2 = d.contact_geom[2L * cid + 1];
    if (g1 < 0 || g2 < 0) continue;
    const int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
    if (body != b1 && body != b2) continue;
    float f = d.efc_force[wr + r];
    if (m.opt_cone == CONE_PYRAMIDAL)
      for (int i = 1; i < 2 * (d.contact_dim[cid] - 1); i++) {
        const int a = d.contact_efc_address[(long)cid * m.nmaxpyramid + i];
        if (a >= 0 && a < d.njmax) f += d.efc_force[wr + a];
      }
    if (f <= 0.0f) continue;
    const float* n = d.contact_frame + 9L * cid;
    const float nn = sqrtf(dot3(n, n)) * f;
    const float sg = body == b2 ? -1.0f : 1.0f;
    float dir[3], dif[3], lp[3], lv[3];
    for (int i = 0; i < 3; i++) {
      dir[i] = nn > 0.0f ? sg * n[i] * f / nn : 0.0f;
      dif[i] = d.contact_pos[3L * cid + i] - sxpos[i];
    }
    mat_t_vec(lp, sxmat, dif);
    mat_t_vec(lv, sxmat, dir);
    if (ray_geom_local(m.site_type[site], ssize, lp, lv) >= 0.0f) total += f;
  }
  return total;
}

// the efc row of the limit on joint / tendon `id` (sensor.py:243-278: any limit row with that id) or -1
__device__ __forceinline__ int limit_row(const mjw_data_t& d, int wid, int id) {
  const int lo = d.ne[wid] + d.nf[wid], hi = min(lo + d.nl[wid], d.njmax);
  const long wr = (long)wid * d.njmax;
  int r = -1;
  for (int e = lo; e < hi; e++)
    if (d.efc_id[wr + e] == id && (d.efc_type[wr + e] == CNSTR_LIMIT_JOINT || d.efc_type[wr + e] == CNSTR_LIMIT_TENDON)) r = e;
  return r;
}

// sensor.py:2700-2890 energy_pos: -sum m g . xipos over the bodies, joint and tendon springs
__device__ float energy_potential(const mjw_model_t& m, const mjw_data_t& d, int wid, const float* qpos, const float* xipos) {
  float e = 0.0f;
  const float* grav = MR(opt_gravity);
  const float* mass = MR(body_mass);
  if (!(m.opt_disableflags & DSBL_GRAVITY))
    for (int b = 1; b < m.nbody; b++) e -= mass[b] * dot3(grav, xipos + 3 * b);
  if (m.opt_disableflags & DSBL_SPRING) return e;
  const float* stiff = MR(jnt_stiffness);
  const float* qs = MR(qpos_spring);
  for (int j = 0; j < m.njnt; j++) {
    const float k = stiff[j];
    if (k == 0.0f) continue;
    const int a = m.jnt_qposadr[j], t = m.jnt_type[j];
    if (t == JNT_FREE || t == JNT_BALL) {
      float lin = 0.0f;
      int q0 = a;
      if (t == JNT_FREE) {
        for (int i = 0; i < 3; i++) lin += (qpos[a + i] - qs[a + i]) * (qpos[a + i] - qs[a + i]);
        q0 = a + 3;
      }
      float q[4] = {qpos[q0], qpos[q0 + 1], qpos[q0 + 2], qpos[q0 + 3]}, dif[3];
      normalize4(q);
      quat_sub(dif, q, qs + q0);
      e += 0.5f * k * (lin + dot3(dif, dif));
    } else {
      const float dq = qpos[a] - qs[a];
      e += 0.5f * k * dq * dq;
    }
  }
  const float* tst = MR(tendon_stiffness);
  const float* tls = MR(tendon_lengthspring);
  for (int t = 0; t < m.ntendon; t++) {
    if (tst[t] == 0.0f) continue;
    const float L = d.ten_length[(long)wid * m.ntendon + t], lo = tls[2 * t], hi = tls[2 * t + 1];
    const float disp = L > hi ? hi - L : (L < lo ? lo - L : 0.0f);
    e += 0.5f * tst[t] * disp * disp;
  }
  return e;
}

// sensor.py:2893-2940 energy_vel: 0.5 qvel' M qvel (dense qM rows of nv_pad, or the sparse ancestor rows)
__device__ float energy_kinetic(const mjw_model_t& m, const mjw_data_t& d, int wid, const float* qvel) {
  float e = 0.0f;
  if (m.is_sparse) {
    const float* M = d.qM + (long)wid * m.nM;
    for (int i = 0; i < m.nv; i++)
      for (int k = 0; k < m.M_rownnz[i]; k++) {
        const int j = m.M_colind[m.M_rowadr[i] + k];
        e += (j == i ? 1.0f : 2.0f) * qvel[i] * M[m.M_rowadr[i] + k] * qvel[j];
      }
  } else {
    const int np = m.nv_pad;
    const float* M = d.qM + (long)wid * np * np;
    for (int i = 0; i < m.nv; i++) {
      float row = 0.0f;
      for (int j = 0; j < m.nv; j++) row += M[i * np + j] * qvel[j];
      e += qvel[i] * row;
    }
  }
  return 0.5f * e;
}

// smooth.py:2932-3084 subtree_vel, by one lane (sensor models only): subtree linear velocity and angular
// momentum into the Data, children before parents (bodies are in DFS pre-order)
__device__ void subtree_vel(const mjw_model_t& m, const mjw_data_t& d, int wid, const float* cvel, const float* com) {
  const long wb = (long)wid * m.nbody;
  float* lv = d.subtree_linvel + wb * 3;
  float* am = d.subtree_angmom + wb * 3;
  const float* xipos = d.xipos + wb * 3;
  const float* ximat = d.ximat + wb * 9;
  const float* mass = MR(body_mass);
  const float* smass = MR(body_subtreemass);
  const float* inertia = MR(body_inertia);
  for (int b = 0; b < m.nbody; b++) {
    const float* cv = cvel + 6 * b;
    const float* sc = com + 3 * m.body_rootid[b];
    float dif[3], c[3], dv[3];
    for (int i = 0; i < 3; i++) dif[i] = xipos[3 * b + i] - sc[i];
    cross3(c, dif, cv);
    for (int i = 0; i < 3; i++) lv[3 * b + i] = mass[b] * (cv[3 + i] - c[i]);
    mat_t_vec(dv, ximat + 9 * b, cv);
    for (int i = 0; i < 3; i++) dv[i] *= inertia[3 * b + i];
    matvec3(am + 3 * b, ximat + 9 * b, dv);
  }
  for (int b = m.nbody - 1; b >= 0; b--) {
    if (b > 0)
      for (int i = 0; i < 3; i++) lv[3 * m.body_parentid[b] + i] += lv[3 * b + i];
    const float sm = fmaxf(MJW_MINVAL, smass[b]);
    for (int i = 0; i < 3; i++) lv[3 * b + i] /= sm;
  }
  for (int b = m.nbody - 1; b > 0; b--) {
    const int p = m.body_parentid[b];
    const float* cv = cvel + 6 * b;
    const float* sc = com + 3 * m.body_rootid[b];
    float dif[3], c[3], dx[3], dp[3], dL[3];
    for (int i = 0; i < 3; i++) dif[i] = xipos[3 * b + i] - sc[i];
    cross3(c, dif, cv);
    for (int i = 0; i < 3; i++) {
      dx[i] = xipos[3 * b + i] - com[3 * b + i];
      dp[i] = (cv[3 + i] - c[i] - lv[3 * b + i]) * mass[b];
    }
    cross3(dL, dx, dp);
    for (int i = 0; i < 3; i++) am[3 * b + i] += dL[i];
    for (int i = 0; i < 3; i++) am[3 * p + i] += am[3 * b + i];
    for (int i = 0; i < 3; i++) {
      dx[i] = com[3 * b + i] - com[3 * p + i];
      dp[i] = (lv[3 * b + i] - lv[3 * p + i]) * smass[b];
    }
    cross3(dL, dx, dp);
    for (int i = 0; i < 3; i++) am[3 * p + i] += dL[i];
  }
}

// ---- collision sensors (sensor.py:604-680, 710-757): the smallest-distance contact over a sensor's geom
// pairs, each pair's contacts from the primitive narrowphase (collision_primitive.py) -----------------
struct CollBest {
  float dist;
  float p1[3], p2[3];
  bool flip;
};

// sensor.py:744-757 (_sensor_collision): contact points pos -+ dist / 2 along the normal
__device__ __forceinline__ void coll_offer(CollBest& b, float dist, const float* pos, const float* nrm, bool flip) {
  if (!(dist < b.dist)) return;
  b.dist = dist;
  b.flip = flip;
  for (int i = 0; i < 3; i++) {
    b.p1[i] = pos[i] - 0.5f * dist * nrm[i];
    b.p2[i] = pos[i] + 0.5f * dist * nrm[i];
  }
}

// every contact collision_primitive.py writes for the type-sorted pair (g1, g2) -- inside or outside the
// margin, as write_contact keeps sensor contacts (collision_core.py:199-213) -- offered to b
// (record e: convex pairs read the result the wave computed in lockstep, sensor_convex_records)
__device__ void coll_pair(const mjw_model_t& m, int wid, const Frames& F, int g1, int g2, int pairid, bool flip, CollBest& b, int e) {
  const float* geom_size = MR(geom_size);
  const float* gmargin = MR(geom_margin);
  const float margin = pairid > -1 ? MR(pair_margin)[pairid] : gmargin[g1] + gmargin[g2];
  const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  if (sensor_convex(t1, t2) || t1 == GEOM_HFIELD) {
    const float* q = F.scc + SCC_WORDS * e;
    for (int i = 0; i < (int)q[0]; i++) coll_offer(b, q[1 + 7 * i], q + 2 + 7 * i, q + 5 + 7 * i, flip);
    return;
  }
  const float* p1 = F.gxpos + 3 * g1;
  const float* p2 = F.gxpos + 3 * g2;
  const float* r1 = F.gxmat + 9 * g1;
  const float* r2 = F.gxmat + 9 * g2;
  const float* s1 = geom_size + 3 * g1;
  const float* s2 = geom_size + 3 * g2;
  const float n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]};
  float pos[3], nrm[3];
  if (t1 == GEOM_PLANE && t2 == GEOM_BOX) {  // collision_primitive.py:737-790: all 8 corners
    for (int k = 0; k < 8; k++) {
      const float dist = plane_box_corner(k, n1, p1, p2, r2, s2, pos);
      coll_offer(b, dist, pos, n1, flip);
    }
    return;
  }
  if (t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) {  // collision_primitive.py:964-1040: 4 candidates
    for (int k = 0; k < 4; k++) {
      float dist;
      plane_cylinder_k(k, n1, p1, p2, n2, s2[0], s2[1], &dist, pos);
      coll_offer(b, dist, pos, n1, flip);
    }
    return;
  }
  Con2 c;
  c.n = 0;
  if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) {
    c.dist[0] = plane_sphere(c.pos[0], n1, p1, p2, s2[0]);
    make_frame(c.frame[0], n1);
    c.n = 1;
  } else if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
    plane_capsule(c, n1, p1, p2, n2, s2[0], s2[1]);
  } else if (t1 == GEOM_PLANE && t2 == GEOM_ELLIPSOID) {
    c.dist[0] = plane_ellipsoid(c.pos[0], n1, p1, p2, r2, s2);
    make_frame(c.frame[0], n1);
    c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) {
    c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], p2, s2[0]);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
    float a[3], bb[3], pt[3];
    for (int i = 0; i < 3; i++) { a[i] = p2[i] - n2[i] * s2[1]; bb[i] = p2[i] + n2[i] * s2[1]; }
    closest_segment_point(pt, a, bb, p1);
    c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], pt, s2[0]);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER) {
    c.dist[0] = sphere_cylinder(c.pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_BOX) {
    c.dist[0] = sphere_box(c.pos[0], nrm, p1, s1[0], p2, r2, s2);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
    capsule_capsule(c, p1, n1, s1[0], s1[1], p2, n2, s2[0], s2[1], margin);
  } else if (t1 == GEOM_CAPSULE && t2 == GEOM_BOX) {
    capsule_box(c, p1, n1, s1[0], s1[1], p2, r2, s2);
  }
  for (int i = 0; i < c.n && i < 2; i++) coll_offer(b, c.dist[i], c.pos[i], c.frame[i], flip);
}

// collision_convex.py:763-852 for collision-sensor pairs (pairid[1] >= 0): GJK / EPA with an unbounded
// cutoff (1e32), so separated pairs report their distance too; dist += margin; the first witness pair's
// midpoint and the flipped frame's normal (frame *= -1, :849-852).  The whole wave runs each convex record
// of the position-stage collision sensors in lockstep over the LDS workspace W (mjw_ccd.h) and stores
// (count, dist, pos[3], normal[3]) at out + SCC_WORDS * record.  Heightfield records run the heightfield
// routine (collision_convex.py:158-697: every kept prism contact, frames unflipped) with their contacts'
// margins.  Separate from the lane-per-sensor loop.
__device__ void sensor_convex_records(const mjw_model_t& m, const Frames& F, int wid, float* W, float* out) {
  const float* gsize = MR(geom_size);
  const float* gmargin = MR(geom_margin);
  const float* mesh_vert = MR(mesh_vert);
  const CcdLay CL = ccd_layout(m.ccd_epa_iterations, m.nhfield > 0, m.nmaxpolygon, m.nmaxmeshdeg);
  const MeshPoly MP = mesh_poly(m);
  const int lane = (int)(threadIdx.x & 63);
  for (int k = 0; k < m.nsensor; k++) {
    const int t = m.sensor_type[k];
    if (t != SENS_GEOMDIST && t != SENS_GEOMNORMAL && t != SENS_GEOMFROMTO) continue;
    const int adr = m.sensor_collision_adr[k];
    for (int e = adr; e < adr + m.sensor_collision_num[k]; e++) {
      const int* r = m.sensor_collision_pair + 4 * e;
      const int g1 = r[0], g2 = r[1], t1 = m.geom_type[g1], t2 = m.geom_type[g2];
      if (!sensor_convex(t1, t2) && t1 != GEOM_HFIELD) continue;
      const int md1 = t1 == GEOM_MESH ? m.geom_dataid[g1] : -1, md2 = t2 == GEOM_MESH ? m.geom_dataid[g2] : -1;
      const float margin = r[2] > -1 ? MR(pair_margin)[r[2]] : gmargin[g1] + gmargin[g2];
      if (t1 == GEOM_HFIELD) {
        const int hid = m.geom_dataid[g1];
        CcdWS cw;
        cw.W = W;
        cw.L = CL;
        const int n = hfield_pair(cw, m.ccd_epa_iterations, MR(opt_ccd_tolerance)[0], m.opt_ccd_iterations, gmargin[g1] + gmargin[g2],
                                  margin, F.gxpos + 3 * g1, F.gxmat + 9 * g1, MR(hfield_size) + 4 * hid, m.hfield_nrow[hid],
                                  m.hfield_ncol[hid], MR(hfield_data) + m.hfield_adr[hid], F.gxpos + 3 * g2, F.gxmat + 9 * g2,
                                  gsize + 3 * g2, MR(geom_rbound)[g2], t2, md2 >= 0 ? mesh_vert + 3 * (long)m.mesh_vertadr[md2] : nullptr,
                                  md2 >= 0 ? m.mesh_vertnum[md2] : 0, W + CL.out);
        if (lane == 0) {
          const float* o = W + CL.out;
          float* q = out + SCC_WORDS * e;
          q[0] = (float)n;
          for (int i = 0; i < n; i++) {
            q[1 + 7 * i] = o[4 + 4 * i];
            for (int k = 0; k < 3; k++) { q[2 + 7 * i + k] = o[5 + 4 * i + k]; q[5 + 7 * i + k] = o[20 + 3 * i + k]; }
          }
        }
        __syncthreads();
        continue;
      }
      put_cgeom(W + CL.geoms, F.gxpos + 3 * g1, F.gxmat + 9 * g1, gsize + 3 * g1, t1, md1 >= 0 ? m.mesh_vertadr[md1] : 0,
                md1 >= 0 ? m.mesh_vertnum[md1] : 0, md1);
      put_cgeom(W + CL.geoms + CGEOM_WORDS, F.gxpos + 3 * g2, F.gxmat + 9 * g2, gsize + 3 * g2, t2, md2 >= 0 ? m.mesh_vertadr[md2] : 0,
                md2 >= 0 ? m.mesh_vertnum[md2] : 0, md2);
      __syncthreads();
      const int nc = ccd_pair(W, m.ccd_epa_iterations, MR(opt_ccd_tolerance)[0], m.opt_ccd_iterations, margin, mesh_vert, 1.0e32f, &MP,
                              (m.opt_enableflags & ENBL_MULTICCD) != 0, m.nmaxpolygon, m.nmaxmeshdeg);
      if (lane == 0) {
        const float* o = W + CL.out;
        float nrm[3] = {o[1], o[2], o[3]};
        normalize3(nrm);
        float* q = out + SCC_WORDS * e;
        q[0] = nc > 0 ? 1.0f : 0.0f;
        q[1] = o[0];
        for (int i = 0; i < 3; i++) { q[2 + i] = o[4 + i]; q[5 + i] = -nrm[i]; }
      }
      __syncthreads();
    }
  }
}

// sensor.py:604-680: GEOMDIST (dim 1), GEOMNORMAL (3) or GEOMFROMTO (6) of sensor s
__device__ void collision_sensor(const mjw_model_t& m, const mjw_data_t& d, int wid, const Frames& F, int s) {
  const int t = m.sensor_type[s];
  const float cutoff = MR(sensor_cutoff)[s];
  CollBest b;
  b.dist = cutoff;
  b.flip = false;
  for (int i = 0; i < 3; i++) b.p1[i] = b.p2[i] = 0.0f;
  const int adr = m.sensor_collision_adr[s];
  for (int e = 0; e < m.sensor_collision_num[s]; e++) {
    const int* r = m.sensor_collision_pair + 4 * (adr + e);
    coll_pair(m, wid, F, r[0], r[1], r[2], r[3] != 0, b, adr + e);
  }
  float v[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  int dim = 1;
  if (t == SENS_GEOMDIST) {
    v[0] = b.dist;
  } else if (t == SENS_GEOMNORMAL) {
    dim = 3;
    if (b.dist <= cutoff) {
      float nn[3] = {b.p2[0] - b.p1[0], b.p2[1] - b.p1[1], b.p2[2] - b.p1[2]};
      normalize3(nn);
      for (int i = 0; i < 3; i++) v[i] = b.flip ? -nn[i] : nn[i];
    }
  } else {
    dim = 6;
    if (b.dist <= cutoff)
      for (int i = 0; i < 3; i++) {
        v[i] = b.flip ? b.p2[i] : b.p1[i];
        v[3 + i] = b.flip ? b.p1[i] : b.p2[i];
      }
  }
  sensor_write(m, d, wid, s, v, dim);
}

// util_misc.py:603-632 inside_geom
__device__ __forceinline__ bool inside_geom(const float* pos, const float* mat, const float* size, int type, const float* pt) {
  const float vec[3] = {pt[0] - pos[0], pt[1] - pos[1], pt[2] - pos[2]};
  if (type == GEOM_SPHERE) return dot3(vec, vec) < size[0] * size[0];
  float pl[3];
  mat_t_vec(pl, mat, vec);
  if (type == GEOM_CAPSULE) {
    const float z = pl[2], zd = z - clampf(z, -size[1], size[1]);
    return pl[0] * pl[0] + pl[1] * pl[1] + zd * zd < size[0] * size[0];
  }
  if (type == GEOM_ELLIPSOID) {
    const float q[3] = {pl[0] / size[0], pl[1] / size[1], pl[2] / size[2]};
    return dot3(q, q) < 1.0f;
  }
  if (type == GEOM_CYLINDER) return fabsf(pl[2]) < size[1] && pl[0] * pl[0] + pl[1] * pl[1] < size[0] * size[0];
  if (type == GEOM_BOX) return fabsf(pl[0]) < size[0] && fabsf(pl[1]) < size[1] && fabsf(pl[2]) < size[2];
  if (type == GEOM_PLANE) return pl[2] < 0.0f;
  return false;
}

// ---- contact sensor (sensor.py:1750-1940 output, 2275-2430 matching) ---------------------------------
// support.py:241-308 contact_force_fn: the contact's 6D force in its own frame (pyramid decoded)
__device__ void contact_force_local(const mjw_model_t& m, const mjw_data_t& d, int wid, int cid, float* f) {
  for (int i = 0; i < 6; i++) f[i] = 0.0f;
  const int condim = d.contact_dim[cid];
  const int adr = d.contact_efc_address[(long)cid * m.nmaxpyramid];
  if (adr < 0) return;
  const float* ef = d.efc_force + (long)wid * d.njmax;
  if (m.opt_cone == CONE_PYRAMIDAL) {
    if (condim == 1) { f[0] = ef[adr]; return; }
    const float* mu = d.contact_friction + 5L * cid;
    for (int i = 0; i < condim - 1; i++) {
      const int a = 2 * i + adr;
      const float d1 = a < d.njmax ? ef[a] : 0.0f, d2 = a + 1 < d.njmax ? ef[a + 1] : 0.0f;
      f[0] += d1 + d2;
      f[i + 1] = (d1 - d2) * mu[i];
    }
  } else {
    for (int i = 0; i < condim; i++) {
      const int a = d.contact_efc_address[(long)cid * m.nmaxpyramid + i];
      if (a >= 0 && a < d.njmax) f[i] = ef[a];
    }
  }
}

// sensor.py:2258-2272 _check_match (XBODY: the contact body's ancestors, i.e. the subtree of objid)
__device__ __forceinline__ bool contact_obj_match(const mjw_model_t& m, int body, int geom, int type, int id) {
  if (type == OBJ_UNKNOWN || type == OBJ_SITE) return true;  // no object / the site zone was tested already
  if (type == OBJ_GEOM) return id == geom;
  if (type == OBJ_BODY) return id == body;
  if (type == OBJ_XBODY) {
    while (body > id) body = m.body_parentid[body];
    return body == id;
  }
  return false;
}

// the world's slot range of the contact pool, [k0, k1): ncon_world (first slot, span), filled by the pool_ranges
// launch before the sensor kernel on the dense path (sensor_launch) and by the collision kernel on the sparse
// path.  The world's contacts are the slots of the range whose worldid is wid, in pool (= narrowphase) order;
// other worlds' slots can interleave when a world staged its contacts over several rounds.
__device__ __forceinline__ void world_pool_range(const mjw_data_t& d, int wid, int& k0, int& k1) {
  k0 = d.ncon_world[2L * wid];
  k1 = min(min(d.nacon[0], d.naconmax), k0 + d.ncon_world[2L * wid + 1]);
}
// contact k of the pool is a constraint contact of world wid (sensor.py:2313-2316: the contact sensor keeps
// every CONSTRAINT-typed contact, with rows or not; contact_force_local gives zero force without rows)
__device__ __forceinline__ bool world_constraint_contact(const mjw_data_t& d, int wid, int k) {
  return d.contact_worldid[k] == wid && (d.contact_type[k] & 1);
}

// sensor.py:2085-2118 _preprocess_tactile_contacts for one weld body: the partner geoms of the world's
// contacts on weld body pw -- geom2 for a contact whose geom1 is on it, then geom1 for one whose geom2 is --
// in pool order, the first MJ_MAXCONPAIR (50) kept in `list` (LDS); every contact of the pool counts,
// sensor-only ones included.  Whole wave, lane = contact; returns the count kept.
__device__ int tactile_partners(const mjw_model_t& m, const mjw_data_t& d, int wid, int pw, int* list, int lane) {
  int k0, k1;
  world_pool_range(d, wid, k0, k1);
  int cnt = 0;
  for (int base = k0; base < k1 && cnt < 50; base += 64) {
    const int k = base + lane;
    int ga = -1, gb = -1;
    if (k < k1 && d.contact_worldid[k] == wid) {
      const int g1 = d.contact_geom[2L * k], g2 = d.contact_geom[2L * k + 1];
      if (g1 >= 0 && g2 >= 0) {
        if (m.body_weldid[m.geom_bodyid[g1]] == pw) ga = g2;
        if (m.body_weldid[m.geom_bodyid[g2]] == pw) gb = g1;
      }
    }
    const int n = (ga >= 0) + (gb >= 0);
    int incl = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    int pos = cnt + incl - n;
    if (ga >= 0) {
      if (pos < 50) list[pos] = ga;
      pos++;
    }
    if (gb >= 0 && pos < 50) list[pos] = gb;
    cnt += __shfl(incl, 63, 64);
  }
  __syncthreads();
  return min(cnt, 50);
}

// collision_sdf.py:157-183, 393-400: primitive signed distances in the geom frame (box: radial field inside);
// other geom types have none here (0: no pressure)
__device__ __forceinline__ float tactile_sdf(int type, const float* p, const float* size) {
  if (type == GEOM_PLANE) return p[2];
  if (type == GEOM_SPHERE) return sqrtf(dot3(p, p)) - size[0];
  if (type == GEOM_BOX) {
    float a[3];
    for (int i = 0; i < 3; i++) a[i] = fabsf(p[i]) - size[i];
    if (a[0] >= 0.0f || a[1] >= 0.0f || a[2] >= 0.0f) {
      const float b0 = fmaxf(a[0], 0.0f), b1 = fmaxf(a[1], 0.0f), b2 = fmaxf(a[2], 0.0f);
      return sqrtf(b0 * b0 + b1 * b1 + b2 * b2) + fminf(fmaxf(fmaxf(a[0], a[1]), a[2]), 0.0f);
    }
    float f[3];
    for (int i = 0; i < 3; i++) f[i] = -size[i] / a[i];
    const float fn = sqrtf(dot3(f, f));
    float tmin = MJW_MAXVAL;
    for (int i = 0; i < 3; i++) tmin = fminf(tmin, -a[i] / fabsf(f[i] / fn));
    return -tmin;
  }
  if (type == GEOM_ELLIPSOID) {
    float sp[3], s2[3];
    for (int i = 0; i < 3; i++) { sp[i] = p[i] / size[i]; s2[i] = p[i] / (size[i] * size[i]); }
    const float k0 = sqrtf(dot3(sp, sp)), k1 = sqrtf(dot3(s2, s2));
    return k0 * (k0 - 1.0f) / (k1 != 0.0f ? k1 : 1e-12f);
  }
  return 0.0f;
}

// sensor.py:2121-2252 tactile, one sensor by the whole wave (lane = taxel): each vertex of the sensor's
// mesh, placed with the sensor geom's pose, takes pressure depth / max(0.05 - depth, MINVAL) from every
// distinct geom among the first MJ_MAXCONPAIR (50) contact partners of the sensor geom's weld body at which
// the SDF is negative.  The partner list (tactile_partners, LDS `list`) is built once per sensor and world
// in pool order (the reference's atomic order is arbitrary).  Layout [normal (nvt), tangent 1 (nvt),
// tangent 2 (nvt)]; the tangential slip terms need per-vertex tangent frames, which the compiler's meshes
// do not have (mesh_normalnum = vertnum), so they are 0.
__device__ void tactile_sensor(const mjw_model_t& m, const mjw_data_t& d, int wid, const Frames& F, int s, int lane, int* list) {
  const int mesh = m.sensor_objid[s], geom = m.sensor_refid[s];
  const int nvt = m.mesh_vertnum[mesh];
  float* out = d.sensordata + (long)wid * m.nsensordata + m.sensor_adr[s];
  const int pw = m.body_weldid[m.geom_bodyid[geom]];
  const int npart = tactile_partners(m, d, wid, pw, list, lane);
  const float* gx = F.gxpos + 3 * geom;
  const float* gm = F.gxmat + 9 * geom;
  const float* vert = MR(mesh_vert) + 3 * (long)m.mesh_vertadr[mesh];
  const float* nrm0 = MR(mesh_normal) + 3 * (long)m.mesh_normaladr[mesh];
  const float* gsize = MR(geom_size);
  for (int v = lane; v < nvt; v += 64) {
    float x[3];
    for (int i = 0; i < 3; i++) x[i] = gm[3 * i] * vert[3 * v] + gm[3 * i + 1] * vert[3 * v + 1] + gm[3 * i + 2] * vert[3 * v + 2] + gx[i];
    const float* nrm = nrm0 + 3 * v;
    const float nn = dot3(nrm, nrm);
    float total = 0.0f;
    for (int p = 0; p < npart; p++) {
      const int g = list[p];
      bool dup = false;
      for (int p2 = 0; p2 < p && !dup; p2++) dup = list[p2] == g;
      if (dup) continue;
      const float* px = F.gxpos + 3 * g;
      const float* pm = F.gxmat + 9 * g;
      float dx[3], q[3];
      for (int i = 0; i < 3; i++) dx[i] = x[i] - px[i];
      mat_t_vec(q, pm, dx);
      const float depth = fminf(tactile_sdf(m.geom_type[g], q, gsize + 3 * g), 0.0f);
      if (depth >= 0.0f) continue;
      total += depth / fmaxf(0.05f - depth, MJW_MINVAL) * nn;
    }
    out[v] = total;
    out[nvt + v] = 0.0f;
    out[2 * nvt + v] = 0.0f;
  }
}

// sensor.py:2330-2375: does contact cid match sensor s, and in which direction (+-1; 0: no match)
__device__ float contact_match(const mjw_model_t& m, const mjw_data_t& d, int wid, const Frames& F, int s, int cid) {
  const int ot = m.sensor_objtype[s], oid = m.sensor_objid[s], rt = m.sensor_reftype[s], rid = m.sensor_refid[s];
  if (ot == OBJ_SITE) {
    float sp[3], sR[9];
    site_pose(m, wid, F, oid, sp, sR);
    if (!inside_geom(sp, sR, MR(site_size) + 3 * oid, m.site_type[oid], d.contact_pos + 3L * cid)) return 0.0f;
  }
  if (ot == OBJ_UNKNOWN && rt == OBJ_UNKNOWN) return 1.0f;
  const int g1 = d.contact_geom[2L * cid], g2 = d.contact_geom[2L * cid + 1];
  const int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
  const bool m11 = contact_obj_match(m, b1, g1, ot, oid), m12 = contact_obj_match(m, b2, g2, ot, oid);
  const bool m21 = contact_obj_match(m, b1, g1, rt, rid), m22 = contact_obj_match(m, b2, g2, rt, rid);
  if (!m11 && !m12) return 0.0f;
  if (!m21 && !m22) return 0.0f;
  if (ot != OBJ_UNKNOWN && rt != OBJ_UNKNOWN) {
    const bool reg = m11 && m22, rev = m12 && m21;
    if (!reg && !rev) return 0.0f;
    return (rev && !reg) ? -1.0f : 1.0f;
  }
  if (ot != OBJ_UNKNOWN) return m11 ? 1.0f : -1.0f;
  return m22 ? 1.0f : -1.0f;
}

// one contact sensor of world wid by the calling lane.  Matches are taken in the world's contact order (as
// MuJoCo's mj_sensorAcc does; the reference's atomic match order is arbitrary), at most opt
// contact_sensor_maxmatch of them; reduce mindist / maxforce pick the `num` smallest criteria (ties by that
// order, a stable sort) by repeated selection, netforce sums them about the force-weighted centroid
__device__ void contact_sensor(const mjw_model_t& m, const mjw_data_t& d, int wid, const Frames& F, int s) {
  const int spec = m.sensor_intprm[3 * s], reduce = m.sensor_intprm[3 * s + 1];
  int size = 0;
  const int fsz[7] = {1, 3, 3, 1, 3, 3, 3};
  for (int i = 0; i < 7; i++)
    if (spec & (1 << i)) size += fsz[i];
  if (size == 0) return;
  const int dim = m.sensor_dim[s], num = dim / size;
  float* out = d.sensordata + (long)wid * m.nsensordata + m.sensor_adr[s];
  int k0, k1;
  world_pool_range(d, wid, k0, k1);
  const int maxmatch = m.opt_contact_sensor_maxmatch;
  auto criteria = [&](int cid) -> float {
    if (reduce == 1) return d.contact_dist[cid];
    float f[6];
    contact_force_local(m, d, wid, cid, f);
    return -(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
  };
  // pass 1: the match count (all matches: `found`) and, for netforce, the sums
  int nmatch = 0;
  float np[3] = {0, 0, 0}, nf[3] = {0, 0, 0}, nt[3] = {0, 0, 0}, wsum = 0.0f;
  for (int cid = k0; cid < k1; cid++) {
    if (!world_constraint_contact(d, wid, cid)) continue;
    const float dir = contact_match(m, d, wid, F, s, cid);
    if (dir == 0.0f) continue;
    const int k = nmatch++;
    if (reduce != 3 || k >= maxmatch) continue;
    float f[6];
    contact_force_local(m, d, wid, cid, f);
    const float w = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    const float* cp = d.contact_pos + 3L * cid;
    const float* fr = d.contact_frame + 9L * cid;
    for (int i = 0; i < 3; i++) np[i] += w * cp[i];
    wsum += w;
    float fg[3], tg[3], c[3];
    for (int i = 0; i < 3; i++) {
      fg[i] = dir * (fr[i] * f[0] + fr[3 + i] * f[1] + fr[6 + i] * f[2]);  // frame^T @ (dir f)
      tg[i] = dir * (fr[i] * f[3] + fr[3 + i] * f[4] + fr[6 + i] * f[5]);
    }
    cross3(c, cp, fg);
    for (int i = 0; i < 3; i++) { nf[i] += fg[i]; nt[i] += tg[i] + c[i]; }
  }
  if (reduce == 3) {
    float c[3];
    for (int i = 0; i < 3; i++) np[i] /= fmaxf(wsum, MJW_MINVAL);
    cross3(c, np, nf);
    for (int i = 0; i < 3; i++) nt[i] -= c[i];
    int a = 0;
    if (spec & 1) out[a++] = (float)nmatch;
    if (spec & 2) for (int i = 0; i < 3; i++) out[a++] = nf[i];
    if (spec & 4) for (int i = 0; i < 3; i++) out[a++] = nt[i];
    if (spec & 8) out[a++] = 0.0f;
    if (spec & 16) for (int i = 0; i < 3; i++) out[a++] = np[i];
    if (spec & 32) { out[a++] = 1.0f; out[a++] = 0.0f; out[a++] = 0.0f; }
    if (spec & 64) { out[a++] = 0.0f; out[a++] = 1.0f; out[a++] = 0.0f; }
    return;
  }
  const int nslots = min(min(nmatch, maxmatch), num);
  float last_c = -MJW_MAXVAL;
  int last_k = -1;
  for (int i = 0; i < nslots; i++) {
    // slot i: the i-th match in order (none) or the next (criteria, order) after the previous slot's
    int cid = -1, k = 0, best_k = -1;
    float dir = 0.0f, best_c = MJW_MAXVAL;
    for (int c_ = k0; c_ < k1 && k < maxmatch; c_++) {
      if (!world_constraint_contact(d, wid, c_)) continue;
      const float dr = contact_match(m, d, wid, F, s, c_);
      if (dr == 0.0f) continue;
      if (reduce == 0) {
        if (k == i) { cid = c_; dir = dr; break; }
      } else {
        const float cr = criteria(c_);
        const bool after = cr > last_c || (cr == last_c && k > last_k);
        if (after && (cr < best_c || best_k < 0)) { best_c = cr; best_k = k; cid = c_; dir = dr; }
      }
      k++;
    }
    if (reduce != 0) { last_c = best_c; last_k = best_k; }
    if (cid < 0) break;
    float* o = out + i * size;
    int a = 0;
    float f[6] = {0, 0, 0, 0, 0, 0};
    if (spec & 6) contact_force_local(m, d, wid, cid, f);
    const float* fr = d.contact_frame + 9L * cid;
    if (spec & 1) o[a++] = (float)nmatch;
    if (spec & 2) { o[a++] = f[0]; o[a++] = f[1]; o[a++] = dir * f[2]; }
    if (spec & 4) { o[a++] = f[3]; o[a++] = f[4]; o[a++] = dir * f[5]; }
    if (spec & 8) o[a++] = d.contact_dist[cid];
    if (spec & 16) for (int j = 0; j < 3; j++) o[a++] = d.contact_pos[3L * cid + j];
    if (spec & 32) for (int j = 0; j < 3; j++) o[a++] = dir * fr[j];
    if (spec & 64) for (int j = 0; j < 3; j++) o[a++] = dir * fr[3 + j];
  }
  for (int i = max(nslots, 0); i < num; i++)
    for (int j = 0; j < size; j++) out[i * size + j] = 0.0f;
}

// one position- or velocity-stage sensor (sensor.py:459-706 / 1251-1373, supported types); COLL: with the
// collision sensors (their narrowphase is compiled into the models' kernel that has them only)
template <bool COLL>
__device__ void sensor_posvel_one(const mjw_model_t& m, const mjw_data_t& d, int wid, const Frames& F, int s, const float* qpos,
                                  const float* qvel, const float* act_len, const float* act_vel, float time) {
  const int t = m.sensor_type[s], id = m.sensor_objid[s], ot = m.sensor_objtype[s];
  const int rid = m.sensor_refid[s], rt = m.sensor_reftype[s];
  float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int dim = 3;
  if (t == SENS_MAGNETOMETER) {  // sensor.py:114-125
    float p[3], R[9];
    site_pose(m, wid, F, id, p, R);
    mat_t_vec(v, R, MR(opt_magnetic));
  } else if (t == SENS_JOINTPOS) {
    v[0] = qpos[m.jnt_qposadr[id]]; dim = 1;
  } else if (t == SENS_ACTUATORPOS) {
    v[0] = act_len[id]; dim = 1;
  } else if (t == SENS_BALLQUAT) {  // sensor.py:232-240
    for (int i = 0; i < 4; i++) v[i] = qpos[m.jnt_qposadr[id] + i];
    normalize4(v);
    dim = 4;
  } else if (t == SENS_FRAMEPOS) {  // sensor.py:282-338
    float p[3], R[9];
    obj_frame(m, wid, F, ot, id, p, R);
    if (rid == -1) {
      for (int i = 0; i < 3; i++) v[i] = p[i];
    } else {
      // reference branch order: the XBODY test reads objtype (sensor.py:323-326)
      int rt2 = rt == OBJ_BODY ? OBJ_BODY : (ot == OBJ_XBODY ? OBJ_XBODY : ((rt == OBJ_GEOM || rt == OBJ_SITE || rt == OBJ_CAMERA) ? rt : OBJ_UNKNOWN));
      float pr[3], Rr[9], dif[3];
      obj_frame(m, wid, F, rt2, rid, pr, Rr);
      for (int i = 0; i < 3; i++) dif[i] = p[i] - pr[i];
      mat_t_vec(v, Rr, dif);
    }
  } else if (t == SENS_FRAMEXAXIS || t == SENS_FRAMEYAXIS || t == SENS_FRAMEZAXIS) {  // sensor.py:341-391
    const int ax = t - SENS_FRAMEXAXIS;
    float p[3], R[9];
    obj_frame(m, wid, F, ot, id, p, R);
    float a[3] = {R[ax], R[3 + ax], R[6 + ax]};
    if (rid == -1) {
      for (int i = 0; i < 3; i++) v[i] = a[i];
    } else {
      float pr[3], Rr[9];
      obj_frame(m, wid, F, rt, rid, pr, Rr);
      mat_t_vec(v, Rr, a);
    }
  } else if (t == SENS_FRAMEQUAT) {  // sensor.py:394-446
    float q[4];
    frame_quat(m, wid, F, ot, id, q);
    if (rid == -1) {
      for (int i = 0; i < 4; i++) v[i] = q[i];
    } else {
      float qr[4], qi[4];
      frame_quat(m, wid, F, rt, rid, qr);
      qi[0] = qr[0]; qi[1] = -qr[1]; qi[2] = -qr[2]; qi[3] = -qr[3];
      mul_quat(v, qi, q);
    }
    dim = 4;
  } else if (t == SENS_CAMPROJECTION) {  // sensor.py:128-190: pixel coordinates of site `id` in camera `rid`
    float sp[3], sR[9], cp[3], cR[9], dif[3], pc[3];
    site_pose(m, wid, F, id, sp, sR);
    obj_frame(m, wid, F, OBJ_CAMERA, rid, cp, cR);
    for (int i = 0; i < 3; i++) dif[i] = sp[i] - cp[i];
    mat_t_vec(pc, cR, dif);  // rotation @ translation @ [x; 1]: the point in the camera frame
    const int rx = m.cam_resolution[2 * rid], ry = m.cam_resolution[2 * rid + 1];
    const float* ss = MR(cam_sensorsize) + 2 * rid;
    const float* in = MR(cam_intrinsic) + 4 * rid;
    float fx, fy;
    if (ss[0] != 0.0f && ss[1] != 0.0f) {
      fx = in[0] / (ss[0] + MJW_MINVAL) * (float)rx;
      fy = in[1] / (ss[1] + MJW_MINVAL) * (float)ry;
    } else {
      fx = fy = 0.5f / tanf(MR(cam_fovy)[rid] * (3.14159265358979f / 360.0f)) * (float)ry;
    }
    // image @ focal: (-fx x + rx/2 z, fy y + ry/2 z, z), divided by z clamped away from 0
    const float u = -fx * pc[0] + 0.5f * (float)rx * pc[2], w = fy * pc[1] + 0.5f * (float)ry * pc[2];
    float den = pc[2];
    if (fabsf(den) < MJW_MINVAL) den = clampf(den, -MJW_MINVAL, MJW_MINVAL);
    v[0] = u / den; v[1] = w / den; dim = 2;
  } else if (t == SENS_SUBTREECOM) {
    for (int i = 0; i < 3; i++) v[i] = F.subtree_com[3 * id + i];
  } else if (t == SENS_CLOCK) {
    v[0] = time; dim = 1;
  } else if (t == SENS_TENDONPOS) {  // sensor.py:222-224
    v[0] = d.ten_length[(long)wid * m.ntendon + id]; dim = 1;
  } else if (t == SENS_TENDONVEL) {  // sensor.py:957-959
    v[0] = d.ten_velocity[(long)wid * m.ntendon + id]; dim = 1;
  } else if (t == SENS_JOINTLIMITPOS || t == SENS_TENDONLIMITPOS || t == SENS_JOINTLIMITVEL || t == SENS_TENDONLIMITVEL) {
    const int r = limit_row(d, wid, id);  // sensor.py:243-278, 972-1007 (no row: the zeroed sensordata)
    const long e = (long)wid * d.njmax + r;
    const bool pos = t == SENS_JOINTLIMITPOS || t == SENS_TENDONLIMITPOS;
    v[0] = r < 0 ? 0.0f : (pos ? d.efc_pos[e] - d.efc_margin[e] : d.efc_vel[e]);
    dim = 1;
  } else if (t == SENS_SUBTREELINVEL || t == SENS_SUBTREEANGMOM) {  // sensor.py:1240-1248 (subtree_vel ran first)
    const float* src = (t == SENS_SUBTREELINVEL ? d.subtree_linvel : d.subtree_angmom) + ((long)wid * m.nbody + id) * 3;
    for (int i = 0; i < 3; i++) v[i] = src[i];
  } else if (COLL && (t == SENS_GEOMDIST || t == SENS_GEOMNORMAL || t == SENS_GEOMFROMTO)) {
    collision_sensor(m, d, wid, F, s);
    return;
  } else if (t == SENS_INSIDESITE) {  // sensor.py:681-697
    float p[3], R[9], sp[3], sR[9];
    obj_frame(m, wid, F, ot, id, p, R);
    site_pose(m, wid, F, rid, sp, sR);
    v[0] = inside_geom(sp, sR, MR(site_size) + 3 * rid, m.site_type[rid], p) ? 1.0f : 0.0f;
    dim = 1;
  } else if (t == SENS_E_POTENTIAL) {  // sensor.py:698-700
    v[0] = energy_potential(m, d, wid, qpos, F.xipos); dim = 1;
  } else if (t == SENS_E_KINETIC) {  // sensor.py:701-703
    v[0] = energy_kinetic(m, d, wid, qvel); dim = 1;
  } else if (t == SENS_GYRO || t == SENS_VELOCIMETER) {  // sensor.py:909-949
    float p[3], R[9];
    site_pose(m, wid, F, id, p, R);
    const int b = m.site_bodyid[id];
    const float* cv = F.cvel + 6 * b;
    if (t == SENS_GYRO) {
      mat_t_vec(v, R, cv);
    } else {
      const float* com = F.subtree_com + 3 * m.body_rootid[b];
      float dif[3], c[3], lin[3];
      for (int i = 0; i < 3; i++) dif[i] = p[i] - com[i];
      cross3(c, dif, cv);
      for (int i = 0; i < 3; i++) lin[i] = cv[3 + i] - c[i];
      mat_t_vec(v, R, lin);
    }
  } else if (t == SENS_JOINTVEL) {
    v[0] = qvel[m.jnt_dofadr[id]]; dim = 1;
  } else if (t == SENS_ACTUATORVEL) {
    v[0] = act_vel[id]; dim = 1;
  } else if (t == SENS_BALLANGVEL) {
    for (int i = 0; i < 3; i++) v[i] = qvel[m.jnt_dofadr[id] + i];
  } else if (t == SENS_FRAMELINVEL) {  // sensor.py:1053-1156
    float p[3], R[9], pr[3], Rr[9], off[3], offr[3], c[3], xl[3];
    obj_frame(m, wid, F, ot, id, p, R);
    obj_frame(m, wid, F, rt, rid, pr, Rr);
    const float* cv = cvel_offset(m, wid, F, ot, id, off);
    const float* cvr = cvel_offset(m, wid, F, rt, rid, offr);
    cross3(c, off, cv);
    for (int i = 0; i < 3; i++) xl[i] = cv[3 + i] - c[i];
    if (rid > -1) {
      float cr[3], rvec[3], rc[3], rel[3];
      cross3(cr, offr, cvr);
      for (int i = 0; i < 3; i++) rvec[i] = p[i] - pr[i];
      cross3(rc, rvec, cvr);
      for (int i = 0; i < 3; i++) rel[i] = xl[i] - (cvr[3 + i] - cr[i]) + rc[i];
      mat_t_vec(v, Rr, rel);
    } else {
      for (int i = 0; i < 3; i++) v[i] = xl[i];
    }
  } else if (t == SENS_FRAMEANGVEL) {  // sensor.py:1159-1238
    float off[3];
    const float* cv = cvel_offset(m, wid, F, ot, id, off);
    if (rid > -1) {
      float pr[3], Rr[9];
      obj_frame(m, wid, F, rt, rid, pr, Rr);
      const float* cvr = cvel_offset(m, wid, F, rt, rid, off);
      float dw[3] = {cv[0] - cvr[0], cv[1] - cvr[1], cv[2] - cvr[2]};
      mat_t_vec(v, Rr, dw);
    } else {
      for (int i = 0; i < 3; i++) v[i] = cv[i];
    }
  } else {
    return;
  }
  sensor_write(m, d, wid, s, v, dim);
}

}  // namespace mjw
